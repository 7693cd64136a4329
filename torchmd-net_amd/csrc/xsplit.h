// Exact three-piece bf16 split of fp32 operands for the bf16 MFMA at fp32 accuracy (the scheme of
// gemm.hip's k_proj_x3 / k_gemm_x3): x = h + m + l with h = bf16(x), m = bf16(x - h), l = bf16(x - h - m)
// (truncations: every difference is exact), and a product sum over the six piece pairs with i + j <= 2,
// small terms first -- the dropped terms are ~2^-24 relative.
#pragma once

namespace tmd {
namespace xs {

using bf8 = __bf16 __attribute__((ext_vector_type(8)));
using f4v = float __attribute__((ext_vector_type(4)));
using u4v = unsigned __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
  h = __float_as_uint(x) & 0xffff0000u;
  const float r1 = x - __uint_as_float(h);
  m = __float_as_uint(r1) & 0xffff0000u;
  l = __float_as_uint(r1 - __uint_as_float(m)) & 0xffff0000u;
}

// 8 consecutive fp32 -> the three bf16 fragments of one MFMA operand
__device__ __forceinline__ void split8(const float4& a, const float4& b, bf8 (&f)[3]) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  unsigned h[8], m[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) split3(x[j], h[j], m[j], l[j]);
  u4v H, M, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // element 2p in the low half of register p
    H[p] = (h[2 * p] >> 16) | h[2 * p + 1];
    M[p] = (m[2 * p] >> 16) | m[2 * p + 1];
    L[p] = (l[2 * p] >> 16) | l[2 * p + 1];
  }
  f[0] = __builtin_bit_cast(bf8, H);
  f[1] = __builtin_bit_cast(bf8, M);
  f[2] = __builtin_bit_cast(bf8, L);
}

// acc += sum over the piece pairs (w_i, a_j), i + j <= 2, small first
__device__ __forceinline__ f4v mfma_x3(const bf8 (&w)[3], const bf8 (&a)[3], f4v acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], a[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], a[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], a[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], a[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], a[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], a[0], acc, 0, 0, 0);
  return acc;
}

}  // namespace xs
}  // namespace tmd
