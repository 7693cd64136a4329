// EquivariantScalar head (reference models/output_modules.py:80-115, blocks models/utils.py:456-522) with
// its per-atom Jacobian, on the bf16 MFMA at fp32 accuracy over 16-atom tiles (the force pass: y and
// J = d y / d (x, vec); eq_head.hip's k_eq_head computes the same per atom with VALU row products).
//
// Why: k_eq_head is a chain of ~20 dependent row products per atom tile, each re-reading its weights from
// L2 for 1-2 atoms (45 us at C2's 576 atoms, 1.3 ms at C5's 50k: latency-bound, ~4 % of the VALU peak).
// Here a workgroup takes 16 atoms and each product phase is a small GEMM: rows = atoms (x 3 Cartesian
// axes for the vector products), columns = output channels, run as v_mfma_f32_16x16x32_bf16 on the exact
// three-piece split of both operands (xsplit.h: the weights pre-split once per weight version,
// tmdnet_proj_split_f32; the activations split from LDS per k-step); everything between the phases
// (norms, SiLU, gates) is elementwise over LDS.
//
// Phases (H = 128, O = Q = 64; vector rows ordered axis-major, row a*16 + t):
//   P1 [vb | v2] = vec [W1; W2]^T            48 x 192 x 128     E1 vec1 = |vb| over the axes
//   P2 u = [x | vec1] U1^T + b1               16 x 128 x 256     E2 s = SiLU(u)
//   P3 o = s U2^T + b2                        16 x 128 x 128     E3 x1 = SiLU(o[:O]), v1 = o[O:] v2
//   P4 vb2 = v1 V1^T                          48 x  64 x  64     E4 vec1' = |vb2|
//   P5 u2 = [x1 | vec1'] P1^T + b1'           16 x  64 x 128     E5 y = p2w[0] . SiLU(u2) + p2b[0];
//                                                                   g_u2 = seed p2w[0] SiLU'(u2)
//   B1 g_h2 = g_u2 P1                         16 x 128 x  64     E6 g_vb2 = g_vec1' / |vb2| vb2
//   B2 g_v1 = g_vb2 V1                        48 x  64 x  64     E7 g_o = [g_x1 SiLU'(xo) | sum_a g_v1 v2],
//                                                                   g_v2 = g_v1 vo
//   B3 g_s = g_o U2                           16 x 128 x 128     E8 g_u = g_s SiLU'(u)
//   B4 [J_x | g_vec1] = g_u U1                16 x 256 x 128     E9 g_vb = g_vec1 / |vb| vb
//   B5 J_vec = [g_vb | g_v2] [W1; W2]         48 x 128 x 192
// (a norm's gradient is 0 where the norm is 0, as the VALU kernel and torch.norm's backward).
// LDS: 116 KB per workgroup (buffers of dead forward values hold the backward's), one workgroup of 8
// waves per CU.
#include "common.h"
#include "tmdnet.h"
#include "xsplit.h"

namespace tmd {
namespace headx {

using xs::bf8;
using f4 = xs::f4v;
constexpr int kH = 128, kO = 64, kT = 16, kNW = 8;

// LDS buffers (floats; row pitches padded by 4 against bank conflicts of the 16 rows a fragment reads)
constexpr int PV = kH + 4;          // 48 rows: vec (P1's input); then u | s | o (16 rows each)
constexpr int PVB = kH + kO + 4;     // 48 rows: [vb | v2] -> [g_vb | g_v2]
constexpr int PHH = 2 * kH + 4;     // 16 rows: [x | vec1] -> [. | g_vec1]
constexpr int P64 = kO + 4;         // 48 rows: v1 -> g_v1; vb2 -> g_vb2; 16 rows: u2 -> g_u2
constexpr int PH2 = 2 * kO + 4;     // 16 rows: [x1 | vec1'] -> g_h2
constexpr int OFF_V = 0, OFF_U = 0, OFF_S = 16 * PV, OFF_O = 32 * PV;
constexpr int OFF_VB = 48 * PV;
constexpr int OFF_HH = OFF_VB + 48 * PVB;
constexpr int OFF_V1 = OFF_HH + 16 * PHH;
constexpr int OFF_VB2 = OFF_V1 + 48 * P64;
constexpr int OFF_H2 = OFF_VB2 + 48 * P64;
constexpr int OFF_U2 = OFF_H2 + 16 * PH2;
constexpr int LDS_FLOATS = OFF_U2 + 16 * P64;

struct Args {
  int n;
  const float* x;
  const float* vec;
  // pre-split weights [3][N][K] bf16 pieces (tmdnet_proj_split_f32 layout)
  const unsigned short *w12, *u1, *u2, *v1, *p1;     // forward: [192][128] [128][256] [128][128] [64][64] [64][128]
  const unsigned short *p1t, *v1t, *u2t, *u1t, *w12t;  // backward: [128][64] [64][64] [128][128] [256][128] [128][192]
  const float *u1b, *u2b, *p1b, *p2w, *p2b;
  float* y;
  float* jx;
  float* jv;
  const float* gy;
};

__device__ __forceinline__ float sigm(float u) { return __builtin_amdgcn_rcpf(1.f + __expf(-u)); }

// A wave's weight fragments for one 16-column output tile: all K / 32 k-steps x 3 pieces, loaded at once
// (one L2 round trip per tile) and -- for a phase's first tile -- issued BEFORE the barrier and the
// elementwise pass that precede the phase (the weights do not depend on the data), so the phase starts
// with them in registers.
template <int KS> struct WFrag {
  bf8 w[KS][3];
};
template <int K, int NB>
__device__ __forceinline__ void wload(WFrag<K / 32>& f, const unsigned short* B, int b_row0, int ntile) {
  constexpr size_t PS = (size_t)NB * K;
  const int lane = threadIdx.x & 63;
  const unsigned short* br = B + (size_t)(b_row0 + 16 * ntile + (lane & 15)) * K + 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < K / 32; ++ks)
#pragma unroll
    for (int p = 0; p < 3; ++p) f.w[ks][p] = *reinterpret_cast<const bf8*>(br + p * PS + 32 * ks);
}
// the first tile's fragments of a phase, prefetched by its wave (no-op for waves without a tile)
template <int N, int K, int NB>
__device__ __forceinline__ WFrag<K / 32> wpre(const unsigned short* B, int b_row0) {
  WFrag<K / 32> f;
  const int wave = threadIdx.x >> 6;
  if (wave < N / 16) wload<K, NB>(f, B, b_row0, wave);
  return f;
}

// out[m][n] = sum_k A[m][k] B[n][k] (+ bias[n]) for m < M, n < N: A fp32 in LDS (pitch LDA), B the three
// bf16 pieces [3][NB][K] in global memory from row b_row0 (piece stride NB * K).  Wave w takes the
// 16-column tiles w, w + 8, ... and, per tile, every 16-row block (the weight fragments reused across
// them); the weight fragment is the MFMA's first operand, so a lane's accumulator holds 4 consecutive
// output columns of one row (16-byte stores).  DST 0: LDS (pitch ldo); 1: J_x rows (global, t < nt);
// 2: J_vec rows (row a*16 + t).  `pre`: the wave's first tile's fragments (wpre).
template <int M, int N, int K, int NB, int LDA, int DST>
__device__ __forceinline__ void mm(const float* A, const unsigned short* B, int b_row0, const float* bias, float* out,
                                   int ldo, int nt, const WFrag<K / 32>& pre) {
  constexpr int MT = M / 16, NTL = N / 16, KS = K / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = 8 * (lane >> 4);
  for (int nt_ = wave; nt_ < NTL; nt_ += kNW) {
    WFrag<KS> f;
    if (nt_ == wave) f = pre;
    else wload<K, NB>(f, B, b_row0, nt_);
    const int n0 = 16 * nt_ + 4 * (lane >> 4);
    const f4 bv = bias ? *reinterpret_cast<const f4*>(bias + n0) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const float* ar = A + (16 * mt + (lane & 15)) * LDA + kq;
      f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf8 a[3];
        xs::split8(*reinterpret_cast<const float4*>(ar + 32 * ks), *reinterpret_cast<const float4*>(ar + 32 * ks + 4),
                   a);
        acc = xs::mfma_x3(f.w[ks], a, acc);
      }
      acc += bv;
      const int m = 16 * mt + (lane & 15);
      if constexpr (DST == 0) {
        *reinterpret_cast<f4*>(out + m * ldo + n0) = acc;
      } else if constexpr (DST == 1) {
        if (m < nt) *reinterpret_cast<f4*>(out + (size_t)m * kH + n0) = acc;
      } else {
        const int a = m >> 4, t = m & 15;
        if (t < nt) *reinterpret_cast<f4*>(out + ((size_t)t * 3 + a) * kH + n0) = acc;
      }
    }
  }
}

__global__ __launch_bounds__(kNW * 64, 1) void k_head_x3(Args P) {
  __shared__ __attribute__((aligned(16))) float sm[LDS_FLOATS];
  const int n0 = blockIdx.x * kT, nt = min(kT, P.n - n0);
  const int tid = threadIdx.x, bs = kNW * 64;
  float* V = sm + OFF_V;
  float* U = sm + OFF_U;
  float* S = sm + OFF_S;
  float* O = sm + OFF_O;
  float* VB = sm + OFF_VB;
  float* HH = sm + OFF_HH;
  float* V1 = sm + OFF_V1;
  float* VB2 = sm + OFF_VB2;
  float* H2 = sm + OFF_H2;
  float* U2 = sm + OFF_U2;
  auto w_p1 = wpre<192, 128, 192>(P.w12, 0);
  // stage x -> HH[:, :H], vec -> V (row a*16 + t); absent atoms read as 0 (16-byte loads)
  for (int i = tid; i < kT * 4 * (kH / 4); i += bs) {
    const int t = i / (4 * (kH / 4)), r = (i / (kH / 4)) % 4, c = 4 * (i % (kH / 4));
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < nt)
      v = r == 0 ? *reinterpret_cast<const float4*>(P.x + (size_t)(n0 + t) * kH + c)
                 : *reinterpret_cast<const float4*>(P.vec + ((size_t)(n0 + t) * 3 + r - 1) * kH + c);
    if (r == 0) *reinterpret_cast<float4*>(HH + t * PHH + c) = v;
    else *reinterpret_cast<float4*>(V + ((r - 1) * 16 + t) * PV + c) = v;
  }
  __syncthreads();
  // ---------------- block 1
  mm<48, 192, 128, 192, PV, 0>(V, P.w12, 0, nullptr, VB, PVB, nt, w_p1);  // [vb | v2]
  auto w_p2 = wpre<128, 256, 128>(P.u1, 0);
  __syncthreads();
  for (int i = tid; i < kT * kH; i += bs) {
    const int t = i / kH, c = i % kH;
    const float a0 = VB[t * PVB + c], a1 = VB[(16 + t) * PVB + c], a2 = VB[(32 + t) * PVB + c];
    HH[t * PHH + kH + c] = sqrtf(a0 * a0 + a1 * a1 + a2 * a2);
  }
  __syncthreads();
  mm<16, 128, 256, 128, PHH, 0>(HH, P.u1, 0, P.u1b, U, PV, nt, w_p2);  // (U overwrites vec: dead after P1)
  auto w_p3 = wpre<128, 128, 128>(P.u2, 0);
  __syncthreads();
  for (int i = tid; i < kT * kH; i += bs) {
    const int t = i / kH, c = i % kH;
    const float u = U[t * PV + c];
    S[t * PV + c] = u * sigm(u);
  }
  __syncthreads();
  mm<16, 128, 128, 128, PV, 0>(S, P.u2, 0, P.u2b, O, PV, nt, w_p3);
  auto w_p4 = wpre<64, 64, 64>(P.v1, 0);
  __syncthreads();
  for (int i = tid; i < kT * kO; i += bs) {
    const int t = i / kO, c = i % kO;
    const float xo = O[t * PV + c], vo = O[t * PV + kO + c];
    H2[t * PH2 + c] = xo * sigm(xo);
#pragma unroll
    for (int a = 0; a < 3; ++a) V1[(a * 16 + t) * P64 + c] = vo * VB[(a * 16 + t) * PVB + kH + c];
  }
  __syncthreads();
  // ---------------- block 2
  mm<48, 64, 64, 64, P64, 0>(V1, P.v1, 0, nullptr, VB2, P64, nt, w_p4);
  auto w_p5 = wpre<64, 128, 64>(P.p1, 0);
  __syncthreads();
  for (int i = tid; i < kT * kO; i += bs) {
    const int t = i / kO, c = i % kO;
    const float a0 = VB2[t * P64 + c], a1 = VB2[(16 + t) * P64 + c], a2 = VB2[(32 + t) * P64 + c];
    H2[t * PH2 + kO + c] = sqrtf(a0 * a0 + a1 * a1 + a2 * a2);
  }
  __syncthreads();
  mm<16, 64, 128, 64, PH2, 0>(H2, P.p1, 0, P.p1b, U2, P64, nt, w_p5);
  auto w_b1 = wpre<128, 64, 128>(P.p1t, 0);
  __syncthreads();
  // y = p2w[0] . SiLU(u2) + p2b[0] (one wave per atom pair), and the reverse seed g_u2 in place of u2
  {
    const int lane = tid & 63, wave = tid >> 6;
    for (int t = wave; t < kT; t += kNW) {
      const float u = U2[t * P64 + lane], sg = sigm(u), w = P.p2w[lane];
      float part = w * u * sg;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
      const float seed = t < nt ? (P.gy ? P.gy[n0 + t] : 1.f) : 0.f;
      if (lane == 0 && t < nt && P.y) P.y[n0 + t] = part + P.p2b[0];
      U2[t * P64 + lane] = seed * w * sg * (1.f + u * (1.f - sg));
    }
  }
  __syncthreads();
  if (P.jx == nullptr) return;
  // ---------------- reverse: block 2
  mm<16, 128, 64, 128, P64, 0>(U2, P.p1t, 0, nullptr, H2, PH2, nt, w_b1);  // g_h2 = [g_x1 | g_vec1']
  auto w_b2 = wpre<64, 64, 64>(P.v1t, 0);
  __syncthreads();
  for (int i = tid; i < kT * kO; i += bs) {
    const int t = i / kO, c = i % kO;
    float b[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) b[a] = VB2[(a * 16 + t) * P64 + c];
    const float nrm = sqrtf(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
    const float sc = nrm > 0.f ? H2[t * PH2 + kO + c] / nrm : 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) VB2[(a * 16 + t) * P64 + c] = sc * b[a];  // g_vb2
  }
  __syncthreads();
  mm<48, 64, 64, 64, P64, 0>(VB2, P.v1t, 0, nullptr, V1, P64, nt, w_b2);  // g_v1 (vec'' has a zero cotangent)
  auto w_b3 = wpre<128, 128, 128>(P.u2t, 0);
  __syncthreads();
  // block 1 gate: g_xo = g_x1 SiLU'(xo), g_vo = sum_a g_v1 v2, g_v2 = g_v1 vo
  for (int i = tid; i < kT * kO; i += bs) {
    const int t = i / kO, c = i % kO;
    const float xo = O[t * PV + c], vo = O[t * PV + kO + c], sg = sigm(xo);
    float gvo = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float g = V1[(a * 16 + t) * P64 + c];
      float* v2 = VB + (a * 16 + t) * PVB + kH + c;
      gvo += g * *v2;
      *v2 = g * vo;  // g_v2
    }
    O[t * PV + c] = H2[t * PH2 + c] * sg * (1.f + xo * (1.f - sg));
    O[t * PV + kO + c] = gvo;
  }
  __syncthreads();
  mm<16, 128, 128, 128, PV, 0>(O, P.u2t, 0, nullptr, S, PV, nt, w_b3);  // g_s
  auto w_b4a = wpre<128, 128, 256>(P.u1t, 0);
  __syncthreads();
  for (int i = tid; i < kT * kH; i += bs) {
    const int t = i / kH, c = i % kH;
    const float u = U[t * PV + c], sg = sigm(u);
    S[t * PV + c] *= sg * (1.f + u * (1.f - sg));  // g_u
  }
  __syncthreads();
  // g_h = g_u U1: the x half is J_x (global), the vec1 half g_vec1 (LDS, over HH's vec1 columns)
  auto w_b4b = wpre<128, 128, 256>(P.u1t, 128);
  mm<16, 128, 128, 256, PV, 1>(S, P.u1t, 0, nullptr, P.jx + (size_t)n0 * kH, 0, nt, w_b4a);
  mm<16, 128, 128, 256, PV, 0>(S, P.u1t, 128, nullptr, HH + kH, PHH, nt, w_b4b);
  auto w_b5 = wpre<128, 192, 128>(P.w12t, 0);
  __syncthreads();
  for (int i = tid; i < kT * kH; i += bs) {
    const int t = i / kH, c = i % kH;
    float b[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) b[a] = VB[(a * 16 + t) * PVB + c];
    const float nrm = sqrtf(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
    const float sc = nrm > 0.f ? HH[t * PHH + kH + c] / nrm : 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) VB[(a * 16 + t) * PVB + c] = sc * b[a];  // g_vb
  }
  __syncthreads();
  mm<48, 128, 192, 128, PVB, 2>(VB, P.w12t, 0, nullptr, P.jv + (size_t)n0 * 3 * kH, 0, nt, w_b5);  // J_vec
}

// ---- the weights' three-piece splits, all ten matrices in ONE launch (inside a captured step it runs on
// every replay, so the pieces always match the current weights).  Entry j writes dst rows row0.. and
// columns col0.. of a [NB][KD] piece matrix: dst[row0 + n][col0 + k] = T ? src[k][n] : src[n][k].
struct SplitEntry {
  const float* src;
  int ld, T, N, K, KD, NB, row0, col0;
  unsigned short* dst;
};
constexpr int kSplitEntries = 12;
struct SplitTable {
  SplitEntry e[kSplitEntries];
  int start[kSplitEntries + 1];  // element prefix
};

__global__ __launch_bounds__(256) void k_split_all(SplitTable T) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= T.start[kSplitEntries]) return;
  int j = 0;
  while (i >= T.start[j + 1]) ++j;
  const SplitEntry& E = T.e[j];
  const int r = i - T.start[j], n = r / E.K, k = r % E.K;
  const float x = E.T ? E.src[(size_t)k * E.ld + n] : E.src[(size_t)n * E.ld + k];
  unsigned h, m, l;
  xs::split3(x, h, m, l);
  const size_t o = (size_t)(E.row0 + n) * E.KD + E.col0 + k, ps = (size_t)E.NB * E.KD;
  E.dst[o] = (unsigned short)(h >> 16);
  E.dst[ps + o] = (unsigned short)(m >> 16);
  E.dst[2 * ps + o] = (unsigned short)(l >> 16);
}

}  // namespace headx
}  // namespace tmd

using namespace tmd;

// element counts of the ten piece matrices (tmdnet_eq_head_x3_f32's `pieces` order), each [3][N][K]
static const int kPieceNK[10][2] = {{192, 128}, {128, 256}, {128, 128}, {64, 64}, {64, 128},
                                    {128, 64},  {64, 64},   {128, 128}, {256, 128}, {128, 192}};

extern "C" size_t tmdnet_eq_head_x3_pieces_bytes(int hidden) {
  if (hidden != headx::kH) return 0;
  size_t t = 0;
  for (auto& nk : kPieceNK) t += (size_t)3 * nk[0] * nk[1] * sizeof(unsigned short);
  return t;
}

extern "C" int tmdnet_eq_head_x3_split_f32(int hidden, const void* const* weights, void* pieces_buf, void* stream) {
  if (!weights || !pieces_buf) return kBadArgument;
  if (hidden != headx::kH) return kUnsupported;
  if (((uintptr_t)pieces_buf) & 15) return kUnsupported;
  const float* const* w = (const float* const*)weights;  // tmdnet_eq_head_fwd's 12-weight order
  const float *W1 = w[0], *W2 = w[1], *U1 = w[2], *U2 = w[4], *V1 = w[6], *P1 = w[8];
  unsigned short* pc[10];
  unsigned short* p = (unsigned short*)pieces_buf;
  for (int i = 0; i < 10; ++i) {
    pc[i] = p;
    p += (size_t)3 * kPieceNK[i][0] * kPieceNK[i][1];
  }
  constexpr int H = headx::kH, O = headx::kO;
  headx::SplitTable T{};
  //            src ld  T  N    K    KD     NB     row0 col0 dst
  T.e[0] = {W1, H, 0, H, H, H, H + O, 0, 0, pc[0]};              // [W1; W2]
  T.e[1] = {W2, H, 0, O, H, H, H + O, H, 0, pc[0]};
  T.e[2] = {U1, 2 * H, 0, H, 2 * H, 2 * H, H, 0, 0, pc[1]};      // U1
  T.e[3] = {U2, H, 0, H, H, H, H, 0, 0, pc[2]};                  // U2
  T.e[4] = {V1, O, 0, O, O, O, O, 0, 0, pc[3]};                  // V1
  T.e[5] = {P1, 2 * O, 0, O, 2 * O, 2 * O, O, 0, 0, pc[4]};      // P1
  T.e[6] = {P1, 2 * O, 1, 2 * O, O, O, 2 * O, 0, 0, pc[5]};      // P1^T
  T.e[7] = {V1, O, 1, O, O, O, O, 0, 0, pc[6]};                  // V1^T
  T.e[8] = {U2, H, 1, H, H, H, H, 0, 0, pc[7]};                  // U2^T
  T.e[9] = {U1, 2 * H, 1, 2 * H, H, H, 2 * H, 0, 0, pc[8]};      // U1^T
  T.e[10] = {W1, H, 1, H, H, H + O, H, 0, 0, pc[9]};             // [W1; W2]^T = [W1^T | W2^T]
  T.e[11] = {W2, H, 1, H, O, H + O, H, 0, H, pc[9]};
  T.start[0] = 0;
  for (int j = 0; j < headx::kSplitEntries; ++j) {
    if (!T.e[j].src) return kBadArgument;
    T.start[j + 1] = T.start[j] + T.e[j].N * T.e[j].K;
  }
  const int total = T.start[headx::kSplitEntries];
  hipLaunchKernelGGL(headx::k_split_all, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, T);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_eq_head_x3_f32(int n_atoms, int hidden, const void* x, const void* vec,
                                     const void* const* pieces, const void* const* vectors, void* y, void* jac_x,
                                     void* jac_vec, const void* grad_y, void* stream) {
  if (n_atoms < 0 || !x || !vec || !pieces || !vectors) return kBadArgument;
  if (hidden != headx::kH) return kUnsupported;
  if ((jac_x == nullptr) != (jac_vec == nullptr)) return kBadArgument;
  if (n_atoms == 0) return kOk;
  for (int i = 0; i < 10; ++i)
    if (!pieces[i] || (((uintptr_t)pieces[i]) & 15)) return kBadArgument;
  for (int i = 0; i < 5; ++i)
    if (!vectors[i]) return kBadArgument;
  if ((((uintptr_t)x) | ((uintptr_t)vec) | ((uintptr_t)jac_x) | ((uintptr_t)jac_vec) | ((uintptr_t)vectors[0]) |
       ((uintptr_t)vectors[1]) | ((uintptr_t)vectors[2])) & 15)
    return kUnsupported;
  headx::Args P{};
  P.n = n_atoms;
  P.x = (const float*)x;
  P.vec = (const float*)vec;
  const unsigned short* const* pc = (const unsigned short* const*)pieces;
  P.w12 = pc[0]; P.u1 = pc[1]; P.u2 = pc[2]; P.v1 = pc[3]; P.p1 = pc[4];
  P.p1t = pc[5]; P.v1t = pc[6]; P.u2t = pc[7]; P.u1t = pc[8]; P.w12t = pc[9];
  const float* const* vv = (const float* const*)vectors;
  P.u1b = vv[0]; P.u2b = vv[1]; P.p1b = vv[2]; P.p2w = vv[3]; P.p2b = vv[4];
  P.y = (float*)y;
  P.jx = (float*)jac_x;
  P.jv = (float*)jac_vec;
  P.gy = (const float*)grad_y;
  const dim3 g((n_atoms + headx::kT - 1) / headx::kT), b(headx::kNW * 64);
  hipLaunchKernelGGL(headx::k_head_x3, g, b, 0, (hipStream_t)stream, P);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
