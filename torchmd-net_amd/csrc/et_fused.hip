// Equivariant-Transformer message with the dk/dv projection FUSED into the edge kernels ("FEP"): the
// forward and the force pass's backward ("dr mode") of the ET message, with the projection of the RBF
// features formed on the fp16 MFMA inside the edge kernel instead of being written to and re-read from
// HBM as pair rows.
//
// Reference: EquivariantMultiHeadAttention dk_proj / dv_proj (models/torchmd_et.py:282-291),
// message / aggregate (:314-347); the RBF it projects, ExpNormalSmearing / GaussianSmearing and the
// CosineCutoff (models/utils.py:272-390); the backward is the autograd of those lines through
// f = rbf(r) (the force pass, models/model.py:286-298).
//
// Why: the unfused path writes the projection rows of every edge pair (2 KB per row at H = 128, 2.8 GB
// per layer at C5) and the message kernels read them back once per DIRECTION (the two edges of a pair
// sit in different destination rows, far apart in time): 2.4x the distinct bytes of the forward, and the
// force pass also streams d(dk,dv)/dr rows the same way.  Here the projection
// never leaves the chip.  What remains in memory is the edge stream (src, r, C, unit vector: 24 B per
// edge) and the node-row gathers (L2 / Infinity-Cache resident for spatially ordered atoms).
//
// Accuracy: fp32-GEMM level without the fp32 MFMA (1/16 of the fp16 rate).  Both operands are split
// into two fp16 pieces, x = x0 + x1 (x0 = fp16(x), x1 = fp16(x - x0), exact difference), after an exact
// power-of-two scaling (the weight per output row to max |w| < 2^14, the RBF values -- all in [0, 1] --
// by 2^14, their r-derivative per EDGE to max < 2^14); the three products x0 y0 + x0 y1 + x1 y0 are
// exact in the fp32 accumulator and the dropped x1 y1 and the split residuals are ~2^-22 relative --
// below fp32 GEMM rounding at K = 64.
//
// Layout (round 4): the MFMA v_mfma_f32_16x16x32_f16 takes the WEIGHT block as its A operand (16 output
// channels x 32 k, the LDS image) and the RBF tile as B (32 k x 16 edges), so its accumulator holds, per
// lane, FOUR CONSECUTIVE CHANNELS (4 g + i, g = lane >> 4) of ONE EDGE (c = lane & 15).  Every node-row
// gather of an edge is then one 16-byte load per lane (k, v, vec: channels 16 h + 4 g .. + 3 of the
// lane's own source), the per-edge scalars are the lane's own (no cross-lane hand-out), and the head sums
// (16 channels = 4 lanes x 4 values) are an in-lane sum plus two v_permlane{32,16}_swap.  (The round-3
// kernel had the operands the other way round: four edges x one channel per lane, 4-byte gathers --
// issue-bound at 72 % VALU / 15 % of the fp16 MFMA.)  A lane accumulates its edge slot's messages over
// the row's 16-edge tiles in registers; the 16 slots are summed once per node (DPP row sums).
//
// Work decomposition: one workgroup per CU (the 128 KB weight image fills its LDS), waves taking work
// items (node, head slice) from an LDS counter over the workgroup's contiguous node range (XCD-contiguous
// block remap).  Forward: HPW heads per item; backward: a DESTINATION pass (all 8 heads per item: the
// per-edge sums g_cut, g_unit, g_r over every channel stay in one wave; d pre / d r = W f'(r) formed on
// the MFMA beside the projection) and a SOURCE pass over the same rows read as reversed edges (gk, gv,
// gvec_in; no per-edge outputs, so HPW heads per item).  Deterministic, no atomics on outputs.
#include <cstdlib>

#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace fep {

using h8 = _Float16 __attribute__((ext_vector_type(8)));
using f4 = float __attribute__((ext_vector_type(4)));
using u4 = unsigned __attribute__((ext_vector_type(4)));

constexpr float kFScale = 16384.f;  // 2^14: the RBF values (in [0, 1]) before their fp16 split
constexpr int kH = 128;             // channels: the LDS image holds 4H weight rows
constexpr int kD = 4 * kH;
constexpr int kHeads = 8;           // d = 16: one MFMA row block per head and projection part

// 16-byte chunk swizzle of the weight image (rows of R fp16; lane l reads row (l & 15), chunk
// (l >> 4) + 4 ks): conflict-free ds_read_b128 for every lane group (checked exhaustively)
template <int KS> __host__ __device__ __forceinline__ int swz(int row, int ch) {
  return ch ^ ((KS == 2 ? row : (row >> 1)) & (4 * KS - 1));
}

// Weight rows (planar [dk | dv_x | dv_1 | dv_2] order, fp32 [D][R]) -> the LDS image: two fp16 pieces
// [2][D][R] (swizzled chunks) of w * 2^s_row, and per row 2^-s_row / 2^14 (the accumulator scale)
// and the bias.  One thread per row.
template <int KS>
__global__ void k_split(int D, const float* __restrict__ W, int ldw, const float* __restrict__ b,
                        _Float16* __restrict__ img, float* __restrict__ wsc, float* __restrict__ bias) {
  constexpr int R = 32 * KS;
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= D) return;
  const float* w = W + (size_t)row * ldw;
  float m = 0.f;
  for (int k = 0; k < R; ++k) m = fmaxf(m, fabsf(w[k]));
  int ex = 0;
  if (m > 0.f) frexpf(m, &ex);  // m < 2^ex
  // (capped at 2^30: the t-domain forward divides the bias by the accumulator scale, which must stay
  // finite; a row below 2^-16 carries a negligible share of its pre-activation anyway)
  const int s = m > 0.f ? min(14 - ex, 30) : 0;
  for (int k = 0; k < R; ++k) {
    const float x = ldexpf(w[k], s);
    const _Float16 h = (_Float16)x;
    const _Float16 l = (_Float16)(x - (float)h);
    const size_t o = (size_t)row * R + swz<KS>(row, k >> 3) * 8 + (k & 7);
    img[o] = h;
    img[(size_t)D * R + o] = l;
  }
  wsc[row] = ldexpf(1.f, -s) / kFScale;
  bias[row] = b ? b[row] : 0.f;
}

// ------------------------------------------------------------------ lane-level helpers
// sum over the 16 lanes of a DPP row (bit-identical in every lane: each stage adds a commutative pair)
template <int CTRL> __device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float x) {
  x += dpp<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp<0x141>(x);  // row_half_mirror
  x += dpp<0x140>(x);  // row_mirror
  return x;
}
// sum / max over the four lane groups g (lanes c, c + 16, c + 32, c + 48) -- gfx950's lane-half and
// row-pair swaps; every lane gets the same bits (both halves add the same two values in the same order)
__device__ __forceinline__ float gsum(float x) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float gmax(float x) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// Node-row gathers through buffer resources: per edge one 32-bit byte offset (row start + the lane's
// channel group), the head's byte offset in an SGPR (soffset), the part's as the immediate.  An edge past
// the row (or vec absent: a zero-size resource) reads 0.
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// a byte offset past every resource's range (buffer loads return 0), with room for the head / part
// offsets added to it (< 4 KB)
constexpr int kOOB = 0x7FFF0000;
template <int IMM>
__device__ __forceinline__ f4 bld4(rsrc_t r, int voff, int soff) {
  static_assert(IMM >= 0 && IMM < 4096, "buffer immediate offset");
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + IMM, soff, 0));
}

template <int I> struct IC { static constexpr int value = I; };
template <int N, int I = 0, typename F> __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<N, I + 1>(f);
  }
}

// The RBF tile as the MFMA's B operand, PRECOMPUTED once per projection row (pair row) and evaluation
// (every layer shares it): row p of the fragment buffer holds [B0 | B1 | D0 | D1], R fp16 each -- the
// two pieces of f(r_p) * 2^14 and of f'(r_p) * 2^sd_p with the row's own power-of-two scale
// (|f'| is not bounded by 1; dscale[p] = 2^(14 - sd_p) turns the weight's accumulator scale, which
// assumes the 2^14 of f, into the derivative's).  A lane of the edge kernels loads its edge's
// 8-value chunk k = 32 ks + 8 g .. + 7 of each piece: one 16-byte load.  The edge-geometry kernel's
// formulas (edge_geom.hip basis()).
template <int KS>
__global__ __launch_bounds__(256) void k_frags(long long rows, const float* __restrict__ r,
                                               const float* __restrict__ mu, const float* __restrict__ beta,
                                               int rbf, float cl, float cu, float alpha, _Float16* __restrict__ fr,
                                               float* __restrict__ dscale) {
  // R lanes per row (lane = k): coalesced 2-byte stores, the derivative's max a lane-group reduction
  constexpr int R = 32 * KS;
  constexpr float kPi = 3.14159265358979323846f;
  const long long p = (long long)blockIdx.x * (256 / R) + threadIdx.x / R;
  const int k = threadIdx.x % R;
  const bool live = p < rows;
  const float rf = live ? r[p] : 0.f;
  const bool in = rf < cu;
  const float cut0 = in ? 0.5f * (cosf(rf * kPi / cu) + 1.f) : 0.f;
  const float dcut0 = in ? -0.5f * sinf(rf * kPi / cu) * kPi / cu : 0.f;
  const float ue = expf(alpha * (cl - rf));
  float f, d;
  if (rbf == TMDNET_RBF_EXPNORM) {
    const float z = ue - mu[k], b = beta[k];
    const float gg = expf(-b * z * z);
    f = cut0 * gg;
    d = dcut0 * gg + cut0 * gg * (2.f * b * z * alpha * ue);  // d/dr: du = -alpha ue
  } else {
    const float z = rf - mu[k], co = beta[0];
    f = expf(co * z * z);
    d = f * 2.f * co * z;
  }
  float mx = fabsf(d);
#pragma unroll
  for (int o = R / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (!live) return;
  int ex = 0;
  if (mx > 0.f) frexpf(mx, &ex);
  const int sd = mx > 0.f ? 14 - ex : 0;
  if (k == 0) dscale[p] = ldexpf(1.f, 14 - sd);
  _Float16* o = fr + p * 4 * R;
  const float x = f * kFScale;
  const _Float16 hi = (_Float16)x;
  o[k] = hi;
  o[R + k] = (_Float16)(x - (float)hi);
  const float y = ldexpf(d, sd);
  const _Float16 yh = (_Float16)y;
  o[2 * R + k] = yh;
  o[3 * R + k] = (_Float16)(y - (float)yh);
}

// the lane's B fragments (piece 0 / 1 at byte offsets 0 / 2R of section `sec`) of its edge's frag row
template <int KS>
__device__ __forceinline__ void load_frags(rsrc_t Rf, int fo, int g, int sec, h8 (&b0)[KS], h8 (&b1)[KS]) {
  constexpr int R = 32 * KS;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int o = fo + sec * 4 * R + (32 * ks + 8 * g) * 2;
    b0[ks] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(Rf, o, 0, 0));
    b1[ks] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(Rf, o + 2 * R, 0, 0));
  }
}

// Byte offset in the weight image of the lane's A fragment for k-step ks of block 0, piece 0: lane l
// reads row (l & 15) + 16 blk, chunk swz(row, (l >> 4) + 4 ks) -- the swizzle depends on row & 7 (KS = 2)
// or (row >> 1) & 3 (KS = 1) only, so block and piece add CONSTANT offsets (ds_read immediates).
template <int KS>
__device__ __forceinline__ int wfrag_base(int lane, int ks) {
  constexpr int R = 32 * KS;
  const int row = lane & 15;
  return (row * R + swz<KS>(row, (lane >> 4) + 4 * ks) * 8) * (int)sizeof(_Float16);
}

// One 16-channel block of the tile's projection: acc[i] = sum_k W[16 blk + 4 g + i][k] B[k][c] -- the
// weight block is the A operand, the RBF (or its derivative) tile B.  Pieces: small terms first.
template <int KS, int D = kD>
__device__ __forceinline__ f4 block_acc(const char* wl, const int (&wb)[KS], int blk, const h8 (&b0)[KS],
                                        const h8 (&b1)[KS]) {
  constexpr int R = 32 * KS, PB = D * R * (int)sizeof(_Float16);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const char* f0 = wl + wb[ks] + blk * 16 * R * (int)sizeof(_Float16);
    const h8 w0 = *reinterpret_cast<const h8*>(f0);
    const h8 w1 = *reinterpret_cast<const h8*>(f0 + PB);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b1[ks], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, b0[ks], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b0[ks], acc, 0, 0, 0);
  }
  return acc;
}
// pre-activation: acc * scale + bias of the lane's four channels
template <int KS, int D = kD>
__device__ __forceinline__ f4 block_pre(const char* wl, const int (&wb)[KS], const float* sc, const float* sb,
                                        int blk, const h8 (&b0)[KS], const h8 (&b1)[KS], int g) {
  const f4 acc = block_acc<KS, D>(wl, wb, blk, b0, b1);
  const f4 s = *reinterpret_cast<const f4*>(sc + 16 * blk + 4 * g);
  const f4 b = *reinterpret_cast<const f4*>(sb + 16 * blk + 4 * g);
  return acc * s + b;
}
// ---- "t-domain" SiLU (forward and source pass).  With t = -log2(e) pre, SiLU(pre) = pre / (1 + 2^t) =
// -ln2 * u(t), u(t) = t / (1 + 2^t): the exponent is v_exp_f32 of t itself (no multiply), and the bias add
// and the -log2(e) factor fold into the MFMA chain -- it starts from the row's bias divided by the
// accumulator scale (exact: the scale is a power of two) and one multiply by scale * -log2(e) gives t.
// The -ln2 of every SiLU value is folded into a staged node operand or applied once to the sums (callers).
// Per head and 16-edge tile this removes 16 adds and 16 multiplies of ~180 VALU instructions.
constexpr float kNegLog2e = -1.44269504088896340736f;
constexpr float kNegLn2 = -0.693147180559945309417f;
__device__ __forceinline__ float silu_u(float t) {
  return t * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
}
// t of the lane's four channels of block blk (sct = scale * -log2(e), sbt = bias / scale, both in LDS)
template <int KS>
__device__ __forceinline__ f4 block_t(const char* wl, const int (&wb)[KS], const float* sct, const float* sbt, int blk,
                                      const h8 (&b0)[KS], const h8 (&b1)[KS], int g) {
  constexpr int R = 32 * KS, PB = kD * R * (int)sizeof(_Float16);
  f4 acc = *reinterpret_cast<const f4*>(sbt + 16 * blk + 4 * g);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const char* f0 = wl + wb[ks] + blk * 16 * R * (int)sizeof(_Float16);
    const h8 w0 = *reinterpret_cast<const h8*>(f0);
    const h8 w1 = *reinterpret_cast<const h8*>(f0 + PB);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b1[ks], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, b0[ks], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b0[ks], acc, 0, 0, 0);
  }
  return acc * *reinterpret_cast<const f4*>(sct + 16 * blk + 4 * g);
}

// d pre / d r: W f' (no bias), scaled back by the row scale and the edge's derivative scale
template <int KS>
__device__ __forceinline__ f4 block_dpre(const char* wl, const int (&wb)[KS], const float* sc, float dsc, int blk,
                                         const h8 (&d0)[KS], const h8 (&d1)[KS], int g) {
  const f4 acc = block_acc<KS>(wl, wb, blk, d0, d1);
  const f4 s = *reinterpret_cast<const f4*>(sc + 16 * blk + 4 * g);
  return acc * (s * dsc);
}

// pre and d pre / d r of one block from ONE read of its weight fragments (the destination pass)
template <int KS, int D = kD>
__device__ __forceinline__ void block_pre_dpre(const char* wl, const int (&wb)[KS], const float* sc, const float* sb,
                                               float dsc, int blk, const h8 (&b0)[KS], const h8 (&b1)[KS],
                                               const h8 (&d0)[KS], const h8 (&d1)[KS], int g, f4& pre, f4& dpre) {
  constexpr int R = 32 * KS, PB = D * R * (int)sizeof(_Float16);
  f4 a = {0.f, 0.f, 0.f, 0.f}, d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const char* f0 = wl + wb[ks] + blk * 16 * R * (int)sizeof(_Float16);
    const h8 w0 = *reinterpret_cast<const h8*>(f0);
    const h8 w1 = *reinterpret_cast<const h8*>(f0 + PB);
    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b1[ks], a, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, d1[ks], d, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, b0[ks], a, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, d0[ks], d, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b0[ks], a, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, d0[ks], d, 0, 0, 0);
  }
  const f4 s = *reinterpret_cast<const f4*>(sc + 16 * blk + 4 * g);
  const f4 b = *reinterpret_cast<const f4*>(sb + 16 * blk + 4 * g);
  pre = a * s + b;
  dpre = d * (s * dsc);
}

// t (as block_t) and d pre / d r up to the edge's derivative scale (W f' times the row scale; the caller
// multiplies its r-sums by dsc once per edge) from ONE read of the block's weight fragments (the
// destination pass); sct / sbt the t-domain constants, sc the raw row scales
template <int KS>
__device__ __forceinline__ void block_t_dr(const char* wl, const int (&wb)[KS], const float* sct, const float* sbt,
                                           const float* sc, int blk, const h8 (&b0)[KS], const h8 (&b1)[KS],
                                           const h8 (&d0)[KS], const h8 (&d1)[KS], int g, f4& t, f4& dr) {
  constexpr int R = 32 * KS, PB = kD * R * (int)sizeof(_Float16);
  f4 a = *reinterpret_cast<const f4*>(sbt + 16 * blk + 4 * g), d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const char* f0 = wl + wb[ks] + blk * 16 * R * (int)sizeof(_Float16);
    const h8 w0 = *reinterpret_cast<const h8*>(f0);
    const h8 w1 = *reinterpret_cast<const h8*>(f0 + PB);
    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b1[ks], a, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, d1[ks], d, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, b0[ks], a, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, d0[ks], d, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, b0[ks], a, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, d0[ks], d, 0, 0, 0);
  }
  t = a * *reinterpret_cast<const f4*>(sct + 16 * blk + 4 * g);
  dr = d * *reinterpret_cast<const f4*>(sc + 16 * blk + 4 * g);
}
// t-domain SiLU with its derivative: sig = 1 / (1 + 2^t), u = t sig (SiLU = -ln2 u) and
// SiLU'(pre) = sig + SiLU (1 - sig) = sig - ln2 (u - u sig)
struct SiluT {
  float sig, u, d;
  __device__ __forceinline__ explicit SiluT(float t) {
    sig = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
    u = t * sig;
    d = fmaf(kNegLn2, fmaf(-u, sig, u), sig);
  }
};

// the seven 16-byte node-row gathers of one head for the lane's edge: k, v (x | v1 | v2), vec (3 axes)
struct Gat {
  f4 kk, vx, v1, v2, w0, w1, w2;
};
template <bool PL>
__device__ __forceinline__ void gather_kvw(Gat& X, rsrc_t Rk, rsrc_t Rv, rsrc_t Rw, int ok_, int ov_, int ow_, int h) {
  constexpr int PV = 4 * (PL ? kH : 16);
  const int sk = __builtin_amdgcn_readfirstlane(64 * h);
  const int sv = __builtin_amdgcn_readfirstlane(4 * (PL ? 16 : 48) * h);
  X.kk = bld4<0>(Rk, ok_, sk);
  X.vx = bld4<0>(Rv, ov_, sv);
  X.v1 = bld4<PV>(Rv, ov_, sv);
  X.v2 = bld4<2 * PV>(Rv, ov_, sv);
  X.w0 = bld4<0>(Rw, ow_, sk);
  X.w1 = bld4<4 * kH>(Rw, ow_, sk);
  X.w2 = bld4<8 * kH>(Rw, ow_, sk);
}

// the weight image and the row scales / biases into LDS (every thread of the workgroup)
template <int KS, int NT>
__device__ __forceinline__ void load_image(_Float16* w, float* s_sc, float* s_b, const _Float16* img, const float* wsc,
                                           const float* bias) {
  constexpr int R = 32 * KS;
  const u4* g = reinterpret_cast<const u4*>(img);
  u4* l = reinterpret_cast<u4*>(w);
  for (int i = threadIdx.x; i < 2 * kD * R / 8; i += NT) l[i] = g[i];
  for (int i = threadIdx.x; i < kD; i += NT) { s_sc[i] = wsc[i]; s_b[i] = bias[i]; }
}

// the same with the t-domain constants: scale * -log2(e) and bias / scale (the scale is 2^-k: exact)
template <int KS, int NT>
__device__ __forceinline__ void load_image_t(_Float16* w, float* s_sc, float* s_b, const _Float16* img,
                                             const float* wsc, const float* bias) {
  constexpr int R = 32 * KS;
  const u4* g = reinterpret_cast<const u4*>(img);
  u4* l = reinterpret_cast<u4*>(w);
  for (int i = threadIdx.x; i < 2 * kD * R / 8; i += NT) l[i] = g[i];
  for (int i = threadIdx.x; i < kD; i += NT) {
    const float sc = wsc[i];
    s_sc[i] = sc * kNegLog2e;
    s_b[i] = bias[i] / sc;  // sc = 2^-k: exact
  }
}

// per-lane A-fragment offsets of the item's head slice (block h0 of every part), opaque to the optimiser:
// the weight fragments are the same for every tile, and without it the compiler hoists all blocks'
// fragments out of the tile loop (hundreds of VGPRs)
template <int KS>
__device__ __forceinline__ void frag_offsets(int lane, int h0, int (&wb)[KS]) {
  constexpr int R = 32 * KS;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    wb[ks] = wfrag_base<KS>(lane, ks) + h0 * 16 * R * (int)sizeof(_Float16);
    asm volatile("" : "+v"(wb[ks]));
  }
}

// v row layout: planar [x | v1 | v2] H-blocks (PL) or the reference's per-head [x|v1|v2] d-blocks
template <bool PL> struct VL {
  static constexpr int head = PL ? 16 : 48;  // floats from head h to head h + 1 (x part)
  static constexpr int part = PL ? kH : 16;  // floats from part p to part p + 1
};

// The workgroup's nodes.  Hardware deals workgroups round-robin over the 8 XCDs; each XCD takes one
// contiguous node range, cut into chunks of `chk` nodes dealt round-robin to the XCD's m workgroups (the
// j-th takes chunks j, j + m, ...).  At any moment the XCD's CUs then work on ONE window of about m * chk
// consecutive -- Morton-ordered, so spatially close -- nodes whose source rows they share in that XCD's
// L2 (a contiguous range per workgroup spread an XCD's in-flight nodes over m separate windows).
struct Work {
  int x0, x1, j, m, chk, items;
};
template <int G>
__device__ __forceinline__ Work work_range(int n, int chk) {
  const int nwg = gridDim.x;
  Work W;
  W.chk = chk;
  if (nwg >= 16 && nwg % 8 == 0) {
    const int per = (n + 7) / 8, x = blockIdx.x % 8;
    W.x0 = min(n, x * per);
    W.x1 = min(n, W.x0 + per);
    W.j = blockIdx.x / 8;
    W.m = nwg / 8;
  } else {
    W.x0 = 0;
    W.x1 = n;
    W.j = blockIdx.x;
    W.m = nwg;
  }
  const int nch = (W.x1 - W.x0 + chk - 1) / chk;
  const int mine = W.j < nch ? (nch - W.j + W.m - 1) / W.m : 0;
  W.items = mine * chk * G;
  return W;
}
// item -> (node, slice); false past the end of the XCD's range (a partial last chunk)
template <int G>
__device__ __forceinline__ bool work_item(const Work& W, int it, int& t, int& sl) {
  const int per = W.chk * G, k = it / per, rem = it - k * per;
  t = W.x0 + (W.j + k * W.m) * W.chk + rem / G;
  sl = rem % G;
  return t < W.x1;
}
__device__ __forceinline__ int next_item(int* counter) {
  int it = 0;
  if (lane_id() == 0) it = atomicAdd(counter, 1);
  return __builtin_amdgcn_readfirstlane(__shfl(it, 0));
}

// one edge slot's per-tile inputs: source, cutoff, unit vector, fragment row offset
struct Edge {
  int s, fo;
  float C, ux, uy, uz;
  bool ok;
};
__device__ __forceinline__ Edge load_edge(int e, int re, const int32_t* src, const float* C, const float* u,
                                          const int32_t* frow, int frow_bytes, float usign) {
  Edge E;
  E.ok = e < re;
  E.s = 0;
  E.fo = kOOB;
  E.C = E.ux = E.uy = E.uz = 0.f;
  if (E.ok) {
    E.s = src[e];
    E.fo = frow[e] * frow_bytes;
    E.C = C[e];
    E.ux = usign * u[3 * (size_t)e];
    E.uy = usign * u[3 * (size_t)e + 1];
    E.uz = usign * u[3 * (size_t)e + 2];
  }
  return E;
}

// ------------------------------------------------------------------ forward
struct Fwd {
  int n, cap, chunk;
  const int32_t* row_ptr;
  const int32_t* src;
  const float* q; int ldq;
  const float* k; int ldk;
  const float* v; int ldv;
  const float* vec;  // [N][3][H] or NULL (layer 0)
  const float* C;
  const float* u;
  const int32_t* frow;  // fragment row of every edge (its pair row)
  const _Float16* fr;
  unsigned fr_bytes;
  const _Float16* img;
  const float* wsc;
  const float* bias;
  float* xo;
  float* veco;
};

// HPW heads per work item (G = 8 / HPW items per node); NW waves per workgroup
// HP: head-pipelined gathers -- head hh + 1's seven gathers are issued before head hh computes, so they
// have a whole head's MFMA and SiLU work to land (one extra set of gather registers); HP = 2 also issues
// the next tile's first head during the last head (the set then lives across the tile loop)
template <int KS, int HPW, int NW, bool PL, int HP = 0>
__global__ __launch_bounds__(NW * 64, 1) void k_fwd(Fwd P) {
  constexpr int R = 32 * KS, H = kH, G = kHeads / HPW, BS = 16 * R * (int)sizeof(_Float16);
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ __attribute__((aligned(16))) float s_sc[kD];
  __shared__ __attribute__((aligned(16))) float s_b[kD];
  __shared__ __attribute__((aligned(16))) float s_q[NW][16 * HPW];  // the item's q channels (per wave)
  __shared__ int s_next;
  load_image_t<KS, NW * 64>(w, s_sc, s_b, P.img, P.wsc, P.bias);
  if (threadIdx.x == 0) s_next = 0;
  __syncthreads();
  const Work W = work_range<G>(P.n, P.chunk);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4, wid = threadIdx.x >> 6;
  const rsrc_t Rk = make_rsrc(P.k, (unsigned)P.n * P.ldk * 4u), Rv = make_rsrc(P.v, (unsigned)P.n * P.ldv * 4u);
  const rsrc_t Rw = make_rsrc(P.vec, P.vec ? (unsigned)P.n * 3u * H * 4u : 0u);
  const rsrc_t Rf = make_rsrc(P.fr, P.fr_bytes);
  float* sq = s_q[wid];
  for (;;) {
    const int it = next_item(&s_next);
    if (it >= W.items) break;
    int t, sl;
    if (!work_item<G>(W, it, t, sl)) continue;
    const int h0 = sl * HPW;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    __builtin_amdgcn_wave_barrier();  // the previous item's reads of sq are done (in-order LDS)
    if (lane < 4 * HPW)  // q * -ln2: the dk SiLU's t-domain factor (silu_u)
      *reinterpret_cast<f4*>(sq + 4 * lane) =
          kNegLn2 * *reinterpret_cast<const f4*>(P.q + (size_t)t * P.ldq + 16 * h0 + 4 * lane);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f4 ax[HPW], a0[HPW], a1[HPW], a2[HPW];
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) ax[hh] = a0[hh] = a1[hh] = a2[hh] = f4{0.f, 0.f, 0.f, 0.f};
    const float* sct = s_sc + 16 * h0;
    const float* sbt = s_b + 16 * h0;
    // the next tile's edge scalars are loaded while this tile computes: a tile waits on one memory round
    // trip (its fragments and gathers), not two
    Edge En = load_edge(rb + c, re, P.src, P.C, P.u, P.frow, 8 * R, 1.f);
    Gat Xc;  // HP: the gathers of the head about to compute (issued one head ahead, across tiles too)
    for (int base = rb; base < re; base += 16) {
      const Edge E = En;
      TMD_DCHECK(E.s >= 0 && E.s < P.n);
      h8 B0[KS], B1[KS];
      load_frags<KS>(Rf, E.fo, g, 0, B0, B1);
      if (base + 16 < re) En = load_edge(base + 16 + c, re, P.src, P.C, P.u, P.frow, 8 * R, 1.f);
      // an edge past the row gathers from beyond the resources' ranges: its k, v and vec are 0, so its
      // terms vanish without masks (C = 0 as well)
      const int ok_ = E.ok ? (E.s * P.ldk + 4 * g) * 4 : kOOB;
      const int ov_ = E.ok ? (E.s * P.ldv + 4 * g) * 4 : kOOB;
      const int ow_ = E.ok ? (E.s * 3 * H + 4 * g) * 4 : kOOB;
      int wb[KS];
      frag_offsets<KS>(lane, h0, wb);
      const char* wt = reinterpret_cast<const char*>(w);
      if (HP == 1 || (HP == 2 && base == rb)) gather_kvw<PL>(Xc, Rk, Rv, Rw, ok_, ov_, ow_, h0);
      static_for<HPW>([&](auto hc) {
        constexpr int hh = decltype(hc)::value;
        Gat X, Xn;
        if (HP) {
          if (hh + 1 < HPW) {
            gather_kvw<PL>(Xn, Rk, Rv, Rw, ok_, ov_, ow_, h0 + hh + 1);
          } else if (HP == 2 && base + 16 < re) {  // the next tile's first head (its edge scalars are in En)
            gather_kvw<PL>(Xn, Rk, Rv, Rw, En.ok ? (En.s * P.ldk + 4 * g) * 4 : kOOB,
                           En.ok ? (En.s * P.ldv + 4 * g) * 4 : kOOB, En.ok ? (En.s * 3 * H + 4 * g) * 4 : kOOB, h0);
          }
          X = Xc;
        } else {
          gather_kvw<PL>(X, Rk, Rv, Rw, ok_, ov_, ow_, h0 + hh);
        }
        // t-domain: silu(pre) = -ln2 u(t); the -ln2 is in the staged q (dk) and applied to the sums (dv)
        const f4 pk = block_t<KS>(wt, wb, sct, sbt, hh, B0, B1, g);
        const f4 px = block_t<KS>(wt, wb, sct, sbt, 8 + hh, B0, B1, g);
        const f4 p1 = block_t<KS>(wt, wb, sct, sbt, 16 + hh, B0, B1, g);
        const f4 p2 = block_t<KS>(wt, wb, sct, sbt, 24 + hh, B0, B1, g);
        const f4 qv = *reinterpret_cast<const f4*>(sq + 16 * hh + 4 * g);
        float part = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) part += qv[i] * X.kk[i] * silu_u(pk[i]);
        const float att = gsum(part);
        const float a = Silu<float>(att).s * E.C;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ax[hh][i] += X.vx[i] * silu_u(px[i]) * a;
          const float v1e = X.v1[i] * silu_u(p1[i]);
          const float v2e = X.v2[i] * silu_u(p2[i]);
          a0[hh][i] += X.w0[i] * v1e + v2e * E.ux;
          a1[hh][i] += X.w1[i] * v1e + v2e * E.uy;
          a2[hh][i] += X.w2[i] * v1e + v2e * E.uz;
        }
        if (HP) Xc = Xn;
        __builtin_amdgcn_sched_barrier(0);
      });
      (void)BS;
    }
    // sum the 16 edge slots (lanes of a row); lane (g, c < HPW) stores head h0 + c's four channels 4 g + i
    f4 X{}, V0{}, V1{}, V2{};
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      f4 sx, s0, s1, s2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sx[i] = row_sum16(ax[hh][i]);
        s0[i] = row_sum16(a0[hh][i]);
        s1[i] = row_sum16(a1[hh][i]);
        s2[i] = row_sum16(a2[hh][i]);
      }
      if (c == hh) { X = sx; V0 = s0; V1 = s1; V2 = s2; }
    }
    if (c < HPW) {
      const int ch = 16 * (h0 + c) + 4 * g;
      X *= kNegLn2;  // the dv SiLUs' t-domain factor
      V0 *= kNegLn2;
      V1 *= kNegLn2;
      V2 *= kNegLn2;
      *reinterpret_cast<f4*>(P.xo + (size_t)t * H + ch) = X;
      float* vo = P.veco + (size_t)t * 3 * H + ch;
      *reinterpret_cast<f4*>(vo) = V0;
      *reinterpret_cast<f4*>(vo + H) = V1;
      *reinterpret_cast<f4*>(vo + 2 * H) = V2;
    }
  }
}

// ------------------------------------------------------------------ backward (force pass, "dr mode")
struct Bwd {
  int n, cap, acc, chunk;
  const int32_t* row_ptr;
  const int32_t* src;
  const float* q; int ldq;
  const float* k; int ldk;
  const float* v; int ldv;
  const float* vec;
  const float* C;
  const float* u;
  const int32_t* frow;
  const _Float16* fr;
  const float* dscale;
  unsigned fr_bytes;
  const _Float16* img;
  const float* wsc;
  const float* bias;
  const float* gx;    // [N][H]   dL/d x_agg
  const float* gvec;  // [N][3][H] dL/d vec_agg (and the layer's residual cotangent)
  float* gq;          // ld ldq
  float* gk;          // ld ldk
  float* gv;          // ld ldv (layout of v)
  float* gveci;       // [N][3][H] or NULL
  float* gC;
  float* gu;
  float* gr;
  float* part;        // [S][5][cap] per-slice edge sums (S = 8 / HPW > 1), summed by k_edge_combine
};

// Destination pass: for edge e = (t <- s) of t's row: gq[t] and the per-edge g_cut, g_unit, g_r (the
// projection gradient contracted with d pre / d r in registers).  HPW heads per work item; t's q, gx,
// gvec channels of the slice staged in the wave's LDS slot.  The per-edge sums run over every channel:
// with one slice (HPW = 8) they are written directly, else each slice writes its part for k_edge_combine.
template <int KS, int HPW, int NW, bool PL, int HP = 0>
__global__ __launch_bounds__(NW * 64, 1) void k_bwd_dst(Bwd P) {
  constexpr int R = 32 * KS, H = kH, G = kHeads / HPW, CH = 16 * HPW;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ __attribute__((aligned(16))) float s_sc[kD];
  __shared__ __attribute__((aligned(16))) float s_b[kD];
  __shared__ __attribute__((aligned(16))) float s_raw[kD];  // the raw row scales (d pre / d r)
  __shared__ __attribute__((aligned(16))) float s_node[NW][5 * CH];  // q | gx | gvec (3) of the slice
  __shared__ int s_next;
  load_image_t<KS, NW * 64>(w, s_sc, s_b, P.img, P.wsc, P.bias);
  for (int i = threadIdx.x; i < kD; i += NW * 64) s_raw[i] = P.wsc[i];
  if (threadIdx.x == 0) s_next = 0;
  if (G == 1) {  // static-capacity lists: edge slots past the last row belong to no row -- zeroed here
    const int e0 = min(P.row_ptr[P.n], P.cap);
    for (int e = e0 + blockIdx.x * NW * 64 + threadIdx.x; e < P.cap; e += gridDim.x * NW * 64) {
      P.gC[e] = 0.f;
      P.gu[3 * (size_t)e] = P.gu[3 * (size_t)e + 1] = P.gu[3 * (size_t)e + 2] = 0.f;
      P.gr[e] = 0.f;
    }
  }
  __syncthreads();
  const Work W = work_range<G>(P.n, P.chunk);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4, wid = threadIdx.x >> 6;
  const bool acc_edge = P.acc & TMDNET_ACC_EDGE, ag = P.acc & TMDNET_ACC_GRADS;
  const rsrc_t Rk = make_rsrc(P.k, (unsigned)P.n * P.ldk * 4u), Rv = make_rsrc(P.v, (unsigned)P.n * P.ldv * 4u);
  const rsrc_t Rw = make_rsrc(P.vec, P.vec ? (unsigned)P.n * 3u * H * 4u : 0u);
  const rsrc_t Rf = make_rsrc(P.fr, P.fr_bytes);
  float* nd = s_node[wid];
  for (;;) {
    const int it = next_item(&s_next);
    if (it >= W.items) break;
    int t, sl;
    if (!work_item<G>(W, it, t, sl)) continue;
    const int h0 = sl * HPW;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    // stage the slice's q[t] | gx[t] | gvec[t] channels (5 CH floats)
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < 5 * CH / 4; i += 64) {
      const int part = i / (CH / 4), j = i % (CH / 4);
      const float* sp = part == 0 ? P.q + (size_t)t * P.ldq : part == 1 ? P.gx + (size_t)t * H
                                                             : P.gvec + ((size_t)t * 3 + (part - 2)) * H;
      *reinterpret_cast<f4*>(nd + 4 * i) = *reinterpret_cast<const f4*>(sp + 16 * h0 + 4 * j);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float* sct = s_sc + 16 * h0;
    const float* sbt = s_b + 16 * h0;
    const float* scr = s_raw + 16 * h0;
    f4 gq[HPW];
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) gq[hh] = f4{0.f, 0.f, 0.f, 0.f};
    Edge En = load_edge(rb + c, re, P.src, P.C, P.u, P.frow, 8 * R, 1.f);  // (next tile's scalars: as k_fwd)
    Gat Xc;
    for (int base = rb; base < re; base += 16) {
      const int e = base + c;
      const Edge E = En;
      if (base + 16 < re) En = load_edge(base + 16 + c, re, P.src, P.C, P.u, P.frow, 8 * R, 1.f);
      TMD_DCHECK(E.s >= 0 && E.s < P.n);
      h8 B0[KS], B1[KS], D0[KS], D1[KS];
      load_frags<KS>(Rf, E.fo, g, 0, B0, B1);
      load_frags<KS>(Rf, E.fo, g, 1, D0, D1);
      const float dsc = E.ok ? P.dscale[E.fo / (8 * R)] : 1.f;
      const int ok_ = E.ok ? (E.s * P.ldk + 4 * g) * 4 : kOOB;
      const int ov_ = E.ok ? (E.s * P.ldv + 4 * g) * 4 : kOOB;
      const int ow_ = E.ok ? (E.s * 3 * H + 4 * g) * 4 : kOOB;
      int wb[KS];
      frag_offsets<KS>(lane, h0, wb);
      const char* wt = reinterpret_cast<const char*>(w);
      float eC = 0.f, er = 0.f, eu0 = 0.f, eu1 = 0.f, eu2 = 0.f;
      if (HP == 1 || (HP == 2 && base == rb)) gather_kvw<PL>(Xc, Rk, Rv, Rw, ok_, ov_, ow_, h0);
      static_for<HPW>([&](auto hc) {
        constexpr int hh = decltype(hc)::value;
        Gat X, Xn;
        if (HP) {  // head-pipelined gathers, as k_fwd
          if (hh + 1 < HPW) {
            gather_kvw<PL>(Xn, Rk, Rv, Rw, ok_, ov_, ow_, h0 + hh + 1);
          } else if (HP == 2 && base + 16 < re) {
            gather_kvw<PL>(Xn, Rk, Rv, Rw, En.ok ? (En.s * P.ldk + 4 * g) * 4 : kOOB,
                           En.ok ? (En.s * P.ldv + 4 * g) * 4 : kOOB, En.ok ? (En.s * 3 * H + 4 * g) * 4 : kOOB, h0);
          }
          X = Xc;
        } else {
          gather_kvw<PL>(X, Rk, Rv, Rw, ok_, ov_, ow_, h0 + hh);
        }
        const f4 qd = *reinterpret_cast<const f4*>(nd + 16 * hh + 4 * g);
        const f4 gxd = *reinterpret_cast<const f4*>(nd + CH + 16 * hh + 4 * g);
        // the attention part (dk, dv_x blocks) first: its head sums gate every other term.  t-domain
        // (SiluT): the SiLU values enter as u = SiLU / -ln2 -- the head sums, gq and g_unit take the -ln2
        // once -- and the r-sums as (d pre / d r) / dsc, multiplied by dsc once per edge
        f4 tk, rk, tx, rx;
        block_t_dr<KS>(wt, wb, sct, sbt, scr, hh, B0, B1, D0, D1, g, tk, rk);
        block_t_dr<KS>(wt, wb, sct, sbt, scr, 8 + hh, B0, B1, D0, D1, g, tx, rx);
        f4 kdu;
        float pa = 0.f, pg = 0.f, sk = 0.f, sx = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const SiluT fk(tk[i]), fx(tx[i]);
          const float qk = qd[i] * X.kk[i], gv = gxd[i] * X.vx[i];
          kdu[i] = X.kk[i] * fk.u;
          pa = fmaf(qk, fk.u, pa);
          sk = fmaf(qk, fk.d * rk[i], sk);
          pg = fmaf(gv, fx.u, pg);
          sx = fmaf(gv, fx.d * rx[i], sx);
        }
        const float att = kNegLn2 * gsum(pa), ga = kNegLn2 * gsum(pg);
        const Silu<float> sa(att);
        const float a = sa.s * E.C;
        const float gs = ga * E.C * sa.d(att);
        eC += ga * sa.s;
        er = fmaf(gs, sk, fmaf(a, sx, er));
#pragma unroll
        for (int i = 0; i < 4; ++i) gq[hh][i] = fmaf(gs, kdu[i], gq[hh][i]);
        // the vector parts (dv_1, dv_2 blocks)
        const f4 g0 = *reinterpret_cast<const f4*>(nd + 2 * CH + 16 * hh + 4 * g);
        const f4 g1 = *reinterpret_cast<const f4*>(nd + 3 * CH + 16 * hh + 4 * g);
        const f4 g2 = *reinterpret_cast<const f4*>(nd + 4 * CH + 16 * hh + 4 * g);
        f4 t1, r1, t2, r2;
        block_t_dr<KS>(wt, wb, sct, sbt, scr, 16 + hh, B0, B1, D0, D1, g, t1, r1);
        block_t_dr<KS>(wt, wb, sct, sbt, scr, 24 + hh, B0, B1, D0, D1, g, t2, r2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const SiluT f1(t1[i]), f2(t2[i]);
          const float gv1e = g0[i] * X.w0[i] + g1[i] * X.w1[i] + g2[i] * X.w2[i];
          const float gv2e = g0[i] * E.ux + g1[i] * E.uy + g2[i] * E.uz;
          er = fmaf(gv1e * X.v1[i], f1.d * r1[i], er);
          er = fmaf(gv2e * X.v2[i], f2.d * r2[i], er);
          const float v2u = X.v2[i] * f2.u;
          eu0 = fmaf(g0[i], v2u, eu0);
          eu1 = fmaf(g1[i], v2u, eu1);
          eu2 = fmaf(g2[i], v2u, eu2);
        }
        if (HP) Xc = Xn;
        __builtin_amdgcn_sched_barrier(0);
      });
      // the edge sums over the 4 lane groups (eC is already a head total in every lane)
      er = dsc * gsum(er);
      eu0 = kNegLn2 * gsum(eu0);
      eu1 = kNegLn2 * gsum(eu1);
      eu2 = kNegLn2 * gsum(eu2);
      if (g == 0 && E.ok) {
        if (G == 1) {
          float* gu = P.gu + 3 * (size_t)e;
          if (acc_edge) {
            P.gC[e] += eC;
            gu[0] += eu0; gu[1] += eu1; gu[2] += eu2;
            P.gr[e] += er;
          } else {
            P.gC[e] = eC;
            gu[0] = eu0; gu[1] = eu1; gu[2] = eu2;
            P.gr[e] = er;
          }
        } else {
          float* pp = P.part + (size_t)sl * 5 * P.cap + e;
          pp[0] = eC;
          pp[P.cap] = eu0;
          pp[2 * (size_t)P.cap] = eu1;
          pp[3 * (size_t)P.cap] = eu2;
          pp[4 * (size_t)P.cap] = er;
        }
      }
    }
    // gq: sum the 16 edge slots; lane (g, c < HPW) stores head h0 + c's channels 4 g + i
    f4 Q{};
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      f4 sq;
#pragma unroll
      for (int i = 0; i < 4; ++i) sq[i] = kNegLn2 * row_sum16(gq[hh][i]);
      if (c == hh) Q = sq;
    }
    if (c < HPW) {
      float* d = P.gq + (size_t)t * P.ldq + 16 * (h0 + c) + 4 * g;
      if (ag) Q += *reinterpret_cast<const f4*>(d);
      *reinterpret_cast<f4*>(d) = Q;
    }
  }
}

// the per-slice edge sums of the destination pass -> g_cut, g_unit, g_r (in slice order: deterministic);
// also zeroes the static-capacity padding slots [row_ptr[n], cap)
__global__ __launch_bounds__(256) void k_edge_combine(Bwd P, int S) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= P.cap) return;
  const int e0 = min(P.row_ptr[P.n], P.cap);
  float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < e0) {
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int j = 0; j < 5; ++j) v[j] += P.part[((size_t)s * 5 + j) * P.cap + e];
  }
  float* gu = P.gu + 3 * (size_t)e;
  if ((P.acc & TMDNET_ACC_EDGE) && e < e0) {
    P.gC[e] += v[0];
    gu[0] += v[1]; gu[1] += v[2]; gu[2] += v[3];
    P.gr[e] += v[4];
  } else {
    P.gC[e] = v[0];
    gu[0] = v[1]; gu[1] = v[2]; gu[2] = v[3];
    P.gr[e] = v[4];
  }
}

// Source pass: node j as the source of the reversed edges j -> m of its row (same dk / dv / cutoff,
// unit vector negated): gk, gv (v's layout), gvec_in (+ the residual cotangent with
// TMDNET_ACC_VEC_RESIDUAL).  HPW heads per work item; j's k / v / vec channels in registers.
template <int KS, int HPW, int NW, bool PL>
__global__ __launch_bounds__(NW * 64, 1) void k_bwd_src(Bwd P) {
  constexpr int R = 32 * KS, H = kH, G = kHeads / HPW, CH = 16 * HPW;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ __attribute__((aligned(16))) float s_sc[kD];
  __shared__ __attribute__((aligned(16))) float s_b[kD];
  __shared__ __attribute__((aligned(16))) float s_node[NW][6 * CH];  // k | v_x | v_1 | vec (3) of the slice
  __shared__ int s_next;
  load_image_t<KS, NW * 64>(w, s_sc, s_b, P.img, P.wsc, P.bias);
  if (threadIdx.x == 0) s_next = 0;
  __syncthreads();
  const Work W = work_range<G>(P.n, P.chunk);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4, wid = threadIdx.x >> 6;
  const bool ag = P.acc & TMDNET_ACC_GRADS, resid = P.acc & TMDNET_ACC_VEC_RESIDUAL;
  float* nd = s_node[wid];
  const rsrc_t Rq = make_rsrc(P.q, (unsigned)P.n * P.ldq * 4u), Rgx = make_rsrc(P.gx, (unsigned)P.n * H * 4u);
  const rsrc_t Rgv = make_rsrc(P.gvec, (unsigned)P.n * 3u * H * 4u);
  const rsrc_t Rf = make_rsrc(P.fr, P.fr_bytes);
  constexpr int PV = VL<PL>::part;
  for (;;) {
    const int it = next_item(&s_next);
    if (it >= W.items) break;
    int j, sl;
    if (!work_item<G>(W, it, j, sl)) continue;
    const int h0 = sl * HPW;
    const int rb = min(P.row_ptr[j], P.cap), re = min(P.row_ptr[j + 1], P.cap);
    // stage j's k, v_x, v_1, vec channels of the slice (6 CH floats; vec absent: zeros)
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < 6 * CH / 4; i += 64) {
      const int part = i / (CH / 4), jj = i % (CH / 4), hh = jj / 4, o = 4 * (jj % 4);
      const int h = h0 + hh;
      f4 val{0.f, 0.f, 0.f, 0.f};
      if (part == 0) val = *reinterpret_cast<const f4*>(P.k + (size_t)j * P.ldk + 16 * h + o);
      else if (part <= 2)
        val = *reinterpret_cast<const f4*>(P.v + (size_t)j * P.ldv + VL<PL>::head * h + (part - 1) * PV + o);
      else if (P.vec) val = *reinterpret_cast<const f4*>(P.vec + ((size_t)j * 3 + (part - 3)) * H + 16 * h + o);
      // k, v_x, v_1 times -ln2: the t-domain factor of the SiLU values they multiply (silu_u)
      *reinterpret_cast<f4*>(nd + 4 * i) = part <= 2 ? kNegLn2 * val : val;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f4 gk[HPW], gvx[HPW], gv1[HPW], gv2[HPW], gw0[HPW], gw1[HPW], gw2[HPW];
    const f4 z4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) gk[hh] = gvx[hh] = gv1[hh] = gv2[hh] = gw0[hh] = gw1[hh] = gw2[hh] = z4;
    auto own = [&](int part, int hh) { return *reinterpret_cast<const f4*>(nd + part * CH + 16 * hh + 4 * g); };
    const float* sct = s_sc + 16 * h0;
    const float* sbt = s_b + 16 * h0;
    // the reversed edges j -> m; the next tile's scalars load while this one computes (as k_fwd)
    Edge En = load_edge(rb + c, re, P.src, P.C, P.u, P.frow, 8 * R, -1.f);
    for (int base = rb; base < re; base += 16) {
      const Edge E = En;
      if (base + 16 < re) En = load_edge(base + 16 + c, re, P.src, P.C, P.u, P.frow, 8 * R, -1.f);
      TMD_DCHECK(E.s >= 0 && E.s < P.n);
      h8 B0[KS], B1[KS];
      load_frags<KS>(Rf, E.fo, g, 0, B0, B1);
      const int oq = E.ok ? (E.s * P.ldq + 4 * g) * 4 : kOOB;
      const int ox = E.ok ? (E.s * H + 4 * g) * 4 : kOOB;
      const int og = E.ok ? (E.s * 3 * H + 4 * g) * 4 : kOOB;
      int wb[KS];
      frag_offsets<KS>(lane, h0, wb);
      const char* wt = reinterpret_cast<const char*>(w);
      static_for<HPW>([&](auto hc) {
        constexpr int hh = decltype(hc)::value;
        const int sh = __builtin_amdgcn_readfirstlane(64 * (h0 + hh));
        const f4 qm = bld4<0>(Rq, oq, sh), gxm = bld4<0>(Rgx, ox, sh);
        const f4 g0 = bld4<0>(Rgv, og, sh), g1 = bld4<4 * kH>(Rgv, og, sh), g2 = bld4<8 * kH>(Rgv, og, sh);
        // t-domain SiLU values (silu = -ln2 u): the -ln2 is in the staged k, v_x, v_1 and on the final sums
        const f4 pk = block_t<KS>(wt, wb, sct, sbt, hh, B0, B1, g);
        const f4 px = block_t<KS>(wt, wb, sct, sbt, 8 + hh, B0, B1, g);
        f4 dk, dvx;
        float pa = 0.f, pg = 0.f;
        const f4 kj = own(0, hh), vxj = own(1, hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dk[i] = silu_u(pk[i]);
          dvx[i] = silu_u(px[i]);
          pa += qm[i] * kj[i] * dk[i];
          pg += gxm[i] * vxj[i] * dvx[i];
        }
        const float att = gsum(pa), ga = gsum(pg);
        const Silu<float> sa(att);
        const float a = sa.s * E.C;
        const float gs = ga * E.C * sa.d(att);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gk[hh][i] += gs * qm[i] * dk[i];
          gvx[hh][i] += gxm[i] * a * dvx[i];
        }
        const f4 p1 = block_t<KS>(wt, wb, sct, sbt, 16 + hh, B0, B1, g);
        const f4 p2 = block_t<KS>(wt, wb, sct, sbt, 24 + hh, B0, B1, g);
        const f4 v1j = own(2, hh), w0j = own(3, hh), w1j = own(4, hh), w2j = own(5, hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dv1 = silu_u(p1[i]), dv2 = silu_u(p2[i]);
          const float gv1e = g0[i] * w0j[i] + g1[i] * w1j[i] + g2[i] * w2j[i];
          gv1[hh][i] += gv1e * dv1;
          const float gv2e = g0[i] * E.ux + g1[i] * E.uy + g2[i] * E.uz;
          gv2[hh][i] += gv2e * dv2;
          const float v1e = v1j[i] * dv1;
          gw0[hh][i] += g0[i] * v1e;
          gw1[hh][i] += g1[i] * v1e;
          gw2[hh][i] += g2[i] * v1e;
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    }
    // sum the 16 edge slots; lane (g, c < HPW) stores head h0 + c
    f4 K{}, VX{}, V1{}, V2{}, W0{}, W1{}, W2{};
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      f4 a[7];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[0][i] = row_sum16(gk[hh][i]);
        a[1][i] = row_sum16(gvx[hh][i]);
        a[2][i] = row_sum16(gv1[hh][i]);
        a[3][i] = row_sum16(gv2[hh][i]);
        a[4][i] = row_sum16(gw0[hh][i]);
        a[5][i] = row_sum16(gw1[hh][i]);
        a[6][i] = row_sum16(gw2[hh][i]);
      }
      if (c == hh) { K = a[0]; VX = a[1]; V1 = a[2]; V2 = a[3]; W0 = a[4]; W1 = a[5]; W2 = a[6]; }
    }
    if (c < HPW) {
      const int h = h0 + c;
      K *= kNegLn2;  // the t-domain factor of dk, dv_x, dv_1, dv_2 (gw's is in the staged v_1)
      VX *= kNegLn2;
      V1 *= kNegLn2;
      V2 *= kNegLn2;
      auto put = [&](float* d, f4 val) {
        if (ag) val += *reinterpret_cast<const f4*>(d);
        *reinterpret_cast<f4*>(d) = val;
      };
      put(P.gk + (size_t)j * P.ldk + 16 * h + 4 * g, K);
      float* gvj = P.gv + (size_t)j * P.ldv + VL<PL>::head * h + 4 * g;
      put(gvj, VX);
      put(gvj + PV, V1);
      put(gvj + 2 * PV, V2);
      if (P.gveci) {
        if (resid) {
          const float* rr = P.gvec + (size_t)j * 3 * H + 16 * h + 4 * g;
          W0 += *reinterpret_cast<const f4*>(rr);
          W1 += *reinterpret_cast<const f4*>(rr + H);
          W2 += *reinterpret_cast<const f4*>(rr + 2 * H);
        }
        float* gw = P.gveci + (size_t)j * 3 * H + 16 * h + 4 * g;
        put(gw, W0);
        put(gw + H, W1);
        put(gw + 2 * H, W2);
      }
    }
  }
}

// Merged backward (round 5): ONE pass over node t's row does both passes above.  Edge e = (t <- s) is the
// destination pass's edge and, read reversed (t -> s, unit vector negated), the source pass's edge of t's
// row -- both with the same pair's dk / dv pre-activations, which are now formed (with their r-derivatives)
// once per edge and head instead of once in each pass.  Every output is t's (gq | gk, gv, gvec_in) or e's
// (the per-edge sums), so it stays deterministic without atomics.  Per (edge, head) the lane gathers s's
// k, v, vec (destination terms) and q, gx, gvec (source terms): 12 16-byte loads.
template <int KS, int HPW, int NW, bool PL>
__global__ __launch_bounds__(NW * 64, 1) void k_bwd_row(Bwd P) {
  constexpr int R = 32 * KS, H = kH, G = kHeads / HPW, CH = 16 * HPW;
  // t's staged channels of the slice: q | gx | gvec (3) | k | v_x | v_1 | vec (3)
  constexpr int NQ = 0, NGX = 1, NGV = 2, NK = 5, NVX = 6, NV1 = 7, NW0 = 8, NP = 11;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ __attribute__((aligned(16))) float s_sc[kD];
  __shared__ __attribute__((aligned(16))) float s_b[kD];
  __shared__ __attribute__((aligned(16))) float s_node[NW][NP * CH];
  __shared__ int s_next;
  load_image<KS, NW * 64>(w, s_sc, s_b, P.img, P.wsc, P.bias);
  if (threadIdx.x == 0) s_next = 0;
  if (G == 1) {  // static-capacity lists: edge slots past the last row belong to no row -- zeroed here
    const int e0 = min(P.row_ptr[P.n], P.cap);
    for (int e = e0 + blockIdx.x * NW * 64 + threadIdx.x; e < P.cap; e += gridDim.x * NW * 64) {
      P.gC[e] = 0.f;
      P.gu[3 * (size_t)e] = P.gu[3 * (size_t)e + 1] = P.gu[3 * (size_t)e + 2] = 0.f;
      P.gr[e] = 0.f;
    }
  }
  __syncthreads();
  const Work W = work_range<G>(P.n, P.chunk);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4, wid = threadIdx.x >> 6;
  const bool acc_edge = P.acc & TMDNET_ACC_EDGE, ag = P.acc & TMDNET_ACC_GRADS;
  const bool resid = P.acc & TMDNET_ACC_VEC_RESIDUAL;
  const rsrc_t Rk = make_rsrc(P.k, (unsigned)P.n * P.ldk * 4u), Rv = make_rsrc(P.v, (unsigned)P.n * P.ldv * 4u);
  const rsrc_t Rw = make_rsrc(P.vec, P.vec ? (unsigned)P.n * 3u * H * 4u : 0u);
  const rsrc_t Rq = make_rsrc(P.q, (unsigned)P.n * P.ldq * 4u), Rgx = make_rsrc(P.gx, (unsigned)P.n * H * 4u);
  const rsrc_t Rgv = make_rsrc(P.gvec, (unsigned)P.n * 3u * H * 4u);
  const rsrc_t Rf = make_rsrc(P.fr, P.fr_bytes);
  constexpr int PV = VL<PL>::part;
  float* nd = s_node[wid];
  auto own = [&](int part, int hh) { return *reinterpret_cast<const f4*>(nd + part * CH + 16 * hh + 4 * g); };
  for (;;) {
    const int it = next_item(&s_next);
    if (it >= W.items) break;
    int t, sl;
    if (!work_item<G>(W, it, t, sl)) continue;
    const int h0 = sl * HPW;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < NP * CH / 4; i += 64) {
      const int part = i / (CH / 4), jj = i % (CH / 4), hh = jj / 4, o = 4 * (jj % 4);
      const int h = h0 + hh;
      f4 val{0.f, 0.f, 0.f, 0.f};
      if (part == NQ) val = *reinterpret_cast<const f4*>(P.q + (size_t)t * P.ldq + 16 * h + o);
      else if (part == NGX) val = *reinterpret_cast<const f4*>(P.gx + (size_t)t * H + 16 * h + o);
      else if (part < NK) val = *reinterpret_cast<const f4*>(P.gvec + ((size_t)t * 3 + (part - NGV)) * H + 16 * h + o);
      else if (part == NK) val = *reinterpret_cast<const f4*>(P.k + (size_t)t * P.ldk + 16 * h + o);
      else if (part < NW0)
        val = *reinterpret_cast<const f4*>(P.v + (size_t)t * P.ldv + VL<PL>::head * h + (part - NVX) * PV + o);
      else if (P.vec) val = *reinterpret_cast<const f4*>(P.vec + ((size_t)t * 3 + (part - NW0)) * H + 16 * h + o);
      *reinterpret_cast<f4*>(nd + 4 * i) = val;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float* sct = s_sc + 16 * h0;
    const float* sbt = s_b + 16 * h0;
    const f4 z4{0.f, 0.f, 0.f, 0.f};
    // source-term sums: gk, gv_x, gv_2 and A_a = sum_s gvec[s]_a silu(p1) (a = axis); gvec_in[t]_a =
    // v_1[t] A_a and gv_1[t] = sum_a vec[t]_a A_a are formed from A once per node, not per edge
    f4 gq[HPW], gk[HPW], gvx[HPW], gv2[HPW], A0[HPW], A1[HPW], A2[HPW];
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) gq[hh] = gk[hh] = gvx[hh] = gv2[hh] = A0[hh] = A1[hh] = A2[hh] = z4;
    Edge En = load_edge(rb + c, re, P.src, P.C, P.u, P.frow, 8 * R, 1.f);
    for (int base = rb; base < re; base += 16) {
      const int e = base + c;
      const Edge E = En;
      if (base + 16 < re) En = load_edge(base + 16 + c, re, P.src, P.C, P.u, P.frow, 8 * R, 1.f);
      TMD_DCHECK(E.s >= 0 && E.s < P.n);
      h8 B0[KS], B1[KS], D0[KS], D1[KS];
      load_frags<KS>(Rf, E.fo, g, 0, B0, B1);
      load_frags<KS>(Rf, E.fo, g, 1, D0, D1);
      const float dsc = E.ok ? P.dscale[E.fo / (8 * R)] : 1.f;
      const int ok_ = E.ok ? (E.s * P.ldk + 4 * g) * 4 : kOOB;
      const int ov_ = E.ok ? (E.s * P.ldv + 4 * g) * 4 : kOOB;
      const int ow_ = E.ok ? (E.s * 3 * H + 4 * g) * 4 : kOOB;
      const int oq = E.ok ? (E.s * P.ldq + 4 * g) * 4 : kOOB;
      const int ox = E.ok ? (E.s * H + 4 * g) * 4 : kOOB;
      int wb[KS];
      frag_offsets<KS>(lane, h0, wb);
      const char* wt = reinterpret_cast<const char*>(w);
      float eC = 0.f, er = 0.f, eu0 = 0.f, eu1 = 0.f, eu2 = 0.f;
      static_for<HPW>([&](auto hc) {
        constexpr int hh = decltype(hc)::value;
        // the attention phase's gathers: s's k, v_x (destination terms), q, gx (source terms)
        const int sh = __builtin_amdgcn_readfirstlane(64 * (h0 + hh));
        const int sv = __builtin_amdgcn_readfirstlane(4 * VL<PL>::head * (h0 + hh));
        const f4 kk = bld4<0>(Rk, ok_, sh), vx = bld4<0>(Rv, ov_, sv);
        const f4 qm = bld4<0>(Rq, oq, sh), gxm = bld4<0>(Rgx, ox, sh);
        const f4 qd = own(NQ, hh), gxd = own(NGX, hh), kt = own(NK, hh), vxt = own(NVX, hh);
        // the attention blocks (dk, dv_x) of both directions
        f4 pk, rk, px, rx;
        block_pre_dpre<KS>(wt, wb, sct, sbt, dsc, hh, B0, B1, D0, D1, g, pk, rk);
        block_pre_dpre<KS>(wt, wb, sct, sbt, dsc, 8 + hh, B0, B1, D0, D1, g, px, rx);
        f4 kdk, gpk, gpx, dk, dvx;
        float pa = 0.f, pg = 0.f, qa = 0.f, qg = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const Silu<float> fk(pk[i]);
          dk[i] = fk.s;
          kdk[i] = kk[i] * fk.s;
          gpk[i] = qd[i] * kk[i] * fk.d(pk[i]);  // x gs below
          pa += qd[i] * kdk[i];
          qa += qm[i] * kt[i] * fk.s;
          const Silu<float> fx(px[i]);
          dvx[i] = fx.s;
          pg += gxd[i] * vx[i] * fx.s;
          gpx[i] = gxd[i] * vx[i] * fx.d(px[i]);  // x a below
          qg += gxm[i] * vxt[i] * fx.s;
        }
        const float att = gsum(pa), ga = gsum(pg), att2 = gsum(qa), ga2 = gsum(qg);
        const Silu<float> sa(att), sa2(att2);
        const float a = sa.s * E.C, a2 = sa2.s * E.C;
        const float gs = ga * E.C * sa.d(att), gs2 = ga2 * E.C * sa2.d(att2);
        eC += ga * sa.s;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gq[hh][i] += gs * kdk[i];
          er += gs * gpk[i] * rk[i] + a * gpx[i] * rx[i];
          gk[hh][i] += gs2 * qm[i] * dk[i];
          gvx[hh][i] += gxm[i] * a2 * dvx[i];
        }
        __builtin_amdgcn_sched_barrier(0);
        // the vector phase: s's v_1, v_2, vec (destination) and gvec (source terms)
        constexpr int PVB = 4 * VL<PL>::part;
        const f4 v1 = bld4<PVB>(Rv, ov_, sv), v2 = bld4<2 * PVB>(Rv, ov_, sv);
        const f4 w0 = bld4<0>(Rw, ow_, sh), w1 = bld4<4 * kH>(Rw, ow_, sh), w2 = bld4<8 * kH>(Rw, ow_, sh);
        const f4 m0 = bld4<0>(Rgv, ow_, sh), m1 = bld4<4 * kH>(Rgv, ow_, sh), m2 = bld4<8 * kH>(Rgv, ow_, sh);
        const f4 g0 = own(NGV, hh), g1 = own(NGV + 1, hh), g2 = own(NGV + 2, hh);
        f4 p1, r1, p2, r2;
        block_pre_dpre<KS>(wt, wb, sct, sbt, dsc, 16 + hh, B0, B1, D0, D1, g, p1, r1);
        block_pre_dpre<KS>(wt, wb, sct, sbt, dsc, 24 + hh, B0, B1, D0, D1, g, p2, r2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const Silu<float> f1(p1[i]), f2(p2[i]);
          const float gv1e = g0[i] * w0[i] + g1[i] * w1[i] + g2[i] * w2[i];
          const float gv2e = g0[i] * E.ux + g1[i] * E.uy + g2[i] * E.uz;
          er += gv1e * v1[i] * f1.d(p1[i]) * r1[i] + gv2e * v2[i] * f2.d(p2[i]) * r2[i];
          const float v2e = v2[i] * f2.s;
          eu0 += g0[i] * v2e;
          eu1 += g1[i] * v2e;
          eu2 += g2[i] * v2e;
          // source terms of t -> s (unit vector -u)
          gv2[hh][i] -= (m0[i] * E.ux + m1[i] * E.uy + m2[i] * E.uz) * f2.s;
          A0[hh][i] += m0[i] * f1.s;
          A1[hh][i] += m1[i] * f1.s;
          A2[hh][i] += m2[i] * f1.s;
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      er = gsum(er);
      eu0 = gsum(eu0);
      eu1 = gsum(eu1);
      eu2 = gsum(eu2);
      if (g == 0 && E.ok) {
        if (G == 1) {
          float* gu = P.gu + 3 * (size_t)e;
          if (acc_edge) {
            P.gC[e] += eC;
            gu[0] += eu0; gu[1] += eu1; gu[2] += eu2;
            P.gr[e] += er;
          } else {
            P.gC[e] = eC;
            gu[0] = eu0; gu[1] = eu1; gu[2] = eu2;
            P.gr[e] = er;
          }
        } else {
          float* pp = P.part + (size_t)sl * 5 * P.cap + e;
          pp[0] = eC;
          pp[P.cap] = eu0;
          pp[2 * (size_t)P.cap] = eu1;
          pp[3 * (size_t)P.cap] = eu2;
          pp[4 * (size_t)P.cap] = er;
        }
      }
    }
    // sum the 16 edge slots; lane (g, c < HPW) stores head h0 + c
    f4 Q{}, K{}, VX{}, V2{}, S0{}, S1{}, S2{};
#pragma unroll
    for (int hh = 0; hh < HPW; ++hh) {
      f4 a[7];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[0][i] = row_sum16(gq[hh][i]);
        a[1][i] = row_sum16(gk[hh][i]);
        a[2][i] = row_sum16(gvx[hh][i]);
        a[3][i] = row_sum16(gv2[hh][i]);
        a[4][i] = row_sum16(A0[hh][i]);
        a[5][i] = row_sum16(A1[hh][i]);
        a[6][i] = row_sum16(A2[hh][i]);
      }
      if (c == hh) { Q = a[0]; K = a[1]; VX = a[2]; V2 = a[3]; S0 = a[4]; S1 = a[5]; S2 = a[6]; }
    }
    if (c < HPW) {
      const int h = h0 + c;
      const f4 v1t = own(NV1, c);
      const f4 V1 = own(NW0, c) * S0 + own(NW0 + 1, c) * S1 + own(NW0 + 2, c) * S2;
      f4 W0 = v1t * S0, W1 = v1t * S1, W2 = v1t * S2;
      auto put = [&](float* d, f4 val) {
        if (ag) val += *reinterpret_cast<const f4*>(d);
        *reinterpret_cast<f4*>(d) = val;
      };
      put(P.gq + (size_t)t * P.ldq + 16 * h + 4 * g, Q);
      put(P.gk + (size_t)t * P.ldk + 16 * h + 4 * g, K);
      float* gvt = P.gv + (size_t)t * P.ldv + VL<PL>::head * h + 4 * g;
      put(gvt, VX);
      put(gvt + PV, V1);
      put(gvt + 2 * PV, V2);
      if (P.gveci) {
        if (resid) {
          W0 += own(NGV, c);
          W1 += own(NGV + 1, c);
          W2 += own(NGV + 2, c);
        }
        float* gw = P.gveci + (size_t)t * 3 * H + 16 * h + 4 * g;
        put(gw, W0);
        put(gw + H, W1);
        put(gw + 2 * H, W2);
      }
    }
  }
}

// ------------------------------------------------------------------ neighbour embedding, distance_proj fused
// Reference NeighborEmbedding (models/utils.py:90-108): x_nb[t] = sum_{e in row t, s != t} x[s] *
// (W f(r_e) + b) * C_e, W = distance_proj [H][R].  As the message kernels above: the projection of the
// per-pair RBF fragments on the fp16 MFMA (W the A operand from an LDS image of D = H rows), so neither
// the E x H rows W f + b nor, in the force pass, their gradient (E x H) and its E x R contraction with
// d f / d r exist in memory.  The force pass ("dr mode") needs only the edge gradients:
//   g_C[e] = sum_h gout[t][h] x[s][h] (W f + b)[h],  g_r[e] = C_e sum_h gout[t][h] x[s][h] (W f')[h].
// One work item = one node, all H = 128 channels (8 blocks of 16); a lane holds its edge's channels
// 16 blk + 4 g + i.  Self edges (s == t) contribute nothing (the reference's remove_self_loops).
constexpr int kNbD = kH;  // the image's rows: H output channels
struct NbF {
  int n, cap, chunk, acc;
  const int32_t* row_ptr;
  const int32_t* src;
  const float* x; int ldx;  // [N][H] the embedding rows
  const float* C;
  const int32_t* frow;
  const _Float16* fr;
  const float* dscale;
  unsigned fr_bytes;
  const _Float16* img;
  const float* wsc;
  const float* bias;
  float* out; int ldo;       // forward: x_nb rows (stride ldo)
  const float* xself;        // forward: optional [N][H] rows copied to oself (stride ldo)
  float* oself;
  const float* gout; int ldg;  // backward: dL / d x_nb rows
  float* gC;                   // backward: [cap] dL / d C
  float* gr;                   // backward: [cap] dL / d r
};

template <int KS, int NT>
__device__ __forceinline__ void load_image_nb(_Float16* w, float* s_sc, float* s_b, const NbF& P) {
  constexpr int R = 32 * KS;
  const u4* gi = reinterpret_cast<const u4*>(P.img);
  u4* l = reinterpret_cast<u4*>(w);
  for (int i = threadIdx.x; i < 2 * kNbD * R / 8; i += NT) l[i] = gi[i];
  for (int i = threadIdx.x; i < kNbD; i += NT) { s_sc[i] = P.wsc[i]; s_b[i] = P.bias[i]; }
}

// one 16-edge tile slot: source, cutoff (0 for self / past-the-row edges), fragment row offset
struct NbEdge {
  int s, fo;
  float C;
  bool ok, live;
};
__device__ __forceinline__ NbEdge nb_edge(int e, int re, int t, const NbF& P, int frow_bytes) {
  NbEdge E;
  E.ok = e < re;
  E.s = E.ok ? P.src[e] : 0;
  E.live = E.ok && E.s != t;
  E.fo = E.ok ? P.frow[e] * frow_bytes : kOOB;
  E.C = E.live ? P.C[e] : 0.f;
  return E;
}

template <int KS, int NW>
__global__ __launch_bounds__(NW * 64, 4) void k_nb_fwd(NbF P) {
  constexpr int R = 32 * KS, NB = kNbD / 16;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kNbD * R];
  __shared__ __attribute__((aligned(16))) float s_sc[kNbD];
  __shared__ __attribute__((aligned(16))) float s_b[kNbD];
  __shared__ int s_next;
  load_image_nb<KS, NW * 64>(w, s_sc, s_b, P);
  if (threadIdx.x == 0) s_next = 0;
  __syncthreads();
  const Work W = work_range<1>(P.n, P.chunk);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4;
  const rsrc_t Rx = make_rsrc(P.x, (unsigned)P.n * P.ldx * 4u), Rf = make_rsrc(P.fr, P.fr_bytes);
  const char* wt = reinterpret_cast<const char*>(w);
  for (;;) {
    const int it = next_item(&s_next);
    if (it >= W.items) break;
    int t, sl;
    if (!work_item<1>(W, it, t, sl)) continue;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    f4 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};
    NbEdge En = nb_edge(rb + c, re, t, P, 8 * R);
    for (int base = rb; base < re; base += 16) {
      const NbEdge E = En;
      if (base + 16 < re) En = nb_edge(base + 16 + c, re, t, P, 8 * R);
      h8 B0[KS], B1[KS];
      load_frags<KS>(Rf, E.fo, g, 0, B0, B1);
      const int ox = E.live ? (E.s * P.ldx + 4 * g) * 4 : kOOB;
      f4 xs[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) xs[b] = bld4<0>(Rx, ox, __builtin_amdgcn_readfirstlane(64 * b));
      int wb[KS];
      frag_offsets<KS>(lane, 0, wb);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const f4 pre = block_pre<KS, kNbD>(wt, wb, s_sc, s_b, b, B0, B1, g);
        acc[b] += xs[b] * pre * E.C;
      }
    }
    // the 16 edge slots; lane (g, c < NB) stores block c's channels 16 c + 4 g + i
    f4 o{};
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      f4 sb;
#pragma unroll
      for (int i = 0; i < 4; ++i) sb[i] = row_sum16(acc[b][i]);
      if (c == b) o = sb;
    }
    if (c < NB) {
      const int ch = 16 * c + 4 * g;
      *reinterpret_cast<f4*>(P.out + (size_t)t * P.ldo + ch) = o;
      if (P.xself)
        *reinterpret_cast<f4*>(P.oself + (size_t)t * P.ldo + ch) =
            *reinterpret_cast<const f4*>(P.xself + (size_t)t * kNbD + ch);
    }
  }
}

// the force pass's backward (dr mode): g_C and g_r per edge (written, or added with TMDNET_ACC_EDGE);
// static-capacity padding slots [row_ptr[n], cap) zeroed
template <int KS, int NW>
__global__ __launch_bounds__(NW * 64, 4) void k_nb_bwd(NbF P) {
  constexpr int R = 32 * KS, NB = kNbD / 16;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kNbD * R];
  __shared__ __attribute__((aligned(16))) float s_sc[kNbD];
  __shared__ __attribute__((aligned(16))) float s_b[kNbD];
  __shared__ __attribute__((aligned(16))) float s_go[NW][kNbD];  // gout[t] of the wave's node
  __shared__ int s_next;
  load_image_nb<KS, NW * 64>(w, s_sc, s_b, P);
  if (threadIdx.x == 0) s_next = 0;
  const bool acc_edge = P.acc & TMDNET_ACC_EDGE;
  if (!acc_edge) {
    const int e0 = min(P.row_ptr[P.n], P.cap);
    for (int e = e0 + blockIdx.x * NW * 64 + threadIdx.x; e < P.cap; e += gridDim.x * NW * 64) P.gC[e] = P.gr[e] = 0.f;
  }
  __syncthreads();
  const Work W = work_range<1>(P.n, P.chunk);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4;
  const rsrc_t Rx = make_rsrc(P.x, (unsigned)P.n * P.ldx * 4u), Rf = make_rsrc(P.fr, P.fr_bytes);
  const char* wt = reinterpret_cast<const char*>(w);
  for (;;) {
    const int it = next_item(&s_next);
    if (it >= W.items) break;
    int t, sl;
    if (!work_item<1>(W, it, t, sl)) continue;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    float* go = s_go[threadIdx.x >> 6];
    __builtin_amdgcn_wave_barrier();  // the previous node's reads are done (in-order LDS)
    if (lane < kNbD / 4)
      *reinterpret_cast<f4*>(go + 4 * lane) = *reinterpret_cast<const f4*>(P.gout + (size_t)t * P.ldg + 4 * lane);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    NbEdge En = nb_edge(rb + c, re, t, P, 8 * R);
    for (int base = rb; base < re; base += 16) {
      const int e = base + c;
      const NbEdge E = En;
      if (base + 16 < re) En = nb_edge(base + 16 + c, re, t, P, 8 * R);
      h8 B0[KS], B1[KS], D0[KS], D1[KS];
      load_frags<KS>(Rf, E.fo, g, 0, B0, B1);
      load_frags<KS>(Rf, E.fo, g, 1, D0, D1);
      const float dsc = E.ok ? P.dscale[E.fo / (8 * R)] : 1.f;
      const int ox = E.live ? (E.s * P.ldx + 4 * g) * 4 : kOOB;
      f4 xs[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) xs[b] = bld4<0>(Rx, ox, __builtin_amdgcn_readfirstlane(64 * b));
      int wb[KS];
      frag_offsets<KS>(lane, 0, wb);
      float gc = 0.f, gd = 0.f;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        f4 pre, dpre;
        block_pre_dpre<KS, kNbD>(wt, wb, s_sc, s_b, dsc, b, B0, B1, D0, D1, g, pre, dpre);
        const f4 gx = *reinterpret_cast<const f4*>(go + 16 * b + 4 * g) * xs[b];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gc = fmaf(gx[i], pre[i], gc);
          gd = fmaf(gx[i], dpre[i], gd);
        }
      }
      gc = gsum(gc);
      gd = gsum(gd) * E.C;
      if (g == 0 && E.ok) {
        if (!E.live) gc = gd = 0.f;
        if (acc_edge) {
          P.gC[e] += gc;
          P.gr[e] += gd;
        } else {
          P.gC[e] = gc;
          P.gr[e] = gd;
        }
      }
    }
  }
}

static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

// nodes per scheduling chunk (work_range); TMDNET_FEP_CHUNK overrides (A/B)
static int chunk_nodes() {
  static int c = [] {
    const char* e = getenv("TMDNET_FEP_CHUNK");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 2;
  }();
  return c;
}

// launch-form A/B switches (measured on C5, tools/fep_time.py; one workgroup per CU, no variant spills):
// TMDNET_FEP_FWD_FORM 1 = the round-4 first form, 2 heads per item on 12 waves (1.46 ms vs 1.34 ms for the
// default 4 heads on 8 waves); TMDNET_FEP_DST_FORM 1 = 4 heads on 4 waves (3.78 vs 3.42 ms per backward);
// TMDNET_FEP_SRC_FORM 1 = 2 heads on 12 waves (3.43 vs 3.38).  Measured and dropped: 1 head on 16 waves
// (fwd 1.78, src 3.64), 8 heads on 4 waves (fwd 1.65, dst 3.67, src 4.16), the one-tile-ahead edge
// prefetch with both heads' gathers issued first on 8 waves (fwd 1.51 vs 1.46 at 2 heads).
// Round 5 (default 2 for both): head-pipelined gathers (HP = 1: head hh + 1's issued before head hh
// computes) fwd 1.340 -> 1.313 ms, backward 3.346 -> 3.329; across tiles too (HP = 2, form 3) fwd 2.74
// (79 spilled VGPRs) / 2 heads per item (form 4) 1.51; dst form 3 (HP = 2, 2 spills) 3.367.
static int fwd_form() {
  static int f = [] {
    const char* e = getenv("TMDNET_FEP_FWD_FORM");
    return e ? atoi(e) : 2;
  }();
  return f;
}


static int bwd_form(int which) {
  static int f[2] = {[] {
                       const char* e = getenv("TMDNET_FEP_DST_FORM");
                       return e ? atoi(e) : 2;
                     }(),
                     [] {
                       const char* e = getenv("TMDNET_FEP_SRC_FORM");
                       return e ? atoi(e) : 0;
                     }()};
  return f[which];
}
static int dst_hpw();
// TMDNET_FEP_ROW=1: the merged row pass (k_bwd_row, one head per item on 8 waves) instead of the two
// passes.  Measured at C5 (tools/fep_time.py, ms per backward): two passes 3.38; merged, 1 head on 8
// waves 3.83 (no spills), 2 heads on 4 waves 4.08, 2 heads on 8 waves 4.33 (45 spilled VGPRs).  The
// merged pass forms the projection once instead of twice but issues 12 gathers per (edge, head) back to
// back: both passes are bound by the per-wave latency chain at 2 waves per SIMD, not by the MFMA work
// the merge removes.
static bool row_pass() {
  static bool r = [] {
    const char* e = getenv("TMDNET_FEP_ROW");
    return e && atoi(e) == 1;
  }();
  return r;
}

// launch shapes (heads per work item, waves per workgroup; one workgroup per CU): chosen so that no
// variant spills (tools/regs.py) -- see the launchers
constexpr int kFwdHPW = 4, kFwdNW = 8;
constexpr int kDstHPW = 2, kDstNW = 8;  // 12 waves: 6-14 spilled VGPRs
constexpr int kSrcHPW = 4, kSrcNW = 8;
static int dst_hpw() {
  if (row_pass()) return 1;
  const int f = bwd_form(0);
  return f == 1 ? 4 : kDstHPW;
}

}  // namespace fep
}  // namespace tmd

using namespace tmd;

extern "C" size_t tmdnet_fep_image_bytes(int D, int R) { return (size_t)2 * D * R * sizeof(_Float16); }

extern "C" int tmdnet_fep_split_f32(int D, int R, const void* W, int ldw, const void* bias, void* img, void* wsc,
                                    void* bias_out, void* stream) {
  if (D <= 0 || !W || !img || !wsc || !bias_out) return kBadArgument;
  if ((R != 32 && R != 64) || ldw < R) return kUnsupported;
  const dim3 g((D + 255) / 256), b(256);
  hipStream_t st = (hipStream_t)stream;
  if (R == 64)
    hipLaunchKernelGGL(fep::k_split<2>, g, b, 0, st, D, (const float*)W, ldw, (const float*)bias, (_Float16*)img,
                       (float*)wsc, (float*)bias_out);
  else
    hipLaunchKernelGGL(fep::k_split<1>, g, b, 0, st, D, (const float*)W, ldw, (const float*)bias, (_Float16*)img,
                       (float*)wsc, (float*)bias_out);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" size_t tmdnet_fep_frags_bytes(long long rows, int R) {
  return rows < 0 ? 0 : (size_t)rows * 4 * R * sizeof(_Float16);
}

extern "C" int tmdnet_fep_frags_f32(long long rows, int R, const void* r_rows, const void* mu, const void* beta,
                                    double cutoff_lower, double cutoff_upper, int rbf_type, void* frags, void* dscale,
                                    void* stream) {
  if (rows < 0 || (rows && (!r_rows || !mu || !beta || !frags || !dscale))) return kBadArgument;
  if (R != 32 && R != 64) return kUnsupported;
  if (rows == 0) return kOk;
  const float cl = (float)cutoff_lower, cu = (float)cutoff_upper, alpha = (float)(5.0 / (cutoff_upper - cutoff_lower));
  const long long per = 256 / R;
  const dim3 g((unsigned)((rows + per - 1) / per)), b(256);
  hipStream_t st = (hipStream_t)stream;
  if (R == 64)
    hipLaunchKernelGGL(fep::k_frags<2>, g, b, 0, st, rows, (const float*)r_rows, (const float*)mu, (const float*)beta,
                       rbf_type, cl, cu, alpha, (_Float16*)frags, (float*)dscale);
  else
    hipLaunchKernelGGL(fep::k_frags<1>, g, b, 0, st, rows, (const float*)r_rows, (const float*)mu, (const float*)beta,
                       rbf_type, cl, cu, alpha, (_Float16*)frags, (float*)dscale);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

namespace {
// the shape / layout checks shared by the fused entry points
int fused_check(int n, int H, int heads, int R, int ldq, int ldk, int ldv, const void* q, const void* k, const void* v,
                const void* vec, const void* img, long long frag_rows) {
  if (H != fep::kH || heads != fep::kHeads || (R != 32 && R != 64)) return kUnsupported;
  if (ldq < H || ldk < H || ldv < 3 * H || ldq % 4 || ldk % 4 || ldv % 4) return kBadArgument;
  if ((((uintptr_t)q) | ((uintptr_t)k) | ((uintptr_t)v) | ((uintptr_t)vec) | ((uintptr_t)img)) & 15) return kUnsupported;
  // the gathers address rows through 32-bit byte offsets
  if ((long long)n * (ldq > ldv ? ldq : ldv) * 4 >= fep::kOOB || (long long)n * 3 * H * 4 >= fep::kOOB ||
      frag_rows * 8 * R >= fep::kOOB)
    return kUnsupported;
  return kOk;
}
}  // namespace

extern "C" int tmdnet_et_fused_fwd_f32(int n, int H, int heads, int R, const int32_t* row_ptr, const int32_t* src,
                                       int cap, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                       const void* vec, const void* C, const void* u, const int32_t* frag_rows,
                                       const void* frags, long long n_frag_rows, const void* img, const void* wsc,
                                       const void* bias, void* x_out, void* vec_out, int flags, void* stream) {
  if (n < 0 || !row_ptr || !src || !q || !k || !v || !C || !u || !frag_rows || !frags || !img || !wsc || !bias ||
      !x_out || !vec_out)
    return kBadArgument;
  if (n == 0) return kOk;
  int rc = fused_check(n, H, heads, R, ldq, ldk, ldv, q, k, v, vec, img, n_frag_rows);
  if (rc) return rc;
  if ((((uintptr_t)x_out) | ((uintptr_t)vec_out) | ((uintptr_t)frags)) & 15) return kUnsupported;
  fep::Fwd P{};
  P.n = n; P.cap = cap; P.chunk = fep::chunk_nodes();
  P.row_ptr = row_ptr; P.src = src;
  P.q = (const float*)q; P.ldq = ldq; P.k = (const float*)k; P.ldk = ldk; P.v = (const float*)v; P.ldv = ldv;
  P.vec = (const float*)vec; P.C = (const float*)C; P.u = (const float*)u;
  P.frow = frag_rows; P.fr = (const _Float16*)frags; P.fr_bytes = (unsigned)(n_frag_rows * 8 * R);
  P.img = (const _Float16*)img; P.wsc = (const float*)wsc; P.bias = (const float*)bias;
  P.xo = (float*)x_out; P.veco = (float*)vec_out;
  const int nwg = fep::num_cus();
  const bool pl = flags & TMDNET_ET_V_PLANAR;
  hipStream_t st = (hipStream_t)stream;
  constexpr int NW = fep::kFwdNW, HPW = fep::kFwdHPW;
#define TMD_FEP(KS_, PL_)                                                                                  \
  do {                                                                                                     \
    if (fep::fwd_form() == 1)                                                                              \
      hipLaunchKernelGGL((fep::k_fwd<KS_, 2, 12, PL_>), dim3(nwg), dim3(12 * 64), 0, st, P);                \
    else if (fep::fwd_form() == 2)                                                                         \
      hipLaunchKernelGGL((fep::k_fwd<KS_, HPW, NW, PL_, 1>), dim3(nwg), dim3(NW * 64), 0, st, P);           \
    else if (fep::fwd_form() == 3)                                                                         \
      hipLaunchKernelGGL((fep::k_fwd<KS_, HPW, NW, PL_, 2>), dim3(nwg), dim3(NW * 64), 0, st, P);           \
    else if (fep::fwd_form() == 4)                                                                         \
      hipLaunchKernelGGL((fep::k_fwd<KS_, 2, NW, PL_, 2>), dim3(nwg), dim3(NW * 64), 0, st, P);             \
    else                                                                                                   \
      hipLaunchKernelGGL((fep::k_fwd<KS_, HPW, NW, PL_>), dim3(nwg), dim3(NW * 64), 0, st, P);              \
  } while (0)
  if (R == 64) {
    if (pl) TMD_FEP(2, true); else TMD_FEP(2, false);
  } else {
    if (pl) TMD_FEP(1, true); else TMD_FEP(1, false);
  }
#undef TMD_FEP
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" size_t tmdnet_et_fused_bwd_workspace_bytes(int cap) {
  const int S = fep::kHeads / fep::dst_hpw();
  return S > 1 && cap > 0 ? (size_t)S * 5 * cap * sizeof(float) : 0;
}

extern "C" int tmdnet_et_fused_bwd_f32(int n, int H, int heads, int R, const int32_t* row_ptr, const int32_t* src,
                                       int cap, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                       const void* vec, const void* C, const void* u, const int32_t* frag_rows,
                                       const void* frags, const void* dscale, long long n_frag_rows, const void* img,
                                       const void* wsc, const void* bias, const void* gx, const void* gvec, void* gq,
                                       void* gk, void* gv, void* gvec_in, void* gC, void* gu, void* gdist,
                                       int accumulate, void* workspace, size_t workspace_bytes, void* stream) {
  if (n < 0 || !row_ptr || !src || !q || !k || !v || !C || !u || !frag_rows || !frags || !dscale || !img || !wsc ||
      !bias || !gx || !gvec || !gq || !gk || !gv || !gC || !gu || !gdist)
    return kBadArgument;
  if (n == 0) return kOk;
  int rc = fused_check(n, H, heads, R, ldq, ldk, ldv, q, k, v, vec, img, n_frag_rows);
  if (rc) return rc;
  if ((((uintptr_t)gx) | ((uintptr_t)gvec) | ((uintptr_t)gq) | ((uintptr_t)gk) | ((uintptr_t)gv) |
       ((uintptr_t)gvec_in) | ((uintptr_t)frags)) & 15)
    return kUnsupported;
  const size_t need = tmdnet_et_fused_bwd_workspace_bytes(cap);
  if (need && (!workspace || workspace_bytes < need)) return kWorkspaceTooSmall;
  fep::Bwd P{};
  P.n = n; P.cap = cap; P.acc = accumulate; P.chunk = fep::chunk_nodes();
  P.row_ptr = row_ptr; P.src = src;
  P.q = (const float*)q; P.ldq = ldq; P.k = (const float*)k; P.ldk = ldk; P.v = (const float*)v; P.ldv = ldv;
  P.vec = (const float*)vec; P.C = (const float*)C; P.u = (const float*)u;
  P.frow = frag_rows; P.fr = (const _Float16*)frags; P.dscale = (const float*)dscale;
  P.fr_bytes = (unsigned)(n_frag_rows * 8 * R);
  P.img = (const _Float16*)img; P.wsc = (const float*)wsc; P.bias = (const float*)bias;
  P.gx = (const float*)gx; P.gvec = (const float*)gvec;
  P.gq = (float*)gq; P.gk = (float*)gk; P.gv = (float*)gv; P.gveci = (float*)gvec_in;
  P.gC = (float*)gC; P.gu = (float*)gu; P.gr = (float*)gdist;
  P.part = (float*)workspace;
  const int nwg = fep::num_cus();
  const int S = fep::kHeads / fep::dst_hpw();
  const bool pl = accumulate & TMDNET_ET_V_PLANAR;
  hipStream_t st = (hipStream_t)stream;
  const int dform = fep::bwd_form(0), sform = fep::bwd_form(1);
#define TMD_DST(KS_, PL_, HPW_, NW_) \
  hipLaunchKernelGGL((fep::k_bwd_dst<KS_, HPW_, NW_, PL_>), dim3(nwg), dim3(NW_ * 64), 0, st, P)
#define TMD_SRC(KS_, PL_, HPW_, NW_) \
  hipLaunchKernelGGL((fep::k_bwd_src<KS_, HPW_, NW_, PL_>), dim3(nwg), dim3(NW_ * 64), 0, st, P)
#define TMD_ROW(KS_, PL_, HPW_, NW_) \
  hipLaunchKernelGGL((fep::k_bwd_row<KS_, HPW_, NW_, PL_>), dim3(nwg), dim3(NW_ * 64), 0, st, P)
#define TMD_BWD(KS_, PL_)                                                                                          \
  do {                                                                                                             \
    if (fep::row_pass()) {                                                                                         \
      TMD_ROW(KS_, PL_, 1, 8);                                                                                     \
      if (S > 1) hipLaunchKernelGGL(fep::k_edge_combine, dim3((cap + 255) / 256), dim3(256), 0, st, P, S);         \
      break;                                                                                                       \
    }                                                                                                              \
    if (dform == 1) TMD_DST(KS_, PL_, 4, 4);                                                                        \
    else if (dform == 2 || dform == 3) {                                                                           \
      if (dform == 2)                                                                                              \
        hipLaunchKernelGGL((fep::k_bwd_dst<KS_, fep::kDstHPW, fep::kDstNW, PL_, 1>), dim3(nwg),                    \
                           dim3(fep::kDstNW * 64), 0, st, P);                                                      \
      else                                                                                                         \
        hipLaunchKernelGGL((fep::k_bwd_dst<KS_, fep::kDstHPW, fep::kDstNW, PL_, 2>), dim3(nwg),                    \
                           dim3(fep::kDstNW * 64), 0, st, P);                                                      \
    }                                                                                                              \
    else TMD_DST(KS_, PL_, fep::kDstHPW, fep::kDstNW);                                                              \
    if (S > 1) hipLaunchKernelGGL(fep::k_edge_combine, dim3((cap + 255) / 256), dim3(256), 0, st, P, S);           \
    if (sform == 1) TMD_SRC(KS_, PL_, 2, 12);                                                                       \
    else TMD_SRC(KS_, PL_, fep::kSrcHPW, fep::kSrcNW);                                                              \
  } while (0)
  if (R == 64) {
    if (pl) TMD_BWD(2, true); else TMD_BWD(2, false);
  } else {
    if (pl) TMD_BWD(1, true); else TMD_BWD(1, false);
  }
#undef TMD_BWD
#undef TMD_ROW
#undef TMD_DST
#undef TMD_SRC
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// ---- the fused neighbour embedding (reference NeighborEmbedding, models/utils.py:90-108)
namespace {
constexpr int kNbNW = 8;  // waves per workgroup; two workgroups per CU (32 KB image, <= 128 VGPRs)
int nb_check(int n, int H, int R, const void* x, int ld_x, const void* img, long long frag_rows) {
  if (H != fep::kNbD || (R != 32 && R != 64)) return kUnsupported;
  if (ld_x < H || ld_x % 4) return kBadArgument;
  if ((((uintptr_t)x) | ((uintptr_t)img)) & 15) return kUnsupported;
  if ((long long)n * ld_x * 4 >= fep::kOOB || frag_rows * 8 * R >= fep::kOOB) return kUnsupported;
  return kOk;
}
}  // namespace

extern "C" int tmdnet_nbr_fused_fwd_f32(int n, int H, int R, const int32_t* row_ptr, const int32_t* src, int cap,
                                        const void* x, int ld_x, const void* C, const int32_t* frag_rows,
                                        const void* frags, long long n_frag_rows, const void* img, const void* wsc,
                                        const void* bias, void* out, int ld_out, const void* x_self, void* out_self,
                                        void* stream) {
  if (n < 0 || !row_ptr || !src || !x || !C || !frag_rows || !frags || !img || !wsc || !bias || !out)
    return kBadArgument;
  if ((x_self == nullptr) != (out_self == nullptr)) return kBadArgument;
  if (n == 0) return kOk;
  int rc = nb_check(n, H, R, x, ld_x, img, n_frag_rows);
  if (rc) return rc;
  if (ld_out < H || ld_out % 4 || ((((uintptr_t)out) | ((uintptr_t)out_self) | ((uintptr_t)x_self) |
                                    ((uintptr_t)frags)) & 15))
    return kUnsupported;
  fep::NbF P{};
  P.n = n; P.cap = cap; P.chunk = fep::chunk_nodes();
  P.row_ptr = row_ptr; P.src = src; P.x = (const float*)x; P.ldx = ld_x; P.C = (const float*)C;
  P.frow = frag_rows; P.fr = (const _Float16*)frags; P.fr_bytes = (unsigned)(n_frag_rows * 8 * R);
  P.img = (const _Float16*)img; P.wsc = (const float*)wsc; P.bias = (const float*)bias;
  P.out = (float*)out; P.ldo = ld_out; P.xself = (const float*)x_self; P.oself = (float*)out_self;
  const dim3 g(2 * fep::num_cus()), b(kNbNW * 64);
  hipStream_t st = (hipStream_t)stream;
  if (R == 64) hipLaunchKernelGGL((fep::k_nb_fwd<2, kNbNW>), g, b, 0, st, P);
  else hipLaunchKernelGGL((fep::k_nb_fwd<1, kNbNW>), g, b, 0, st, P);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_nbr_fused_bwd_f32(int n, int H, int R, const int32_t* row_ptr, const int32_t* src, int cap,
                                        const void* x, int ld_x, const void* C, const int32_t* frag_rows,
                                        const void* frags, const void* dscale, long long n_frag_rows,
                                        const void* img, const void* wsc, const void* bias, const void* grad_out,
                                        int ld_grad_out, void* gcut, void* gdist, int accumulate, void* stream) {
  if (n < 0 || !row_ptr || !src || !x || !C || !frag_rows || !frags || !dscale || !img || !wsc || !bias ||
      !grad_out || !gcut || !gdist)
    return kBadArgument;
  if (n == 0) return kOk;
  int rc = nb_check(n, H, R, x, ld_x, img, n_frag_rows);
  if (rc) return rc;
  if (ld_grad_out < H || ld_grad_out % 4 || ((((uintptr_t)grad_out) | ((uintptr_t)frags)) & 15)) return kUnsupported;
  fep::NbF P{};
  P.n = n; P.cap = cap; P.chunk = fep::chunk_nodes(); P.acc = accumulate;
  P.row_ptr = row_ptr; P.src = src; P.x = (const float*)x; P.ldx = ld_x; P.C = (const float*)C;
  P.frow = frag_rows; P.fr = (const _Float16*)frags; P.dscale = (const float*)dscale;
  P.fr_bytes = (unsigned)(n_frag_rows * 8 * R);
  P.img = (const _Float16*)img; P.wsc = (const float*)wsc; P.bias = (const float*)bias;
  P.gout = (const float*)grad_out; P.ldg = ld_grad_out; P.gC = (float*)gcut; P.gr = (float*)gdist;
  const dim3 g(2 * fep::num_cus()), b(kNbNW * 64);
  hipStream_t st = (hipStream_t)stream;
  if (R == 64) hipLaunchKernelGGL((fep::k_nb_bwd<2, kNbNW>), g, b, 0, st, P);
  else hipLaunchKernelGGL((fep::k_nb_bwd<1, kNbNW>), g, b, 0, st, P);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
