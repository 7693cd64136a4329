// Equivariant-Transformer message with the dk/dv projection FUSED into the edge kernel ("FEP"), for
// large graphs (the C5 water box: ~2.7 M edges).
//
// Reference: EquivariantMultiHeadAttention dk_proj / dv_proj (models/torchmd_et.py:282-291),
// message / aggregate (:314-347); the RBF it projects, ExpNormalSmearing / GaussianSmearing
// (models/utils.py:272-344).
//
// The unfused path writes the projection rows of every edge pair (2 KB per row at H = 128, 2.8 GB per
// layer at C5) and the message kernel reads them back once per DIRECTION (the two edges of a pair sit
// in different destination rows, far apart in time): HBM-bound on 2.4x its distinct bytes.  Here the
// projection never leaves the chip: per 16-edge tile the kernel evaluates the RBF of the 16 distances
// in registers, multiplies it by the layer's [dk | dv] weight (held in LDS for the whole launch) on the
// fp16 MFMA, applies SiLU and consumes the result in the message math straight from the accumulator
// registers.  What remains in memory is the edge stream (src, r, C, unit vector: 24 B per edge) and the
// source-row gathers of k / v / vec (L2 / Infinity-Cache resident for spatially ordered atoms).
//
// Accuracy: fp32-GEMM level without the fp32 MFMA (1/16 of the fp16 rate).  Both operands are split
// into two fp16 pieces, x = x0 + 2^-? x1 (x0 = fp16(x), x1 = fp16(x - x0), exact difference), after an
// exact power-of-two scaling (the weight per output row to max |w| < 2^14, the RBF values -- all in
// [0, 1] -- by 2^14); the three products x0 y0 + x0 y1 + x1 y0 are exact in the fp32 accumulator and
// the dropped x1 y1 and the split residuals are ~2^-22 relative -- below fp32 GEMM rounding at K = 64.
//
// MFMA roles (v_mfma_f32_16x16x32_f16): the A operand is the RBF tile (16 edges x 32 k), the B operand
// a 16-row block of W (16 output channels x 32 k), so a lane's four accumulator values are FOUR EDGES
// (4 (lane >> 4) + i) of ONE channel (lane & 15).  With d = H / heads = 16 a column block is exactly
// one head: the q.k.dk head sum is a 16-lane row sum (4 DPP adds), and the aggregation into the
// destination accumulates in registers (one value per lane and block: 32 accumulators), reduced over
// the four lane groups once per node.
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
constexpr int kHeads = 8;           // d = 16: one MFMA column block per head

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
  const int s = m > 0.f ? 14 - ex : 0;
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

struct Fwd {
  int n, cap, rbf;
  const int32_t* row_ptr;
  const int32_t* src;
  const float* q; int ldq;
  const float* k; int ldk;
  const float* v; int ldv;  // planar [x | v1 | v2] H-blocks
  const float* vec;         // [N][3][H] or NULL (layer 0)
  const float* r;
  const float* C;
  const float* u;
  const _Float16* img;
  const float* wsc;
  const float* bias;
  const float* mu;
  const float* beta;
  float cl, cu, alpha;
  float* xo;
  float* veco;
  float* pkv;           // optional: the pre-activation projection rows of the canonical edges (src >= dst)
  int ldp;              // written to row prow[e] (the pair rows a later unfused backward reads); NULL: none
  const int32_t* prow;
  unsigned pbytes;      // the rows' extent in bytes (the store resource's range: no write lands outside)
};

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

// Source-row gathers through buffer resources: per edge one 32-bit byte offset (row start + channel),
// per head / part a constant added as the instruction's immediate offset -- no 64-bit address per
// (head, part, edge).  vec absent (layer 0): a zero-size resource, whose loads return 0.
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld(rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
constexpr int kOOB = 0x7FFFFF00;  // a byte offset past every resource's range (buffer loads return 0)
struct Gat {
  float kk[4], vx[4], v1[4], v2[4], w0[4], w1[4], w2[4];
};
struct Src {
  rsrc_t q, k, v, vec;
  int ok[4], ov[4], ow[4];  // byte offsets of the lane's channel in the four source rows
};
// head h's values (byte offset 64 h: 16 channels of 4 bytes; v / vec parts H * 4 = 512 bytes apart)
template <int HB>
__device__ __forceinline__ void gather(Gat& G, const Src& S) {
  constexpr int PB = kH * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    G.kk[i] = bld(S.k, S.ok[i] + HB);
    G.vx[i] = bld(S.v, S.ov[i] + HB);
    G.v1[i] = bld(S.v, S.ov[i] + HB + PB);
    G.v2[i] = bld(S.v, S.ov[i] + HB + 2 * PB);
    G.w0[i] = bld(S.vec, S.ow[i] + HB);
    G.w1[i] = bld(S.vec, S.ow[i] + HB + PB);
    G.w2[i] = bld(S.vec, S.ow[i] + HB + 2 * PB);
  }
}

// RBF value k at distance r (the edge-geometry kernel's formula, edge_geom.hip basis())
__device__ __forceinline__ float rbf_value(int type, float r, float cut0, float ue, float mu, float beta) {
  if (type == TMDNET_RBF_EXPNORM) {
    const float z = ue - mu;
    return cut0 * expf(-beta * z * z);
  }
  const float z = r - mu;
  return expf(beta * z * z);
}

// Byte offset in the weight image of the lane's fragment for k-step ks of block 0, piece 0: lane l
// reads row (l & 15) + 16 blk, chunk swz(row, (l >> 4) + 4 ks) -- the swizzle depends on row & 7 (KS = 2)
// or (row >> 1) & 3 (KS = 1) only, so block and piece add CONSTANT offsets (ds_read immediates).
template <int KS>
__device__ __forceinline__ int wfrag_base(int lane, int ks) {
  constexpr int R = 32 * KS;
  const int row = lane & 15;
  return (row * R + swz<KS>(row, (lane >> 4) + 4 * ks) * 8) * (int)sizeof(_Float16);
}

template <int I> struct IC { static constexpr int value = I; };
template <int N, int I = 0, typename F> __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<N, I + 1>(f);
  }
}

__device__ __forceinline__ void gather_dyn(Gat& G, const Src& S, int hb) {
  constexpr int PB = kH * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    G.kk[i] = bld(S.k, S.ok[i] + hb);
    G.vx[i] = bld(S.v, S.ov[i] + hb);
    G.v1[i] = bld(S.v, S.ov[i] + hb + PB);
    G.v2[i] = bld(S.v, S.ov[i] + hb + 2 * PB);
    G.w0[i] = bld(S.vec, S.ow[i] + hb);
    G.w1[i] = bld(S.vec, S.ow[i] + hb + PB);
    G.w2[i] = bld(S.vec, S.ow[i] + hb + 2 * PB);
  }
}

// head values with the head's byte offset in an SGPR (the instruction's soffset): no per-load VALU add
__device__ __forceinline__ float blds(rsrc_t r, int off, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0));
}
__device__ __forceinline__ void gather_s(Gat& G, const Src& S, int soff) {
  constexpr int PB = kH * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    G.kk[i] = blds(S.k, S.ok[i], soff);
    G.vx[i] = blds(S.v, S.ov[i], soff);
    G.v1[i] = blds(S.v, S.ov[i] + PB, soff);
    G.v2[i] = blds(S.v, S.ov[i] + 2 * PB, soff);
    G.w0[i] = blds(S.vec, S.ow[i], soff);
    G.w1[i] = blds(S.vec, S.ow[i] + PB, soff);
    G.w2[i] = blds(S.vec, S.ow[i] + 2 * PB, soff);
  }
}
template <int K, int N> __device__ __forceinline__ void rotate_by(float (&a)[N]) {
  float t[K];
#pragma unroll
  for (int i = 0; i < K; ++i) t[i] = a[i];
#pragma unroll
  for (int i = 0; i + K < N; ++i) a[i] = a[i + K];
#pragma unroll
  for (int i = 0; i < K; ++i) a[N - K + i] = t[i];
}

template <int N> __device__ __forceinline__ void rotate(float (&a)[N]) {
  const float f = a[0];
#pragma unroll
  for (int i = 0; i + 1 < N; ++i) a[i] = a[i + 1];
  a[N - 1] = f;
}

// one 16-row block of the tile's pre-activations: acc[i] = pre(edge 4 (lane >> 4) + i, channel lane & 15).
// wb[p][ks]: the lane's fragment byte offsets (wfrag_base) of piece p, already including the image base.
template <int KS>
__device__ __forceinline__ f4 block_pre(const char* wl, const int (&wb)[KS], const float* sc, const float* sb,
                                        int blk, const h8 (&a0)[KS], const h8 (&a1)[KS], int lane) {
  constexpr int R = 32 * KS, PB = kD * R * (int)sizeof(_Float16);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const char* f0 = wl + wb[ks] + blk * 16 * R * (int)sizeof(_Float16);
    const h8 w0 = *reinterpret_cast<const h8*>(f0);
    const h8 w1 = *reinterpret_cast<const h8*>(f0 + PB);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[ks], w0, acc, 0, 0, 0);  // small terms first
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[ks], w1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[ks], w0, acc, 0, 0, 0);
  }
  const int ch = 16 * blk + (lane & 15);
  const float s = sc[ch], b = sb[ch];
  f4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = acc[i] * s + b;
  return o;
}

// one head of a tile: the four projection blocks (dk, dv x / v1 / v2) on the MFMA, then the message
template <int KS>
__device__ __forceinline__ void head_math(const Gat& X, const char* wt, const int (&wb)[KS], const float* sct,
                                          const float* sbt, int h, const h8 (&A0)[KS], const h8 (&A1)[KS], int lane,
                                          float qh, const float (&Ce)[4], const float (&ux)[4], const float (&uy)[4],
                                          const float (&uz)[4], float& ax, float& a0, float& a1,
                                          float& a2, const rsrc_t* Rp = nullptr, const int* op = nullptr) {
  const f4 pk = block_pre<KS>(wt, wb, sct, sbt, h, A0, A1, lane);
  const f4 px = block_pre<KS>(wt, wb, sct, sbt, 8 + h, A0, A1, lane);
  const f4 p1 = block_pre<KS>(wt, wb, sct, sbt, 16 + h, A0, A1, lane);
  const f4 p2 = block_pre<KS>(wt, wb, sct, sbt, 24 + h, A0, A1, lane);
  if (Rp) {  // the canonical edges' projection rows (column 16 blk + channel; other edges: out of range)
    // (the element goes through a scalar first: __builtin_bit_cast of a vector-element lvalue reads
    // element 0 whatever the index -- every edge of a lane group stored edge 0's row)
    const f4 pb[4] = {pk, px, p1, p2};
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float val = pb[b][i];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(val), *Rp, op[i] + 64 * (8 * b + h), 0, 0);
      }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float dk = Silu<float>(pk[i]).s;
    const float att = row_sum16(qh * X.kk[i] * dk);
    const float a = Silu<float>(att).s * Ce[i];
    ax += X.vx[i] * Silu<float>(px[i]).s * a;
    const float v1e = X.v1[i] * Silu<float>(p1[i]).s;
    const float v2e = X.v2[i] * Silu<float>(p2[i]).s;
    a0 += X.w0[i] * v1e + v2e * ux[i];
    a1 += X.w1[i] * v1e + v2e * uy[i];
    a2 += X.w2[i] * v1e + v2e * uz[i];
  }
}

// MODE 0: heads unrolled (static register indices, next head's gathers in flight); MODE 1: a rolled
// head loop whose per-head registers rotate into slot 0 (fewer live registers, two waves per SIMD)
template <int KS, int NW, int MODE, bool ROWS = false>
__global__ __launch_bounds__(NW * 64, 1) void k_fwd(Fwd P) {
  constexpr int R = 32 * KS, H = kH;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ float s_sc[kD], s_b[kD], s_mu[R], s_beta[R];
  __shared__ int s_next;
  {
    const u4* g = reinterpret_cast<const u4*>(P.img);
    u4* l = reinterpret_cast<u4*>(w);
    for (int i = threadIdx.x; i < 2 * kD * R / 8; i += NW * 64) l[i] = g[i];
    for (int i = threadIdx.x; i < kD; i += NW * 64) { s_sc[i] = P.wsc[i]; s_b[i] = P.bias[i]; }
    for (int i = threadIdx.x; i < R; i += NW * 64) {
      s_mu[i] = P.mu[i];
      s_beta[i] = P.rbf == TMDNET_RBF_EXPNORM ? P.beta[i] : P.beta[0];
    }
    if (threadIdx.x == 0) s_next = 0;
  }
  __syncthreads();
  // this workgroup's contiguous node range (XCD-contiguous: neighbouring ranges share an L2); its
  // waves take the nodes one at a time from an LDS counter
  const int nwg = gridDim.x, lb = xcd_remap(blockIdx.x, nwg);
  const int per = (P.n + nwg - 1) / nwg;
  const int n0 = lb * per, n1 = min(P.n, n0 + per);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4;
  Src S;
  S.q = make_rsrc(P.q, (unsigned)P.n * P.ldq * 4u);
  S.k = make_rsrc(P.k, (unsigned)P.n * P.ldk * 4u);
  S.v = make_rsrc(P.v, (unsigned)P.n * P.ldv * 4u);
  S.vec = make_rsrc(P.vec, P.vec ? (unsigned)P.n * 3u * H * 4u : 0u);
  const rsrc_t Rp = make_rsrc(P.pkv, P.pkv ? P.pbytes : 0u);
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(&s_next, 1);
    t = __builtin_amdgcn_readfirstlane(__shfl(t, 0)) + n0;
    if (t >= n1) break;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    const int oq = (t * P.ldq + c) * 4;
    float qh[kHeads], ax[kHeads], a0[kHeads], a1[kHeads], a2[kHeads];
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      qh[h] = P.q[(size_t)t * P.ldq + 16 * h + c];
      ax[h] = a0[h] = a1[h] = a2[h] = 0.f;
    }
    for (int base = rb; base < re; base += 16) {
      // the RBF tile: lane computes edge base + c, k = 32 ks + 8 g + j, split into two fp16 pieces
      h8 A0[KS], A1[KS];
      {
        const int ef = base + c;
        const bool vf = ef < re;
        const float rf = vf ? P.r[ef] : 0.f;
        const float cut0 = rf < P.cu ? 0.5f * (cosf(rf * 3.14159265358979323846f / P.cu) + 1.f) : 0.f;
        const float ue = expf(P.alpha * (P.cl - rf));
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int kk = 32 * ks + 8 * g + j;
            const float f = vf ? rbf_value(P.rbf, rf, cut0, ue, s_mu[kk], s_beta[kk]) : 0.f;
            const float x = f * kFScale;
            const _Float16 hi = (_Float16)x;
            A0[ks][j] = hi;
            A1[ks][j] = (_Float16)(x - (float)hi);
          }
      }
      // the lane's four output edges (base + 4 g + i): source, cutoff, unit vector (0 past the row)
      int s[4], op[4];
      float Ce[4], ux[4], uy[4], uz[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + 4 * g + i;
        const bool ok = e < re;
        s[i] = ok ? P.src[e] : 0;
        if constexpr (ROWS) op[i] = (ok && s[i] >= t) ? (P.prow[e] * P.ldp + c) * 4 : kOOB;
        else op[i] = kOOB;
        TMD_DCHECK(s[i] >= 0 && s[i] < P.n);
        // an edge past the row gathers from beyond the resources' ranges: its loads return 0, so
        // its k, v and vec terms vanish without masks
        S.ok[i] = ok ? (s[i] * P.ldk + c) * 4 : kOOB;
        S.ov[i] = ok ? (s[i] * P.ldv + c) * 4 : kOOB;
        S.ow[i] = ok ? (s[i] * 3 * H + c) * 4 : kOOB;
        Ce[i] = ok ? P.C[e] : 0.f;
        ux[i] = ok ? P.u[3 * (size_t)e] : 0.f;
        uy[i] = ok ? P.u[3 * (size_t)e + 1] : 0.f;
        uz[i] = ok ? P.u[3 * (size_t)e + 2] : 0.f;
      }
      // heads unrolled; the source gathers of head h + 1 are issued before head h's MFMAs and math
      // (two register sets), and the scheduler may not mix heads (one head's registers live at a time)
      // an opaque zero offset on the LDS reads: the weight fragments are the same for every tile, and
      // without it the compiler hoists all 32 blocks' fragments out of the tile loop (512 VGPRs)
      int wb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        wb[ks] = wfrag_base<KS>(lane, ks);
        asm volatile("" : "+v"(wb[ks]));
      }
      int lo = 0;
      asm volatile("" : "+v"(lo));
      const char* wt = reinterpret_cast<const char*>(w);
      const float* sct = s_sc + lo;
      const float* sbt = s_b + lo;
      if constexpr (MODE == 0) {
        Gat G[2];
        gather<0>(G[0], S);
        static_for<kHeads>([&](auto hc) {
          constexpr int h = decltype(hc)::value;
          if constexpr (h + 1 < kHeads) gather<64 * (h + 1)>(G[(h + 1) & 1], S);
          head_math<KS>(G[h & 1], wt, wb, sct, sbt, h, A0, A1, lane, qh[h], Ce, ux, uy, uz, ax[h], a0[h], a1[h],
                        a2[h], ROWS ? &Rp : nullptr, op);
          __builtin_amdgcn_sched_barrier(0);
        });
      } else if constexpr (MODE == 3) {
        // heads in pairs: the pair's loads carry the head offset in an SGPR, q is re-read per head (L1),
        // the four accumulator arrays rotate by two per pair
#pragma unroll 1
        for (int hp = 0; hp < kHeads; hp += 2) {
          const int sh = __builtin_amdgcn_readfirstlane(64 * hp);
          Gat X0, X1;
          gather_s(X0, S, sh);
          gather_s(X1, S, sh + 64);
          const float q0 = blds(S.q, oq, sh), q1 = blds(S.q, oq + 64, sh);
          const char* wtp = wt + hp * 16 * R * (int)sizeof(_Float16);
          head_math<KS>(X0, wtp, wb, sct + 16 * hp, sbt + 16 * hp, 0, A0, A1, lane, q0, Ce, ux, uy, uz, ax[0],
                        a0[0], a1[0], a2[0]);
          head_math<KS>(X1, wtp, wb, sct + 16 * hp, sbt + 16 * hp, 1, A0, A1, lane, q1, Ce, ux, uy, uz, ax[1],
                        a0[1], a1[1], a2[1]);
          rotate_by<2>(ax); rotate_by<2>(a0); rotate_by<2>(a1); rotate_by<2>(a2);
        }
      } else {
#pragma unroll 1
        for (int h = 0; h < kHeads; ++h) {
          Gat X;
          gather_dyn(X, S, 64 * h);
          head_math<KS>(X, wt, wb, sct, sbt, h, A0, A1, lane, qh[0], Ce, ux, uy, uz, ax[0], a0[0], a1[0], a2[0]);
          rotate(qh); rotate(ax); rotate(a0); rotate(a1); rotate(a2);
        }
      }
    }
    // sum over the four lane groups (edges 4 g + i), then group g stores heads 2g, 2g + 1
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      ax[h] += __shfl_xor(ax[h], 16); ax[h] += __shfl_xor(ax[h], 32);
      a0[h] += __shfl_xor(a0[h], 16); a0[h] += __shfl_xor(a0[h], 32);
      a1[h] += __shfl_xor(a1[h], 16); a1[h] += __shfl_xor(a1[h], 32);
      a2[h] += __shfl_xor(a2[h], 16); a2[h] += __shfl_xor(a2[h], 32);
    }
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      if ((h >> 1) != g) continue;
      const int ch = 16 * h + c;
      P.xo[(size_t)t * H + ch] = ax[h];
      float* vo = P.veco + (size_t)t * 3 * H + ch;
      vo[0] = a0[h];
      vo[H] = a1[h];
      vo[2 * H] = a2[h];
    }
  }
}

// ------------------------------------------------------------------ backward (force pass, "dr mode")
// The first-order backward of the fused message for the force evaluation: d(energy)/d(distance) of
// every edge straight from the projection's r-derivative d pre / d r = W f'(r), formed per tile on the
// MFMA beside the projection itself (two products sharing the W fragments), so neither the projection
// rows nor their r-derivative rows exist in memory (the unfused force pass reads both once per
// direction: 3.4x its distinct bytes at C5).  Two passes as the unfused backward: a destination pass
// (gq, and per edge g_cut, g_unit, g_r) and a source pass over the same CSR rows read as reversed edges
// (gk, gv, gvec_in) -- deterministic, no atomics.

struct Bwd {
  int n, cap, rbf, acc;
  const int32_t* row_ptr;
  const int32_t* src;
  const float* q; int ldq;
  const float* k; int ldk;
  const float* v; int ldv;
  const float* vec;
  const float* r;
  const float* C;
  const float* u;
  const _Float16* img;
  const float* wsc;
  const float* bias;
  const float* mu;
  const float* beta;
  float cl, cu, alpha;
  const float* gx;    // [N][H]   dL/d x_agg
  const float* gvec;  // [N][3][H] dL/d vec_agg (and the layer's residual cotangent)
  float* gq;          // ld ldq
  float* gk;          // ld ldk
  float* gv;          // ld ldv (planar)
  float* gveci;       // [N][3][H] or NULL
  float* gC;
  float* gu;
  float* gr;
};

template <int KS, int NW>
__device__ __forceinline__ void load_image(_Float16* w, float* s_sc, float* s_b, float* s_mu, float* s_beta,
                                           const _Float16* img, const float* wsc, const float* bias, const float* mu,
                                           const float* beta, int rbf) {
  constexpr int R = 32 * KS;
  const u4* g = reinterpret_cast<const u4*>(img);
  u4* l = reinterpret_cast<u4*>(w);
  for (int i = threadIdx.x; i < 2 * kD * R / 8; i += NW * 64) l[i] = g[i];
  for (int i = threadIdx.x; i < kD; i += NW * 64) { s_sc[i] = wsc[i]; s_b[i] = bias[i]; }
  for (int i = threadIdx.x; i < R; i += NW * 64) {
    s_mu[i] = mu[i];
    s_beta[i] = rbf == TMDNET_RBF_EXPNORM ? beta[i] : beta[0];
  }
}

// the RBF A fragments of the tile (lane: edge row `c`, k = 32 ks + 8 g + j) and, DER, those of its
// r-derivative with a tile-uniform power-of-two scale 2^sd (|f'| is not bounded by 1); dsc = 2^(14 - sd)
// turns the weight's accumulator scale wsc (which assumes the 2^14 of f) into the derivative's
template <int KS, bool DER>
__device__ __forceinline__ void rbf_frags(int rbf, float rf, bool vf, float cl, float cu, float alpha,
                                          const float* s_mu, const float* s_beta, int g, h8 (&A0)[KS],
                                          h8 (&A1)[KS], h8 (&D0)[KS], h8 (&D1)[KS], float& dsc) {
  constexpr float kPi = 3.14159265358979323846f;
  const bool in = rf < cu;
  const float cut0 = in ? 0.5f * (cosf(rf * kPi / cu) + 1.f) : 0.f;
  const float dcut0 = (DER && in) ? -0.5f * sinf(rf * kPi / cu) * kPi / cu : 0.f;
  const float ue = expf(alpha * (cl - rf));
  float df[KS][8];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 32 * ks + 8 * g + j;
      float f, d;
      if (rbf == TMDNET_RBF_EXPNORM) {
        const float z = ue - s_mu[kk], b = s_beta[kk];
        const float gg = expf(-b * z * z);
        f = cut0 * gg;
        d = dcut0 * gg + cut0 * gg * (2.f * b * z * alpha * ue);  // d/dr: du = -alpha ue
      } else {
        const float z = rf - s_mu[kk], co = s_beta[kk];
        f = expf(co * z * z);
        d = f * 2.f * co * z;
      }
      f = vf ? f : 0.f;
      df[ks][j] = vf ? d : 0.f;
      const float x = f * kFScale;
      const _Float16 hi = (_Float16)x;
      A0[ks][j] = hi;
      A1[ks][j] = (_Float16)(x - (float)hi);
    }
  if constexpr (DER) {
    float mx = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(df[ks][j]));
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    int ex = 0;
    if (mx > 0.f) frexpf(mx, &ex);
    const int sd = mx > 0.f ? 14 - ex : 0;
    dsc = ldexpf(1.f, 14 - sd);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = ldexpf(df[ks][j], sd);
        const _Float16 hi = (_Float16)x;
        D0[ks][j] = hi;
        D1[ks][j] = (_Float16)(x - (float)hi);
      }
  }
}

// d pre / d r of one 16-row block: W f' (no bias), scaled back
template <int KS>
__device__ __forceinline__ f4 block_dpre(const char* wl, const int (&wb)[KS], const float* sc, float dsc, int blk,
                                         const h8 (&d0)[KS], const h8 (&d1)[KS], int lane) {
  constexpr int R = 32 * KS, PB = kD * R * (int)sizeof(_Float16);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const char* f0 = wl + wb[ks] + blk * 16 * R * (int)sizeof(_Float16);
    const h8 w0 = *reinterpret_cast<const h8*>(f0);
    const h8 w1 = *reinterpret_cast<const h8*>(f0 + PB);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(d1[ks], w0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(d0[ks], w1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(d0[ks], w0, acc, 0, 0, 0);
  }
  const float s = sc[16 * blk + (lane & 15)] * dsc;
  f4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = acc[i] * s;
  return o;
}

// Destination pass (dr mode): gq; per edge g_cut, g_unit, g_r (TMDNET_ACC_EDGE: accumulated).
template <int KS, int NW>
__global__ __launch_bounds__(NW * 64, 1) void k_bwd_dst(Bwd P) {
  constexpr int R = 32 * KS, H = kH, PB = kH * 4;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ float s_sc[kD], s_b[kD], s_mu[R], s_beta[R];
  __shared__ int s_next;
  load_image<KS, NW>(w, s_sc, s_b, s_mu, s_beta, P.img, P.wsc, P.bias, P.mu, P.beta, P.rbf);
  if (threadIdx.x == 0) s_next = 0;
  // static-capacity lists: edge slots past the last row belong to no row -- zeroed (spread over the grid)
  {
    const int e0 = min(P.row_ptr[P.n], P.cap);
    for (int e = e0 + blockIdx.x * NW * 64 + threadIdx.x; e < P.cap; e += gridDim.x * NW * 64) {
      P.gC[e] = 0.f;
      P.gu[3 * (size_t)e] = P.gu[3 * (size_t)e + 1] = P.gu[3 * (size_t)e + 2] = 0.f;
      P.gr[e] = 0.f;
    }
  }
  __syncthreads();
  const int nwg = gridDim.x, lb = xcd_remap(blockIdx.x, nwg);
  const int per = (P.n + nwg - 1) / nwg;
  const int n0 = lb * per, n1 = min(P.n, n0 + per);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4;
  const bool acc_edge = P.acc & TMDNET_ACC_EDGE;
  Src S;
  S.q = make_rsrc(P.q, (unsigned)P.n * P.ldq * 4u);
  S.k = make_rsrc(P.k, (unsigned)P.n * P.ldk * 4u);
  S.v = make_rsrc(P.v, (unsigned)P.n * P.ldv * 4u);
  S.vec = make_rsrc(P.vec, P.vec ? (unsigned)P.n * 3u * H * 4u : 0u);
  const rsrc_t Rgx = make_rsrc(P.gx, (unsigned)P.n * H * 4u), Rgv = make_rsrc(P.gvec, (unsigned)P.n * 3u * H * 4u);
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(&s_next, 1);
    t = __builtin_amdgcn_readfirstlane(__shfl(t, 0)) + n0;
    if (t >= n1) break;
    const int rb = min(P.row_ptr[t], P.cap), re = min(P.row_ptr[t + 1], P.cap);
    const int oq = (t * P.ldq + c) * 4, ox = (t * H + c) * 4, og = (t * 3 * H + c) * 4;
    float gq[kHeads];
#pragma unroll
    for (int h = 0; h < kHeads; ++h) gq[h] = 0.f;
    for (int base = rb; base < re; base += 16) {
      h8 A0[KS], A1[KS], D0[KS], D1[KS];
      float dsc = 1.f;
      {
        const int ef = base + c;
        const bool vf = ef < re;
        rbf_frags<KS, true>(P.rbf, vf ? P.r[ef] : 0.f, vf, P.cl, P.cu, P.alpha, s_mu, s_beta, g, A0, A1, D0, D1, dsc);
      }
      int s[4];
      float Ce[4], ux[4], uy[4], uz[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + 4 * g + i;
        const bool ok = e < re;
        s[i] = ok ? P.src[e] : 0;
        TMD_DCHECK(s[i] >= 0 && s[i] < P.n);
        S.ok[i] = ok ? (s[i] * P.ldk + c) * 4 : kOOB;
        S.ov[i] = ok ? (s[i] * P.ldv + c) * 4 : kOOB;
        S.ow[i] = ok ? (s[i] * 3 * H + c) * 4 : kOOB;
        Ce[i] = ok ? P.C[e] : 0.f;
        ux[i] = ok ? P.u[3 * (size_t)e] : 0.f;
        uy[i] = ok ? P.u[3 * (size_t)e + 1] : 0.f;
        uz[i] = ok ? P.u[3 * (size_t)e + 2] : 0.f;
      }
      int wb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        wb[ks] = wfrag_base<KS>(lane, ks);
        asm volatile("" : "+v"(wb[ks]));
      }
      int lo = 0;
      asm volatile("" : "+v"(lo));
      const char* wt = reinterpret_cast<const char*>(w);
      const float* sct = s_sc + lo;
      const float* sbt = s_b + lo;
      float eC[4] = {0.f, 0.f, 0.f, 0.f}, er[4] = {0.f, 0.f, 0.f, 0.f};
      float eu0[4] = {0.f, 0.f, 0.f, 0.f}, eu1[4] = {0.f, 0.f, 0.f, 0.f}, eu2[4] = {0.f, 0.f, 0.f, 0.f};
      static_for<kHeads>([&](auto hc) {
        constexpr int h = decltype(hc)::value, HB = 64 * h;
        Gat X;
        gather<HB>(X, S);
        const float qd = bld(S.q, oq + HB), gxd = bld(Rgx, ox + HB);
        const float g0 = bld(Rgv, og + HB), g1 = bld(Rgv, og + HB + PB), g2 = bld(Rgv, og + HB + 2 * PB);
        const f4 pk = block_pre<KS>(wt, wb, sct, sbt, h, A0, A1, lane);
        const f4 px = block_pre<KS>(wt, wb, sct, sbt, 8 + h, A0, A1, lane);
        const f4 p1 = block_pre<KS>(wt, wb, sct, sbt, 16 + h, A0, A1, lane);
        const f4 p2 = block_pre<KS>(wt, wb, sct, sbt, 24 + h, A0, A1, lane);
        f4 gpk, gpx, gp1, gp2;  // the projection gradient, contracted with d pre / d r below
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const Silu<float> sk(pk[i]), sx(px[i]), s1(p1[i]), s2(p2[i]);
          const float kdk = X.kk[i] * sk.s;
          const float att = row_sum16(qd * kdk);
          const float ga = row_sum16(gxd * X.vx[i] * sx.s);
          const Silu<float> sa(att);
          const float a = sa.s * Ce[i];
          const float gs = ga * Ce[i] * sa.d(att);
          gq[h] += gs * kdk;
          gpk[i] = gs * qd * X.kk[i] * sk.d(pk[i]);
          gpx[i] = gxd * a * X.vx[i] * sx.d(px[i]);
          const float gv1e = g0 * X.w0[i] + g1 * X.w1[i] + g2 * X.w2[i];
          gp1[i] = gv1e * X.v1[i] * s1.d(p1[i]);
          const float gv2e = g0 * ux[i] + g1 * uy[i] + g2 * uz[i];
          gp2[i] = gv2e * X.v2[i] * s2.d(p2[i]);
          eC[i] += ga * sa.s;  // row-uniform: every lane of the row holds the same value
          const float v2e = X.v2[i] * s2.s;
          eu0[i] += g0 * v2e;
          eu1[i] += g1 * v2e;
          eu2[i] += g2 * v2e;
        }
        // the r-derivative blocks one at a time (fewer live accumulators)
        const f4 gpb[4] = {gpk, gpx, gp1, gp2};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const f4 rd = block_dpre<KS>(wt, wb, sct, dsc, 8 * b + h, D0, D1, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i) er[i] += gpb[b][i] * rd[i];
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      // the edge sums over the 16 channels of the row, written by the row's lane 0
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        eu0[i] = row_sum16(eu0[i]);
        eu1[i] = row_sum16(eu1[i]);
        eu2[i] = row_sum16(eu2[i]);
        er[i] = row_sum16(er[i]);
      }
      if (c == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = base + 4 * g + i;
          if (e < re) {
            float* gu = P.gu + 3 * (size_t)e;
            if (acc_edge) {
              P.gC[e] += eC[i];
              gu[0] += eu0[i]; gu[1] += eu1[i]; gu[2] += eu2[i];
              P.gr[e] += er[i];
            } else {
              P.gC[e] = eC[i];
              gu[0] = eu0[i]; gu[1] = eu1[i]; gu[2] = eu2[i];
              P.gr[e] = er[i];
            }
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      gq[h] += __shfl_xor(gq[h], 16);
      gq[h] += __shfl_xor(gq[h], 32);
    }
    const bool ag = P.acc & TMDNET_ACC_GRADS;
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      if ((h >> 1) != g) continue;
      float* d = P.gq + (size_t)t * P.ldq + 16 * h + c;
      *d = ag ? *d + gq[h] : gq[h];
    }
  }
}

// Source pass: node j as the source of the reversed edges j -> m of its row (same dk / dv / cutoff,
// unit vector negated): gk, gv (planar x | v1 | v2), gvec_in (+ the residual cotangent with
// TMDNET_ACC_VEC_RESIDUAL).
struct Dst {
  float q[4], gx[4], g0[4], g1[4], g2[4];
};
template <int HB>
__device__ __forceinline__ void gather_dst(Dst& Y, rsrc_t Rq, rsrc_t Rgx, rsrc_t Rgv, const int (&oq)[4],
                                           const int (&ox)[4], const int (&og)[4]) {
  constexpr int PB = kH * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Y.q[i] = bld(Rq, oq[i] + HB);
    Y.gx[i] = bld(Rgx, ox[i] + HB);
    Y.g0[i] = bld(Rgv, og[i] + HB);
    Y.g1[i] = bld(Rgv, og[i] + HB + PB);
    Y.g2[i] = bld(Rgv, og[i] + HB + 2 * PB);
  }
}

template <int KS, int NW>
__global__ __launch_bounds__(NW * 64, 1) void k_bwd_src(Bwd P) {
  constexpr int R = 32 * KS, H = kH, PB = kH * 4;
  __shared__ __attribute__((aligned(16))) _Float16 w[2 * kD * R];
  __shared__ float s_sc[kD], s_b[kD], s_mu[R], s_beta[R];
  __shared__ int s_next;
  load_image<KS, NW>(w, s_sc, s_b, s_mu, s_beta, P.img, P.wsc, P.bias, P.mu, P.beta, P.rbf);
  if (threadIdx.x == 0) s_next = 0;
  __syncthreads();
  const int nwg = gridDim.x, lb = xcd_remap(blockIdx.x, nwg);
  const int per = (P.n + nwg - 1) / nwg;
  const int n0 = lb * per, n1 = min(P.n, n0 + per);
  const int lane = lane_id(), c = lane & 15, g = lane >> 4;
  const rsrc_t Rq = make_rsrc(P.q, (unsigned)P.n * P.ldq * 4u), Rgx = make_rsrc(P.gx, (unsigned)P.n * H * 4u);
  const rsrc_t Rgv = make_rsrc(P.gvec, (unsigned)P.n * 3u * H * 4u);
  const rsrc_t Rk = make_rsrc(P.k, (unsigned)P.n * P.ldk * 4u), Rv = make_rsrc(P.v, (unsigned)P.n * P.ldv * 4u);
  const rsrc_t Rw = make_rsrc(P.vec, P.vec ? (unsigned)P.n * 3u * H * 4u : 0u);
  const bool ag = P.acc & TMDNET_ACC_GRADS, resid = P.acc & TMDNET_ACC_VEC_RESIDUAL;
  for (;;) {
    int j = 0;
    if (lane == 0) j = atomicAdd(&s_next, 1);
    j = __builtin_amdgcn_readfirstlane(__shfl(j, 0)) + n0;
    if (j >= n1) break;
    const int rb = min(P.row_ptr[j], P.cap), re = min(P.row_ptr[j + 1], P.cap);
    const int ok_ = (j * P.ldk + c) * 4, ov_ = (j * P.ldv + c) * 4, ow_ = (j * 3 * H + c) * 4;
    float gk[kHeads], gvx[kHeads], gv1[kHeads], gv2[kHeads], gw0[kHeads], gw1[kHeads], gw2[kHeads];
#pragma unroll
    for (int h = 0; h < kHeads; ++h) gk[h] = gvx[h] = gv1[h] = gv2[h] = gw0[h] = gw1[h] = gw2[h] = 0.f;
    for (int base = rb; base < re; base += 16) {
      h8 A0[KS], A1[KS], D0[KS], D1[KS];
      float dsc = 1.f;
      {
        const int ef = base + c;
        const bool vf = ef < re;
        rbf_frags<KS, false>(P.rbf, vf ? P.r[ef] : 0.f, vf, P.cl, P.cu, P.alpha, s_mu, s_beta, g, A0, A1, D0, D1,
                             dsc);
      }
      int oq[4], ox[4], og[4];
      float Ce[4], ux[4], uy[4], uz[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + 4 * g + i;
        const bool ok = e < re;
        const int m = ok ? P.src[e] : 0;
        TMD_DCHECK(m >= 0 && m < P.n);
        oq[i] = ok ? (m * P.ldq + c) * 4 : kOOB;
        ox[i] = ok ? (m * H + c) * 4 : kOOB;
        og[i] = ok ? (m * 3 * H + c) * 4 : kOOB;
        Ce[i] = ok ? P.C[e] : 0.f;
        ux[i] = ok ? -P.u[3 * (size_t)e] : 0.f;  // the reversed edge j -> m
        uy[i] = ok ? -P.u[3 * (size_t)e + 1] : 0.f;
        uz[i] = ok ? -P.u[3 * (size_t)e + 2] : 0.f;
      }
      int wb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        wb[ks] = wfrag_base<KS>(lane, ks);
        asm volatile("" : "+v"(wb[ks]));
      }
      int lo = 0;
      asm volatile("" : "+v"(lo));
      const char* wt = reinterpret_cast<const char*>(w);
      const float* sct = s_sc + lo;
      const float* sbt = s_b + lo;
      Dst Y[2];
      gather_dst<0>(Y[0], Rq, Rgx, Rgv, oq, ox, og);
      static_for<kHeads>([&](auto hc) {
        constexpr int h = decltype(hc)::value, HB = 64 * h;
        if constexpr (h + 1 < kHeads) gather_dst<64 * (h + 1)>(Y[(h + 1) & 1], Rq, Rgx, Rgv, oq, ox, og);
        const Dst& X = Y[h & 1];
        const float kj = bld(Rk, ok_ + HB), vxj = bld(Rv, ov_ + HB), v1j = bld(Rv, ov_ + HB + PB);
        const float v2j = bld(Rv, ov_ + HB + 2 * PB);
        const float w0j = bld(Rw, ow_ + HB), w1j = bld(Rw, ow_ + HB + PB), w2j = bld(Rw, ow_ + HB + 2 * PB);
        const f4 pk = block_pre<KS>(wt, wb, sct, sbt, h, A0, A1, lane);
        const f4 px = block_pre<KS>(wt, wb, sct, sbt, 8 + h, A0, A1, lane);
        const f4 p1 = block_pre<KS>(wt, wb, sct, sbt, 16 + h, A0, A1, lane);
        const f4 p2 = block_pre<KS>(wt, wb, sct, sbt, 24 + h, A0, A1, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dk = Silu<float>(pk[i]).s, dvx = Silu<float>(px[i]).s;
          const float dv1 = Silu<float>(p1[i]).s, dv2 = Silu<float>(p2[i]).s;
          const float att = row_sum16(X.q[i] * kj * dk);
          const float ga = row_sum16(X.gx[i] * vxj * dvx);
          const Silu<float> sa(att);
          const float a = sa.s * Ce[i];
          const float gs = ga * Ce[i] * sa.d(att);
          gk[h] += gs * X.q[i] * dk;
          gvx[h] += X.gx[i] * a * dvx;
          const float gv1e = X.g0[i] * w0j + X.g1[i] * w1j + X.g2[i] * w2j;
          gv1[h] += gv1e * dv1;
          const float gv2e = X.g0[i] * ux[i] + X.g1[i] * uy[i] + X.g2[i] * uz[i];
          gv2[h] += gv2e * dv2;
          const float v1e = v1j * dv1;
          gw0[h] += X.g0[i] * v1e;
          gw1[h] += X.g1[i] * v1e;
          gw2[h] += X.g2[i] * v1e;
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    }
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      float* a[7] = {&gk[h], &gvx[h], &gv1[h], &gv2[h], &gw0[h], &gw1[h], &gw2[h]};
#pragma unroll
      for (int z = 0; z < 7; ++z) {
        *a[z] += __shfl_xor(*a[z], 16);
        *a[z] += __shfl_xor(*a[z], 32);
      }
    }
    auto put = [&](float* d, float v) { *d = ag ? *d + v : v; };
#pragma unroll
    for (int h = 0; h < kHeads; ++h) {
      if ((h >> 1) != g) continue;
      const int ch = 16 * h + c;
      put(P.gk + (size_t)j * P.ldk + ch, gk[h]);
      float* gvj = P.gv + (size_t)j * P.ldv + ch;
      put(gvj, gvx[h]);
      put(gvj + H, gv1[h]);
      put(gvj + 2 * H, gv2[h]);
      if (P.gveci) {
        float w0 = gw0[h], w1 = gw1[h], w2 = gw2[h];
        if (resid) {
          const float* rr = P.gvec + (size_t)j * 3 * H + ch;
          w0 += rr[0]; w1 += rr[H]; w2 += rr[2 * H];
        }
        float* gw = P.gveci + (size_t)j * 3 * H + ch;
        put(gw, w0);
        put(gw + H, w1);
        put(gw + 2 * H, w2);
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

extern "C" int tmdnet_et_fused_fwd_f32(int n, int H, int heads, int R, const int32_t* row_ptr, const int32_t* src,
                                       int cap, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                       const void* vec, const void* r, const void* C, const void* u, const void* img,
                                       const void* wsc, const void* bias, const void* mu, const void* beta,
                                       double cutoff_lower, double cutoff_upper, int rbf_type, void* x_out,
                                       void* vec_out, void* pkv_out, int ld_pkv, const int32_t* pk_rows,
                                       long long n_pair_rows, void* stream) {
  if (n < 0 || !row_ptr || !src || !q || !k || !v || !r || !C || !u || !img || !wsc || !bias || !mu || !beta ||
      !x_out || !vec_out || (pkv_out && (!pk_rows || ld_pkv < 4 * H)))
    return kBadArgument;
  // the rows are written through a 32-bit byte offset
  if (pkv_out && n_pair_rows * (long long)ld_pkv * 4 >= 0xFFFFFFF0LL) return kUnsupported;
  if (n == 0) return kOk;
  if (H != fep::kH || heads != fep::kHeads || (R != 32 && R != 64)) return kUnsupported;
  if (ldq < H || ldk < H || ldv < 3 * H) return kBadArgument;
  if (((uintptr_t)img) & 15) return kUnsupported;
  fep::Fwd P{};
  P.n = n; P.cap = cap; P.rbf = rbf_type;
  P.row_ptr = row_ptr; P.src = src;
  P.q = (const float*)q; P.ldq = ldq; P.k = (const float*)k; P.ldk = ldk; P.v = (const float*)v; P.ldv = ldv;
  P.vec = (const float*)vec; P.r = (const float*)r; P.C = (const float*)C; P.u = (const float*)u;
  P.img = (const _Float16*)img; P.wsc = (const float*)wsc; P.bias = (const float*)bias;
  P.mu = (const float*)mu; P.beta = (const float*)beta;
  P.cl = (float)cutoff_lower; P.cu = (float)cutoff_upper;
  P.alpha = (float)(5.0 / (cutoff_upper - cutoff_lower));
  P.xo = (float*)x_out; P.veco = (float*)vec_out;
  P.pkv = (float*)pkv_out; P.ldp = ld_pkv; P.prow = pk_rows;
  P.pbytes = pkv_out ? (unsigned)(n_pair_rows * (long long)ld_pkv * 4) : 0u;
  const int nwg = fep::num_cus();
  // tuning (TMDNET_FEP_MODE): 0 = unrolled heads, one wave per SIMD; 1 = rolled heads, two per SIMD;
  // 2 = unrolled, two per SIMD; 3 = heads in pairs with SGPR head offsets
  static const int mode = getenv("TMDNET_FEP_MODE") ? atoi(getenv("TMDNET_FEP_MODE")) : 2;
  hipStream_t st = (hipStream_t)stream;
#define TMD_FEP(KS_, NW_, M_) hipLaunchKernelGGL((fep::k_fwd<KS_, NW_, M_>), dim3(nwg), dim3(NW_ * 64), 0, st, P)
  // (the row write-out exists in the default variant only)
  if (pkv_out) {
    if (R == 64) hipLaunchKernelGGL((fep::k_fwd<2, 8, 0, true>), dim3(nwg), dim3(512), 0, st, P);
    else hipLaunchKernelGGL((fep::k_fwd<1, 8, 0, true>), dim3(nwg), dim3(512), 0, st, P);
  } else if (R == 64) {
    if (mode == 0) TMD_FEP(2, 4, 0); else if (mode == 2) TMD_FEP(2, 8, 0); else if (mode == 3) TMD_FEP(2, 8, 3);
    else TMD_FEP(2, 8, 1);
  } else {
    if (mode == 0) TMD_FEP(1, 4, 0); else if (mode == 2) TMD_FEP(1, 8, 0); else if (mode == 3) TMD_FEP(1, 8, 3);
    else TMD_FEP(1, 8, 1);
  }
#undef TMD_FEP
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_et_fused_bwd_f32(int n, int H, int heads, int R, const int32_t* row_ptr, const int32_t* src,
                                       int cap, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                       const void* vec, const void* r, const void* C, const void* u, const void* img,
                                       const void* wsc, const void* bias, const void* mu, const void* beta,
                                       double cutoff_lower, double cutoff_upper, int rbf_type, const void* gx,
                                       const void* gvec, void* gq, void* gk, void* gv, void* gvec_in, void* gC,
                                       void* gu, void* gdist, int accumulate, void* stream) {
  if (n < 0 || !row_ptr || !src || !q || !k || !v || !r || !C || !u || !img || !wsc || !bias || !mu || !beta || !gx ||
      !gvec || !gq || !gk || !gv || !gC || !gu || !gdist)
    return kBadArgument;
  if (n == 0) return kOk;
  if (H != fep::kH || heads != fep::kHeads || (R != 32 && R != 64)) return kUnsupported;
  if (ldq < H || ldk < H || ldv < 3 * H) return kBadArgument;
  if (((uintptr_t)img) & 15) return kUnsupported;
  fep::Bwd P{};
  P.n = n; P.cap = cap; P.rbf = rbf_type; P.acc = accumulate;
  P.row_ptr = row_ptr; P.src = src;
  P.q = (const float*)q; P.ldq = ldq; P.k = (const float*)k; P.ldk = ldk; P.v = (const float*)v; P.ldv = ldv;
  P.vec = (const float*)vec; P.r = (const float*)r; P.C = (const float*)C; P.u = (const float*)u;
  P.img = (const _Float16*)img; P.wsc = (const float*)wsc; P.bias = (const float*)bias;
  P.mu = (const float*)mu; P.beta = (const float*)beta;
  P.cl = (float)cutoff_lower; P.cu = (float)cutoff_upper;
  P.alpha = (float)(5.0 / (cutoff_upper - cutoff_lower));
  P.gx = (const float*)gx; P.gvec = (const float*)gvec;
  P.gq = (float*)gq; P.gk = (float*)gk; P.gv = (float*)gv; P.gveci = (float*)gvec_in;
  P.gC = (float*)gC; P.gu = (float*)gu; P.gr = (float*)gdist;
  const int nwg = fep::num_cus();
  constexpr int NW = 8;
  hipStream_t st = (hipStream_t)stream;
  if (R == 64) {
    hipLaunchKernelGGL((fep::k_bwd_dst<2, NW>), dim3(nwg), dim3(NW * 64), 0, st, P);
    hipLaunchKernelGGL((fep::k_bwd_src<2, NW>), dim3(nwg), dim3(NW * 64), 0, st, P);
  } else {
    hipLaunchKernelGGL((fep::k_bwd_dst<1, NW>), dim3(nwg), dim3(NW * 64), 0, st, P);
    hipLaunchKernelGGL((fep::k_bwd_src<1, NW>), dim3(nwg), dim3(NW * 64), 0, st, P);
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
