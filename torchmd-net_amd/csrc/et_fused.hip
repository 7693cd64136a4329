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
                                          float& a2) {
  const f4 pk = block_pre<KS>(wt, wb, sct, sbt, h, A0, A1, lane);
  const f4 px = block_pre<KS>(wt, wb, sct, sbt, 8 + h, A0, A1, lane);
  const f4 p1 = block_pre<KS>(wt, wb, sct, sbt, 16 + h, A0, A1, lane);
  const f4 p2 = block_pre<KS>(wt, wb, sct, sbt, 24 + h, A0, A1, lane);
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
template <int KS, int NW, int MODE>
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
      int s[4];
      float Ce[4], ux[4], uy[4], uz[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + 4 * g + i;
        const bool ok = e < re;
        s[i] = ok ? P.src[e] : 0;
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
                        a2[h]);
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
                                       void* vec_out, void* stream) {
  if (n < 0 || !row_ptr || !src || !q || !k || !v || !r || !C || !u || !img || !wsc || !bias || !mu || !beta ||
      !x_out || !vec_out)
    return kBadArgument;
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
  const int nwg = fep::num_cus();
  // tuning (TMDNET_FEP_MODE): 0 = unrolled heads, one wave per SIMD; 1 = rolled heads, two per SIMD;
  // 2 = unrolled, two per SIMD; 3 = heads in pairs with SGPR head offsets
  static const int mode = getenv("TMDNET_FEP_MODE") ? atoi(getenv("TMDNET_FEP_MODE")) : 2;
  hipStream_t st = (hipStream_t)stream;
#define TMD_FEP(KS_, NW_, M_) hipLaunchKernelGGL((fep::k_fwd<KS_, NW_, M_>), dim3(nwg), dim3(NW_ * 64), 0, st, P)
  if (R == 64) {
    if (mode == 0) TMD_FEP(2, 4, 0); else if (mode == 2) TMD_FEP(2, 8, 0); else if (mode == 3) TMD_FEP(2, 8, 3);
    else TMD_FEP(2, 8, 1);
  } else {
    if (mode == 0) TMD_FEP(1, 4, 0); else if (mode == 2) TMD_FEP(1, 8, 0); else if (mode == 3) TMD_FEP(1, 8, 3);
    else TMD_FEP(1, 8, 1);
  }
#undef TMD_FEP
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
