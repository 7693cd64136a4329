// TensorNet edge kernels: tensor embedding aggregation and tensor message passing.
//
// Reference: TensorEmbedding.forward (models/tensornet.py:287-326), tensor_message_passing +
// Interaction.forward (tensornet.py:329-410).  The reference scatters edge messages into
// edge_index[0] (the SOURCE) with torch_scatter atomics and gathers from edge_index[1].  With the
// symmetric destination-grouped CSR the edges whose source is n are exactly the reverses of row n,
// so one wave per (atom n, 64-channel block) walks row n and accumulates n's outputs in registers:
//   * embedding:  Zij(n->m) = P[n] + Q[m]   (emb2(cat(Z_i, Z_j)) split into per-node halves,
//     P = Z Wa^T + b, Q = Z Wb^T computed as two small GEMMs),
//     I[n] += Zij W1 C Id,  A[n] += Zij W2 C skew(u(n->m)),  S[n] += Zij W3 C sym(u(n->m)),
//     with u(n->m) = -u(e') for the row edge e' = m->n and W, C functions of |r| only;
//   * message:    msg[n] += ea(e',h,0) I[m] + ea(e',h,1) A[m] + ea(e',h,2) S[m].
//
// Layout: COMPACT and component-major, [9][N][H] (tn_node.h): row 0 the isotropic coefficient i
// (I = i Id), rows 1-3 the antisymmetric part (a01, a02, a12), rows 4-8 the symmetric traceless
// part (s00, s11, s01, s02, s12).  I, A, S of one channel are disjoint rows of one buffer, the
// channel mixes of the reference (tensornet.py:318-320, 354-356) are plain GEMMs over those rows,
// and a lane's 9 loads are 9 coalesced 256-byte row segments (the reference's [N][H][3][3] I, A,
// S tensors are 27 values per channel, 18 of them redundant).
// `mult0` (>= 1) is the multiplicity of atom 0's self loop: the reference's static_shapes mode
// turns every (-1,-1) padding slot of the CUDA neighbour list into an extra (0,0) edge with r = 0
// (tensornet.py:215-221), i.e. (max_num_pairs - num_pairs) more copies of that self loop.
// Backward = destination pass (own outputs + per-edge grads) + source pass (gathered inputs' grads).
#include <cstdlib>

#include "common.h"
#include "tmdnet.h"
#include "tn_node.h"

namespace tmd {
namespace tn {

// CP / OP: input / output "pointer" types -- const T* / T* for the first-order kernels, node::DIn / DOut
// (value and tangent arrays) for the embedding's second order on dual numbers (tmdnet_tn_embed_bwd2)
template <typename T, typename CP = const T*, typename OP = T*> struct ArgsT {
  int n, H, nblk, cap;
  size_t nh;                // component stride of the compact layout (N * H)
  T mult0;
  const int32_t* npd;  // device num_pairs: mult0 = 1 + max(0, padcap - *npd) (HIP-graph capturable)
  int padcap;
  const int32_t* row_ptr;
  const int32_t* src;
  // embedding
  CP P; CP Q;               // [N][H]
  CP W; int ldw;            // [E][3H] (W1 | W2 | W3), pre-cutoff
  CP C;                     // [E]
  CP u;                     // [E][3]
  OP E;                     // [9][N][H]
  CP gE;
  OP gP; OP gQ; OP gW; OP gC; OP gu;
  // message
  const T* ea; int ldea;    // [E][3H] interleaved (h, c)
  const T* Tc;              // [9][N][H]
  T* msg;                   // [9][N][H]
  const T* gmsg;
  T* gea; T* gT;
  const T* gTadd;           // [9][N][H] or NULL: added to gT (the component tensor's other consumer)
  // pair rows (large systems): ea / gea hold one row per edge PAIR (the two directions of a pair have the
  // same factors, functions of |r| only), edge k reads row prow[k] (tmdnet_pair_index numbering)
  const int32_t* prow;      // [E] or NULL (per-edge rows)
  const int32_t* pedge;     // [np] the canonical edge of each pair slot
  int np;                   // pair slots
};
template <typename T> using Args = ArgsT<T>;

template <typename AT> __device__ __forceinline__ int ea_row(const AT& A, int k) {
  return A.prow ? A.prow[k] : k;
}

// Multiplicity of atom 0's self loop.  With a device pair count (static_shapes under HIP-graph
// capture) it is computed here: 1 + (reference padding capacity - pairs found), a uniform scalar load.
template <typename T, typename CP, typename OP>
__device__ __forceinline__ T mult0_of(const ArgsT<T, CP, OP>& A) {
  if (A.npd == nullptr) return A.mult0;
  const int pad = A.padcap - __builtin_amdgcn_readfirstlane(A.npd[0]);
  return T(double(1 + (pad > 0 ? pad : 0)));
}

// Static-capacity edge lists: rows [row_ptr[n], cap) of the per-edge gradient outputs belong to no
// CSR row.  They are zeroed here, spread over the whole grid (every thread, before any early exit),
// so the weight-gradient GEMMs over all `cap` rows (the edge / distance MLPs) see zeros, not stale
// memory; the dynamic graph (cap == row_ptr[n]) skips it.
template <typename AT, typename P>
__device__ __forceinline__ void zero_tail_rows(const AT& A, P p, int w) {
  if (!p) return;
  const int e0 = min(A.row_ptr[A.n], A.cap);
  if (e0 >= A.cap) return;
  const long long cnt = (long long)(A.cap - e0) * w;
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  for (long long i = tid; i < cnt; i += nth) p[(size_t)e0 * w + i] = decltype(A.mult0)(0.0);
}

// One workgroup of S waves per (node, 64-channel block): the node's edges are dealt round-robin to the
// S waves (edge b + w, b + w + S, ...), whose partial sums are then folded in wave order through LDS
// (deterministic).  With one wave walking a node's ~20 edges serially, each edge costing a dependent
// src -> row gather, these kernels were latency chains: 11-36 us per launch at C3 (168 atoms).
template <int S> __device__ __forceinline__ void slot_node(int nblk, int& node, int& ch0, int& w) {
  node = blockIdx.x / nblk;
  ch0 = (blockIdx.x % nblk) * TMD_WAVE;
  w = threadIdx.x / TMD_WAVE;
}

// acc (K values per lane) summed over the block's S waves, wave 0 last-to-hold the total; red: S-1 x K x 64
template <typename T, int K, int S>
__device__ __forceinline__ bool fold_waves(T (&acc)[K], T* red) {
  if constexpr (S == 1) {
    return true;
  } else {
    const int w = threadIdx.x / TMD_WAVE, lane = lane_id();
    if (w > 0) {
#pragma unroll
      for (int i = 0; i < K; ++i) red[((w - 1) * K + i) * TMD_WAVE + lane] = acc[i];
    }
    __syncthreads();
    if (w != 0) return false;
#pragma unroll
    for (int s = 1; s < S; ++s)
#pragma unroll
      for (int i = 0; i < K; ++i) acc[i] += red[((s - 1) * K + i) * TMD_WAVE + lane];
    return true;
  }
}

template <typename T, typename P> __device__ __forceinline__ void ldc(T (&o)[9], P p, size_t nh) {
#pragma unroll
  for (int k = 0; k < 9; ++k) o[k] = p[k * nh];
}
template <typename T, typename P> __device__ __forceinline__ void stc(P p, size_t nh, const T (&o)[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) p[k * nh] = o[k];
}

// compact coordinates of skew(v) = [[0,-z,y],[z,0,-x],[-y,x,0]]  (tensornet.py:16-34)
template <typename T> __device__ __forceinline__ void skew_c(T (&a)[3], T x, T y, T z) {
  a[0] = -z; a[1] = y; a[2] = -x;
}
// compact coordinates of sym(v) = v v^T - |v|^2/3 Id  (tensornet.py:37-44)
template <typename T> __device__ __forceinline__ void sym_c(T (&s)[5], T x, T y, T z) {
  const T tr = (x * x + y * y + z * z) / T(3);
  s[0] = x * x - tr; s[1] = y * y - tr; s[2] = x * y; s[3] = x * z; s[4] = y * z;
}
// d<g, skew_c(v)>/dv
template <typename T> __device__ __forceinline__ void dskew_c(const T* g, T& dx, T& dy, T& dz) {
  dx = -g[2]; dy = g[1]; dz = -g[0];
}
// d<g, sym_c(v)>/dv
template <typename T>
__device__ __forceinline__ void dsym_c(const T* g, T x, T y, T z, T& dx, T& dy, T& dz) {
  const T t = (g[0] + g[1]) * (T(2) / T(3));
  dx = T(2) * g[0] * x - t * x + g[2] * y + g[3] * z;
  dy = T(2) * g[1] * y - t * y + g[2] * x + g[4] * z;
  dz = -t * z + g[3] * x + g[4] * y;
}

// ---------------------------------------------------------------- embedding forward
// (T = node::Dual<float|double> with DIn / DOut pointers: the second order, tmdnet_tn_embed_bwd2; shared
// arrays as raw bytes, the dual type having a constructor)
#define TMD_RED(T, NV) \
  __shared__ __attribute__((aligned(16))) unsigned char red_[(NV) * sizeof(T)]; \
  T* red = reinterpret_cast<T*>(red_);

template <typename T, int S, typename AT = Args<T>>
__global__ __launch_bounds__(64 * S) void k_embed_fwd(AT A) {
  TMD_RED(T, S > 1 ? (S - 1) * 9 * TMD_WAVE : 1)
  int n, ch0, w;
  slot_node<S>(A.nblk, n, ch0, w);
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  const T Pn = A.P[(size_t)n * A.H + hc];
  T acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = T(0);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  // two edges per iteration (k, k + S: the one-at-a-time order), every load of both issued before the math
  for (int k = b + w; k < e; k += 2 * S) {
    const bool two = k + S < e;
    const int kk[2] = {k, two ? k + S : k};
    int m[2];
    T q[2], cc[2], wv[2][3], ux[2], uy[2], uz[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      m[j] = A.src[kk[j]];
      TMD_DCHECK(m[j] >= 0 && m[j] < A.n);
      q[j] = A.Q[(size_t)m[j] * A.H + hc];
      cc[j] = A.C[kk[j]];
      const auto wr = A.W + (size_t)kk[j] * A.ldw;
      wv[j][0] = wr[hc]; wv[j][1] = wr[A.H + hc]; wv[j][2] = wr[2 * A.H + hc];
      ux[j] = -A.u[3 * kk[j]]; uy[j] = -A.u[3 * kk[j] + 1]; uz[j] = -A.u[3 * kk[j] + 2];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && !two) break;
      const T mult = (m[j] == n && n == 0) ? mult0_of(A) : T(1);
      const T zc = (Pn + q[j]) * cc[j] * mult;
      const T w1 = wv[j][0] * zc, w2 = wv[j][1] * zc, w3 = wv[j][2] * zc;
      T sk[3], sy[5];
      skew_c(sk, ux[j], uy[j], uz[j]);
      sym_c(sy, ux[j], uy[j], uz[j]);
      acc[0] += w1;
#pragma unroll
      for (int i = 0; i < 3; ++i) acc[1 + i] += w2 * sk[i];
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[4 + i] += w3 * sy[i];
    }
  }
  if (fold_waves<T, 9, S>(acc, red) && on) stc(A.E + (size_t)n * A.H + h, A.nh, acc);
}

// ---------------------------------------------------------------- embedding backward
// destination pass: gP[n], gW[e'], gC[e'], gu[e'].  One wave per node covering all NB channel
// blocks, so the per-edge channel sums (gC, gu) finish inside the wave: plain stores, deterministic.
template <typename T, int NB, int S, typename AT = Args<T>>
__global__ __launch_bounds__(64 * S) void k_embed_bwd_dst(AT A) {
  TMD_RED(T, S > 1 ? (S - 1) * NB * TMD_WAVE : 1)
  zero_tail_rows(A, A.gW, 3 * A.H);
  zero_tail_rows(A, A.gC, 1);
  zero_tail_rows(A, A.gu, 3);
  const int n = blockIdx.x, w = threadIdx.x / TMD_WAVE;  // (the grid is one block per node)
  const int lane = lane_id();
  T g[NB][9], gPn[NB], Pn[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const int h = c * TMD_WAVE + lane;
    const int hc = h < A.H ? h : 0;
    ldc(g[c], A.gE + (size_t)n * A.H + hc, A.nh);
    Pn[c] = A.P[(size_t)n * A.H + hc];
    gPn[c] = T(0);
  }
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  // two edges per iteration (k, k + S): both edges' loads issued first, their eight wave sums interleaved
  for (int k = b + w; k < e; k += 2 * S) {
    const bool two = k + S < e;
    const int kk[2] = {k, two ? k + S : k};
    int m[2];
    T Ck[2], ux[2], uy[2], uz[2], qv[2][NB], wv[2][NB][3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      m[j] = A.src[kk[j]];
      TMD_DCHECK(m[j] >= 0 && m[j] < A.n);
      Ck[j] = A.C[kk[j]];
      ux[j] = -A.u[3 * kk[j]]; uy[j] = -A.u[3 * kk[j] + 1]; uz[j] = -A.u[3 * kk[j] + 2];
      const auto wr = A.W + (size_t)kk[j] * A.ldw;
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        const int h = c * TMD_WAVE + lane;
        const int hc = h < A.H ? h : 0;
        qv[j][c] = A.Q[(size_t)m[j] * A.H + hc];
        wv[j][c][0] = wr[hc]; wv[j][c][1] = wr[A.H + hc]; wv[j][c][2] = wr[2 * A.H + hc];
      }
    }
    T red4[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const T mult = (m[j] == n && n == 0) ? mult0_of(A) : T(1);
      const bool live = j == 0 || two;
      T sk[3], sy[5];
      skew_c(sk, ux[j], uy[j], uz[j]);
      sym_c(sy, ux[j], uy[j], uz[j]);
      const auto gw = A.gW + (size_t)kk[j] * 3 * A.H;
      T gc = T(0), gux = T(0), guy = T(0), guz = T(0);
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        const int h = c * TMD_WAVE + lane;
        const bool on = h < A.H;
        const T z = Pn[c] + qv[j][c];
        const T w1 = wv[j][c][0], w2 = wv[j][c][1], w3 = wv[j][c][2];
        const T g1 = g[c][0] * mult;
        const T g2 = (g[c][1] * sk[0] + g[c][2] * sk[1] + g[c][3] * sk[2]) * mult;
        const T g3 = (g[c][4] * sy[0] + g[c][5] * sy[1] + g[c][6] * sy[2] + g[c][7] * sy[3] +
                      g[c][8] * sy[4]) * mult;
        if (live) gPn[c] += (g1 * w1 + g2 * w2 + g3 * w3) * Ck[j];
        if (on && live) {
          gw[h] = g1 * z * Ck[j];
          gw[A.H + h] = g2 * z * Ck[j];
          gw[2 * A.H + h] = g3 * z * Ck[j];
        }
        if (on) {
          gc += (g1 * w1 + g2 * w2 + g3 * w3) * z;
          // gradient w.r.t. the row edge's u (= -u(n->m)): chain through the sign flip
          T dax, day, daz, dsx, dsy, dsz;
          dskew_c(&g[c][1], dax, day, daz);
          dsym_c(&g[c][4], ux[j], uy[j], uz[j], dsx, dsy, dsz);
          const T a2 = z * w2 * Ck[j] * mult, a3 = z * w3 * Ck[j] * mult;
          gux -= a2 * dax + a3 * dsx;
          guy -= a2 * day + a3 * dsy;
          guz -= a2 * daz + a3 * dsz;
        }
      }
      red4[j][0] = gc; red4[j][1] = gux; red4[j][2] = guy; red4[j][3] = guz;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) red4[j][i] = wave_sum(red4[j][i]);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j == 1 && !two) break;
        A.gC[kk[j]] = red4[j][0];
        A.gu[3 * kk[j]] = red4[j][1];
        A.gu[3 * kk[j] + 1] = red4[j][2];
        A.gu[3 * kk[j] + 2] = red4[j][3];
      }
    }
  }
  if (!fold_waves<T, NB, S>(gPn, red)) return;
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const int h = c * TMD_WAVE + lane;
    if (h < A.H) A.gP[(size_t)n * A.H + h] = gPn[c];
  }
}

// source pass: gQ[m] = sum over reversed edges of the same g_z
template <typename T, int S, typename AT = Args<T>>
__global__ __launch_bounds__(64 * S) void k_embed_bwd_src(AT A) {
  TMD_RED(T, S > 1 ? (S - 1) * TMD_WAVE : 1)
  int m, ch0, w;
  slot_node<S>(A.nblk, m, ch0, w);
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T gQm[1] = {T(0)};
  const int b = min(A.row_ptr[m], A.cap), e = min(A.row_ptr[m + 1], A.cap);
  // two edges per iteration (k, k + S), loads first
  for (int k = b + w; k < e; k += 2 * S) {
    const bool two = k + S < e;
    const int kk[2] = {k, two ? k + S : k};
    int nn[2];
    T g[2][9], wv[2][3], cc[2], u0[2], u1[2], u2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      nn[j] = A.src[kk[j]];  // row edge n->m; its reverse m->n contributed Q[m] to E[n]
      TMD_DCHECK(nn[j] >= 0 && nn[j] < A.n);
      ldc(g[j], A.gE + (size_t)nn[j] * A.H + hc, A.nh);
      const auto wr = A.W + (size_t)kk[j] * A.ldw;
      wv[j][0] = wr[hc]; wv[j][1] = wr[A.H + hc]; wv[j][2] = wr[2 * A.H + hc];
      cc[j] = A.C[kk[j]];
      u0[j] = A.u[3 * kk[j]]; u1[j] = A.u[3 * kk[j] + 1]; u2[j] = A.u[3 * kk[j] + 2];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && !two) break;
      const T mult = (m == nn[j] && nn[j] == 0) ? mult0_of(A) : T(1);
      // u of the reversed edge's own row edge (m->n as seen from row n) is -u(k); the embedding
      // used skew/sym of -(that) = u(k)
      T sk[3], sy[5];
      skew_c(sk, u0[j], u1[j], u2[j]);
      sym_c(sy, u0[j], u1[j], u2[j]);
      const T gg = g[j][0] * wv[j][0] + (g[j][1] * sk[0] + g[j][2] * sk[1] + g[j][3] * sk[2]) * wv[j][1] +
                   (g[j][4] * sy[0] + g[j][5] * sy[1] + g[j][6] * sy[2] + g[j][7] * sy[3] + g[j][8] * sy[4]) *
                       wv[j][2];
      gQm[0] += gg * cc[j] * mult;
    }
  }
  if (fold_waves<T, 1, S>(gQm, red) && on) A.gQ[(size_t)m * A.H + h] = gQm[0];
}

// ---------------------------------------------------------------- message passing
// The row's edges are taken in chunks of 64: lane i loads the chunk's i-th source index (and pair row) in
// ONE coalesced load, and each edge's indices are then broadcast by v_readlane (wave-uniform: the gathers'
// base addresses live in scalar registers).  Each wave takes two of its edges per iteration (j and j + S, the
// same edges and summation order as one at a time), so their 2 x 12 row loads are in flight together instead
// of a src -> row load chain per edge.
__device__ __forceinline__ int bcast(int v, int j) { return __builtin_amdgcn_readlane(v, j); }

template <typename T>
__device__ __forceinline__ void msg_acc(T (&acc)[9], const Args<T>& A, int n, int m, int r, int hc) {
  const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
  const T* er = A.ea + (size_t)r * A.ldea + 3 * hc;
  const T f0 = er[0] * mult, f1 = er[1] * mult, f2 = er[2] * mult;
  T t[9];
  ldc(t, A.Tc + (size_t)m * A.H + hc, A.nh);
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] += node::ctype_scale(i, f0, f1, f2) * t[i];
}

template <typename T, int S>
__global__ __launch_bounds__(64 * S) void k_msg_fwd(Args<T> A) {
  __shared__ T red[S > 1 ? (S - 1) * 9 * TMD_WAVE : 1];
  int n, ch0, w;
  slot_node<S>(A.nblk, n, ch0, w);
  const int lane = lane_id();
  const int h = ch0 + lane;
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = T(0);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int base = b; base < e; base += TMD_WAVE) {
    const int cnt = min(TMD_WAVE, e - base);
    const int sv = lane < cnt ? A.src[base + lane] : 0;
    const int rv = lane < cnt ? ea_row(A, base + lane) : 0;
    int j = w;
    for (; j + S < cnt; j += 2 * S) {
      const int ma = bcast(sv, j), mb = bcast(sv, j + S);
      TMD_DCHECK(ma >= 0 && ma < A.n && mb >= 0 && mb < A.n);
      msg_acc(acc, A, n, ma, bcast(rv, j), hc);
      msg_acc(acc, A, n, mb, bcast(rv, j + S), hc);
    }
    if (j < cnt) msg_acc(acc, A, n, bcast(sv, j), bcast(rv, j), hc);
  }
  if (fold_waves<T, 9, S>(acc, red) && on) stc(A.msg + (size_t)n * A.H + h, A.nh, acc);
}

// destination pass: gea[e'] = <gmsg[n], {I,A,S}[m]>
template <typename T, int S>
__global__ __launch_bounds__(64 * S) void k_msg_bwd_dst(Args<T> A) {
  zero_tail_rows(A, A.gea, 3 * A.H);
  int n, ch0, w;
  slot_node<S>(A.nblk, n, ch0, w);
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T g[9];
  ldc(g, A.gmsg + (size_t)n * A.H + hc, A.nh);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int k = b + w; k < e; k += S) {
    const int m = A.src[k];
    TMD_DCHECK(m >= 0 && m < A.n);
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    T t[9];
    ldc(t, A.Tc + (size_t)m * A.H + hc, A.nh);
    if (on) {
      T* gr = A.gea + (size_t)k * 3 * A.H + 3 * h;
      gr[0] = g[0] * t[0] * mult;
      gr[1] = (g[1] * t[1] + g[2] * t[2] + g[3] * t[3]) * mult;
      gr[2] = (g[4] * t[4] + g[5] * t[5] + g[6] * t[6] + g[7] * t[7] + g[8] * t[8]) * mult;
    }
  }
}

// pair-row destination pass: gea[p] = sum over the pair's two directions of <gmsg[dst], {I,A,S}[src]>, formed
// by the pair's canonical edge (row n, src m >= n; tmdnet_pair_index) from both endpoints' rows -- one write
// per pair instead of one per edge, no atomics.  Inert pair slots (static capacity) are zeroed.  The chunk's
// canonical edges are compacted per wave (ballot rank -> LDS), then taken two per iteration as above.
template <typename T>
__device__ __forceinline__ void pair_grad(const Args<T>& A, int n, int m, int r, int h, int hc, const T (&gn)[9],
                                          const T (&tn_)[9], bool on) {
  const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
  T g0, g1, g2;
  if (m == n) {  // self loop: one direction
    g0 = gn[0] * tn_[0];
    g1 = gn[1] * tn_[1] + gn[2] * tn_[2] + gn[3] * tn_[3];
    g2 = gn[4] * tn_[4] + gn[5] * tn_[5] + gn[6] * tn_[6] + gn[7] * tn_[7] + gn[8] * tn_[8];
  } else {
    T t[9], g[9];
    ldc(t, A.Tc + (size_t)m * A.H + hc, A.nh);
    ldc(g, A.gmsg + (size_t)m * A.H + hc, A.nh);
    g0 = gn[0] * t[0] + g[0] * tn_[0];
    g1 = gn[1] * t[1] + gn[2] * t[2] + gn[3] * t[3] + g[1] * tn_[1] + g[2] * tn_[2] + g[3] * tn_[3];
    g2 = gn[4] * t[4] + gn[5] * t[5] + gn[6] * t[6] + gn[7] * t[7] + gn[8] * t[8] +
         g[4] * tn_[4] + g[5] * tn_[5] + g[6] * tn_[6] + g[7] * tn_[7] + g[8] * tn_[8];
  }
  if (on) {
    T* gr = A.gea + (size_t)r * 3 * A.H + 3 * h;
    gr[0] = g0 * mult;
    gr[1] = g1 * mult;
    gr[2] = g2 * mult;
  }
}

template <typename T, int S>
__global__ __launch_bounds__(64 * S) void k_msg_bwd_pair(Args<T> A) {
  __shared__ int cs[S][TMD_WAVE], cr[S][TMD_WAVE];
  {
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
    const int w3 = 3 * A.H;
    for (long long i = tid; i < (long long)A.np * w3; i += nth) {
      const int p = (int)(i / w3);
      if (A.prow[A.pedge[p]] != p) A.gea[i] = T(0);
    }
  }
  int n, ch0, w;
  slot_node<S>(A.nblk, n, ch0, w);
  const int lane = lane_id();
  const int h = ch0 + lane;
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T gn[9], tn_[9];
  ldc(gn, A.gmsg + (size_t)n * A.H + hc, A.nh);
  ldc(tn_, A.Tc + (size_t)n * A.H + hc, A.nh);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int base = b; base < e; base += TMD_WAVE) {
    const int cnt = min(TMD_WAVE, e - base);
    const int sv = lane < cnt ? A.src[base + lane] : -1;
    const bool own = lane < cnt && sv >= n;  // the pair's other direction is formed by row sv
    const unsigned long long mask = __ballot(own);
    const int no = __popcll(mask);
    if (own) {
      const int rank = __popcll(mask & ((1ull << lane) - 1ull));
      cs[w][rank] = sv;
      cr[w][rank] = A.prow[base + lane];
    }
    __builtin_amdgcn_wave_barrier();
    int j = w;
    for (; j + S < no; j += 2 * S) {
      const int ma = __builtin_amdgcn_readfirstlane(cs[w][j]), mb = __builtin_amdgcn_readfirstlane(cs[w][j + S]);
      const int ra = __builtin_amdgcn_readfirstlane(cr[w][j]), rb = __builtin_amdgcn_readfirstlane(cr[w][j + S]);
      TMD_DCHECK(ma >= 0 && ma < A.n && mb >= 0 && mb < A.n);
      pair_grad(A, n, ma, ra, h, hc, gn, tn_, on);
      pair_grad(A, n, mb, rb, h, hc, gn, tn_, on);
    }
    if (j < no)
      pair_grad(A, n, __builtin_amdgcn_readfirstlane(cs[w][j]), __builtin_amdgcn_readfirstlane(cr[w][j]), h, hc, gn,
                tn_, on);
    __builtin_amdgcn_wave_barrier();  // (the next chunk's compaction rewrites cs / cr)
  }
}

// Pair rows, both backward roles in ONE pass over each row (the neighbours of n are the same set in both):
// per edge (n <- m) the wave gathers gmsg[m] and the pair's factor row once for the source role (gT[n] +=
// ea * gmsg[m]) and, when it is the pair's canonical edge (m >= n, a wave-uniform branch), T[m] for the pair's
// factor gradient (as k_msg_bwd_pair).  Replaces k_msg_bwd_pair + k_msg_bwd_src (gmsg rows gathered once).
template <typename T, int S>
__global__ __launch_bounds__(64 * S) void k_msg_bwd_fused(Args<T> A) {
  __shared__ T red[S > 1 ? (S - 1) * 9 * TMD_WAVE : 1];
  {
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
    const int w3 = 3 * A.H;
    for (long long i = tid; i < (long long)A.np * w3; i += nth) {
      const int p = (int)(i / w3);
      if (A.prow[A.pedge[p]] != p) A.gea[i] = T(0);
    }
  }
  int n, ch0, w;
  slot_node<S>(A.nblk, n, ch0, w);
  const int lane = lane_id();
  const int h = ch0 + lane;
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T gn[9], tn_[9], acc[9];
  ldc(gn, A.gmsg + (size_t)n * A.H + hc, A.nh);
  ldc(tn_, A.Tc + (size_t)n * A.H + hc, A.nh);
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = T(0);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int base = b; base < e; base += TMD_WAVE) {
    const int cnt = min(TMD_WAVE, e - base);
    const int sv = lane < cnt ? A.src[base + lane] : 0;
    const int rv = lane < cnt ? A.prow[base + lane] : 0;
    for (int j = w; j < cnt; j += S) {
      const int m = bcast(sv, j), r = bcast(rv, j);
      TMD_DCHECK(m >= 0 && m < A.n);
      const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
      const T* er = A.ea + (size_t)r * A.ldea + 3 * hc;
      const T f0 = er[0] * mult, f1 = er[1] * mult, f2 = er[2] * mult;
      T g[9];
      ldc(g, A.gmsg + (size_t)m * A.H + hc, A.nh);
      if (m >= n) {  // the pair's canonical edge: its factor gradient from both directions
        T g0, g1, g2;
        if (m == n) {
          g0 = gn[0] * tn_[0];
          g1 = gn[1] * tn_[1] + gn[2] * tn_[2] + gn[3] * tn_[3];
          g2 = gn[4] * tn_[4] + gn[5] * tn_[5] + gn[6] * tn_[6] + gn[7] * tn_[7] + gn[8] * tn_[8];
        } else {
          T t[9];
          ldc(t, A.Tc + (size_t)m * A.H + hc, A.nh);
          g0 = gn[0] * t[0] + g[0] * tn_[0];
          g1 = gn[1] * t[1] + gn[2] * t[2] + gn[3] * t[3] + g[1] * tn_[1] + g[2] * tn_[2] + g[3] * tn_[3];
          g2 = gn[4] * t[4] + gn[5] * t[5] + gn[6] * t[6] + gn[7] * t[7] + gn[8] * t[8] +
               g[4] * tn_[4] + g[5] * tn_[5] + g[6] * tn_[6] + g[7] * tn_[7] + g[8] * tn_[8];
        }
        if (on) {
          T* gr = A.gea + (size_t)r * 3 * A.H + 3 * h;
          gr[0] = g0 * mult;
          gr[1] = g1 * mult;
          gr[2] = g2 * mult;
        }
      }
#pragma unroll
      for (int i = 0; i < 9; ++i) acc[i] += node::ctype_scale(i, f0, f1, f2) * g[i];
    }
  }
  if (!fold_waves<T, 9, S>(acc, red)) return;
  if (A.gTadd && on) {
    T ad[9];
    ldc(ad, A.gTadd + (size_t)n * A.H + h, A.nh);
#pragma unroll
    for (int i = 0; i < 9; ++i) acc[i] += ad[i];
  }
  if (on) stc(A.gT + (size_t)n * A.H + h, A.nh, acc);
}

// source pass: gT[m] = sum over reversed edges ea * gmsg[n]
template <typename T>
__device__ __forceinline__ void src_acc(T (&acc)[9], const Args<T>& A, int m, int n, int r, int hc) {
  const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
  const T* er = A.ea + (size_t)r * A.ldea + 3 * hc;
  const T f0 = er[0] * mult, f1 = er[1] * mult, f2 = er[2] * mult;
  T g[9];
  ldc(g, A.gmsg + (size_t)n * A.H + hc, A.nh);
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] += node::ctype_scale(i, f0, f1, f2) * g[i];
}

template <typename T, int S>
__global__ __launch_bounds__(64 * S) void k_msg_bwd_src(Args<T> A) {
  __shared__ T red[S > 1 ? (S - 1) * 9 * TMD_WAVE : 1];
  int m, ch0, w;
  slot_node<S>(A.nblk, m, ch0, w);
  const int lane = lane_id();
  const int h = ch0 + lane;
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = T(0);
  const int b = min(A.row_ptr[m], A.cap), e = min(A.row_ptr[m + 1], A.cap);
  for (int base = b; base < e; base += TMD_WAVE) {
    const int cnt = min(TMD_WAVE, e - base);
    const int sv = lane < cnt ? A.src[base + lane] : 0;
    const int rv = lane < cnt ? ea_row(A, base + lane) : 0;
    int j = w;
    for (; j + S < cnt; j += 2 * S) {
      const int na = bcast(sv, j), nb = bcast(sv, j + S);
      TMD_DCHECK(na >= 0 && na < A.n && nb >= 0 && nb < A.n);
      src_acc(acc, A, m, na, bcast(rv, j), hc);
      src_acc(acc, A, m, nb, bcast(rv, j + S), hc);
    }
    if (j < cnt) src_acc(acc, A, m, bcast(sv, j), bcast(rv, j), hc);
  }
  if (!fold_waves<T, 9, S>(acc, red)) return;
  if (A.gTadd && on) {
    T ad[9];
    ldc(ad, A.gTadd + (size_t)m * A.H + h, A.nh);
#pragma unroll
    for (int i = 0; i < 9; ++i) acc[i] += ad[i];
  }
  if (on) stc(A.gT + (size_t)m * A.H + h, A.nh, acc);
}

// waves per (node, channel block): TMDNET_TN_S (A/B switch; 1, 2 or 4, default 4), read once per process
// (not per launch: the launch-bound C3 step, and a captured graph must not change form behind its back)
static int slots() {
  static const int s = [] {
    const char* e = getenv("TMDNET_TN_S");
    const int v = e ? atoi(e) : 4;
    return v >= 4 ? 4 : v >= 2 ? 2 : 1;
  }();
  return s;
}

// one S-wave block per (node, channel block) of A.nblk
template <typename T, template <typename, int> class K>
static int launch_s(const Args<T>& A, hipStream_t st) {
  if (A.n <= 0) return kOk;
  const dim3 g((unsigned)((long long)A.n * A.nblk));
  switch (slots()) {
    case 1: hipLaunchKernelGGL((K<T, 1>::fn), g, dim3(64), 0, st, A); break;
    case 2: hipLaunchKernelGGL((K<T, 2>::fn), g, dim3(128), 0, st, A); break;
    default: hipLaunchKernelGGL((K<T, 4>::fn), g, dim3(256), 0, st, A); break;
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
#define TMD_TN_KERNEL(NAME)                                          \
  template <typename T, int S> struct NAME##_k {                     \
    static constexpr void (*fn)(Args<T>) = NAME<T, S>;               \
  };
TMD_TN_KERNEL(k_embed_fwd)
TMD_TN_KERNEL(k_embed_bwd_src)
TMD_TN_KERNEL(k_msg_fwd)
TMD_TN_KERNEL(k_msg_bwd_dst)
TMD_TN_KERNEL(k_msg_bwd_src)
TMD_TN_KERNEL(k_msg_bwd_pair)
TMD_TN_KERNEL(k_msg_bwd_fused)
#undef TMD_TN_KERNEL

template <typename T> static int launch_embed_fwd(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_embed_fwd_k>(A, st);
}
template <typename T> static int launch_embed_bwd_src(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_embed_bwd_src_k>(A, st);
}
template <typename T> static int launch_msg_fwd(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_msg_fwd_k>(A, st);
}
template <typename T> static int launch_msg_bwd_dst(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_msg_bwd_dst_k>(A, st);
}
template <typename T> static int launch_msg_bwd_src(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_msg_bwd_src_k>(A, st);
}
template <typename T> static int launch_msg_bwd_fused(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_msg_bwd_fused_k>(A, st);
}
template <typename T> static int launch_msg_bwd_pair(const Args<T>& A, hipStream_t st) {
  return launch_s<T, k_msg_bwd_pair_k>(A, st);
}

// the embedding destination pass: one S-wave block per node (each wave covers every channel block)
template <typename T>
static int launch_embed_bwd_dst(const Args<T>& A, hipStream_t st) {
  if (A.n <= 0) return kOk;
  const dim3 g((unsigned)A.n);
  // its per-edge channel sums make each edge a longer chain than in the other kernels: 8 waves per node on
  // small systems (C3: 9.4 vs 13.3 us at 4), 2 on large ones, where the nodes alone fill the chip (C5 TensorNet,
  // 50k atoms: 31.5 vs 32.2-32.8 ms per evaluation, tools/tn_c5_time.py); TMDNET_TN_EBD_S = 1 / 2 / 4 / 8 for A/B
  static const int env_s = [] {  // read once per process (as slots())
    const char* e8 = getenv("TMDNET_TN_EBD_S");
    const int v = e8 ? atoi(e8) : 0;
    return v <= 0 ? 0 : v >= 8 ? 8 : v >= 4 ? 4 : v >= 2 ? 2 : 1;
  }();
  const int s = env_s ? env_s : (A.n < 8192 ? 8 : 2);
#define TMD_EBD(NB)                                                                                   \
  if (s == 1) hipLaunchKernelGGL((k_embed_bwd_dst<T, NB, 1>), g, dim3(64), 0, st, A);                 \
  else if (s == 2) hipLaunchKernelGGL((k_embed_bwd_dst<T, NB, 2>), g, dim3(128), 0, st, A);           \
  else if (s == 4) hipLaunchKernelGGL((k_embed_bwd_dst<T, NB, 4>), g, dim3(256), 0, st, A);           \
  else hipLaunchKernelGGL((k_embed_bwd_dst<T, NB, 8>), g, dim3(512), 0, st, A);
  if (A.nblk == 1) { TMD_EBD(1) }
  else if (A.nblk == 2) { TMD_EBD(2) }
  else if (A.nblk <= 4) { TMD_EBD(4) }
  else return kUnsupported;
#undef TMD_EBD
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static Args<T> base(int n, int H, const int32_t* row_ptr, const int32_t* src, int cap, double mult0,
                    const int32_t* npd, int padcap) {
  Args<T> A{};
  A.n = n; A.H = H; A.nblk = (H + TMD_WAVE - 1) / TMD_WAVE; A.cap = cap; A.mult0 = (T)mult0;
  A.nh = (size_t)n * H;
  A.npd = npd; A.padcap = padcap;
  A.row_ptr = row_ptr; A.src = src;
  return A;
}

}  // namespace tn
}  // namespace tmd

using namespace tmd;

#define TN_DISPATCH(dtype, BODY)                  \
  if ((dtype) == TMDNET_F32) {                    \
    using T = float;                              \
    BODY                                          \
  } else if ((dtype) == TMDNET_F64) {             \
    using T = double;                             \
    BODY                                          \
  } else {                                        \
    return kUnsupported;                          \
  }

extern "C" int tmdnet_tn_embed_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                   const int32_t* src, int max_pairs, double self0_mult,
                                   const int32_t* pad_pairs, int pad_capacity,
                                   const void* P, const void* Q, const void* W, int ld_w,
                                   const void* cutoff, const void* unit, void* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                         pad_capacity);
    a.P = (const T*)P; a.Q = (const T*)Q; a.W = (const T*)W; a.ldw = ld_w;
    a.C = (const T*)cutoff; a.u = (const T*)unit; a.E = (T*)out;
    return tn::launch_embed_fwd<T>(a, st);
  })
}

extern "C" int tmdnet_tn_embed_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                   const int32_t* src, int max_pairs, double self0_mult,
                                   const int32_t* pad_pairs, int pad_capacity,
                                   const void* P, const void* Q, const void* W, int ld_w,
                                   const void* cutoff, const void* unit, const void* grad_out,
                                   void* gP, void* gQ, void* gW, void* gcut, void* gunit,
                                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                         pad_capacity);
    a.P = (const T*)P; a.Q = (const T*)Q; a.W = (const T*)W; a.ldw = ld_w;
    a.C = (const T*)cutoff; a.u = (const T*)unit;
    a.gE = (const T*)grad_out;
    a.gP = (T*)gP; a.gQ = (T*)gQ; a.gW = (T*)gW; a.gC = (T*)gcut; a.gu = (T*)gunit;
    const int rc = tn::launch_embed_bwd_dst<T>(a, st);  // (each wave covers every channel block)
    if (rc) return rc;
    return tn::launch_embed_bwd_src<T>(a, st);
  })
}

extern "C" int tmdnet_tn_message_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                     const int32_t* src, int max_pairs, double self0_mult,
                                     const int32_t* pad_pairs, int pad_capacity,
                                     const void* edge_attr, int ld_ea, const void* comp, void* msg,
                                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                         pad_capacity);
    a.ea = (const T*)edge_attr; a.ldea = ld_ea;
    a.Tc = (const T*)comp; a.msg = (T*)msg;
    return tn::launch_msg_fwd<T>(a, st);
  })
}

extern "C" int tmdnet_tn_message_bwd_add(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                         const int32_t* src, int max_pairs, double self0_mult,
                                         const int32_t* pad_pairs, int pad_capacity,
                                         const void* edge_attr, int ld_ea, const void* comp,
                                         const void* grad_msg, const void* g_comp_add, void* g_edge_attr,
                                         void* g_comp, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                         pad_capacity);
    a.ea = (const T*)edge_attr; a.ldea = ld_ea;
    a.Tc = (const T*)comp;
    a.gmsg = (const T*)grad_msg; a.gea = (T*)g_edge_attr; a.gT = (T*)g_comp;
    a.gTadd = (const T*)g_comp_add;
    int rc = tn::launch_msg_bwd_dst<T>(a, st);
    if (rc) return rc;
    return tn::launch_msg_bwd_src<T>(a, st);
  })
}

extern "C" int tmdnet_tn_message_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                     const int32_t* src, int max_pairs, double self0_mult,
                                     const int32_t* pad_pairs, int pad_capacity,
                                     const void* edge_attr, int ld_ea, const void* comp,
                                     const void* grad_msg, void* g_edge_attr, void* g_comp,
                                     void* stream) {
  return tmdnet_tn_message_bwd_add(dtype, n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                                   pad_capacity, edge_attr, ld_ea, comp, grad_msg, nullptr, g_edge_attr, g_comp,
                                   stream);
}

// Pair-row forms of the message (large systems): edge_attr / g_edge_attr hold one row per pair slot of
// tmdnet_pair_index (pair_row [E] -> slot, pair_edge [n_pair_slots] -> canonical edge).
extern "C" int tmdnet_tn_message_fwd_pairs(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                           const int32_t* src, int max_pairs, double self0_mult,
                                           const int32_t* pad_pairs, int pad_capacity, const int32_t* pair_row,
                                           const void* edge_attr, int ld_ea, const void* comp, void* msg,
                                           void* stream) {
  if (!pair_row) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs, pad_capacity);
    a.prow = pair_row;
    a.ea = (const T*)edge_attr; a.ldea = ld_ea;
    a.Tc = (const T*)comp; a.msg = (T*)msg;
    return tn::launch_msg_fwd<T>(a, st);
  })
}

extern "C" int tmdnet_tn_message_bwd_pairs(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                           const int32_t* src, int max_pairs, double self0_mult,
                                           const int32_t* pad_pairs, int pad_capacity, const int32_t* pair_row,
                                           const int32_t* pair_edge, int n_pair_slots, const void* edge_attr,
                                           int ld_ea, const void* comp, const void* grad_msg,
                                           const void* g_comp_add, void* g_edge_attr, void* g_comp, void* stream) {
  if (!pair_row || !pair_edge || n_pair_slots < 0) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs, pad_capacity);
    a.prow = pair_row; a.pedge = pair_edge; a.np = n_pair_slots;
    a.ea = (const T*)edge_attr; a.ldea = ld_ea;
    a.Tc = (const T*)comp;
    a.gmsg = (const T*)grad_msg; a.gea = (T*)g_edge_attr; a.gT = (T*)g_comp;
    a.gTadd = (const T*)g_comp_add;
    // TMDNET_TN_BWD_FUSED=1: both roles in one pass (k_msg_bwd_fused; measured equal at C5: 32.5-33.0 vs
    // 32.7-32.8 ms per evaluation, so the two-kernel form stays the default)
    static const bool fused = [] {
      const char* e = getenv("TMDNET_TN_BWD_FUSED");
      return e && atoi(e) == 1;
    }();
    if (fused && g_edge_attr && g_comp) return tn::launch_msg_bwd_fused<T>(a, st);
    int rc = g_edge_attr ? tn::launch_msg_bwd_pair<T>(a, st) : kOk;
    if (rc) return rc;
    return g_comp ? tn::launch_msg_bwd_src<T>(a, st) : kOk;
  })
}

// Second order of the embedding (forward-over-reverse on dual numbers, as tmdnet_tn_node_bwd2): with the
// first backward (gP, gQ, gW, gcut, gunit) = J^T(theta) gE, theta = (P, Q, W, cut, unit), its VJP for the
// cotangents t_theta of those outputs is
//   d_gE      = J(theta) t_theta                   -- the forward kernel on theta + eps t_theta (eps part)
//   d_theta   = H_<gE, E>(theta) t_theta           -- the first backward on theta + eps t_theta, gE fixed
// (the Hessian of <gE, E(theta)> is symmetric).  The kernels are the first-order ones instantiated on
// node::Dual<T> with value / tangent pointer pairs; a NULL tangent is 0, a NULL output is not written.
namespace tmd {
namespace tn {
template <typename T>
static int embed_bwd2(int n_nodes, int hidden, const int32_t* row_ptr, const int32_t* src, int max_pairs,
                      double self0_mult, const int32_t* pad_pairs, int pad_capacity, const void* P, const void* Q,
                      const void* W, int ld_w, const void* cutoff, const void* unit, const void* grad_out,
                      const void* tP, const void* tQ, const void* tW, const void* tcut, const void* tunit,
                      void* d_grad_out, void* dP, void* dQ, void* dW, void* dcut, void* dunit, hipStream_t st) {
  using D = node::Dual<T>;
  using DI = node::DIn<T>;
  using DO = node::DOut<T>;
  using DA = ArgsT<D, DI, DO>;
  DA a{};
  a.n = n_nodes; a.H = hidden; a.nblk = (hidden + TMD_WAVE - 1) / TMD_WAVE; a.cap = max_pairs;
  a.mult0 = D(self0_mult); a.nh = (size_t)n_nodes * hidden; a.npd = pad_pairs; a.padcap = pad_capacity;
  a.row_ptr = row_ptr; a.src = src;
  a.P = DI{(const T*)P, (const T*)tP}; a.Q = DI{(const T*)Q, (const T*)tQ};
  a.W = DI{(const T*)W, (const T*)tW}; a.ldw = ld_w;
  a.C = DI{(const T*)cutoff, (const T*)tcut}; a.u = DI{(const T*)unit, (const T*)tunit};
  a.gE = DI{(const T*)grad_out, nullptr};
  a.E = DO{nullptr, (T*)d_grad_out};
  a.gP = DO{nullptr, (T*)dP}; a.gQ = DO{nullptr, (T*)dQ}; a.gW = DO{nullptr, (T*)dW};
  a.gC = DO{nullptr, (T*)dcut}; a.gu = DO{nullptr, (T*)dunit};
  const dim3 gs((unsigned)((long long)n_nodes * a.nblk));
  if (d_grad_out) hipLaunchKernelGGL((k_embed_fwd<D, 4, DA>), gs, dim3(256), 0, st, a);
  if (dP || dW || dcut || dunit) {
    const dim3 g((unsigned)n_nodes);
    if (a.nblk == 1) hipLaunchKernelGGL((k_embed_bwd_dst<D, 1, 4, DA>), g, dim3(256), 0, st, a);
    else if (a.nblk == 2) hipLaunchKernelGGL((k_embed_bwd_dst<D, 2, 4, DA>), g, dim3(256), 0, st, a);
    else if (a.nblk <= 4) hipLaunchKernelGGL((k_embed_bwd_dst<D, 4, 4, DA>), g, dim3(256), 0, st, a);
    else return kUnsupported;
  }
  if (dQ) hipLaunchKernelGGL((k_embed_bwd_src<D, 4, DA>), gs, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
}  // namespace tn
}  // namespace tmd

extern "C" int tmdnet_tn_embed_bwd2(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                    const int32_t* src, int max_pairs, double self0_mult,
                                    const int32_t* pad_pairs, int pad_capacity, const void* P, const void* Q,
                                    const void* W, int ld_w, const void* cutoff, const void* unit,
                                    const void* grad_out, const void* tP, const void* tQ, const void* tW,
                                    const void* tcut, const void* tunit, void* d_grad_out, void* dP, void* dQ,
                                    void* dW, void* dcut, void* dunit, void* stream) {
  if (n_nodes <= 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return tn::embed_bwd2<float>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs, pad_capacity, P, Q,
                                 W, ld_w, cutoff, unit, grad_out, tP, tQ, tW, tcut, tunit, d_grad_out, dP, dQ, dW,
                                 dcut, dunit, st);
  if (dtype == TMDNET_F64)
    return tn::embed_bwd2<double>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs, pad_capacity, P,
                                  Q, W, ld_w, cutoff, unit, grad_out, tP, tQ, tW, tcut, tunit, d_grad_out, dP, dQ, dW,
                                  dcut, dunit, st);
  return kUnsupported;
}
