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
// Tensors are (N, H, 3, 3) row-major: a lane owns one channel's 9 contiguous values.
// `mult0` (>= 1) is the multiplicity of atom 0's self loop: the reference's static_shapes mode
// turns every (-1,-1) padding slot of the CUDA neighbour list into an extra (0,0) edge with r = 0
// (tensornet.py:215-221), i.e. (max_num_pairs - num_pairs) more copies of that self loop.
// Backward = destination pass (own outputs + per-edge grads) + source pass (gathered inputs' grads).
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace tn {

template <typename T> struct M3 {
  T v[9];
};

template <typename T> __device__ __forceinline__ void ld9(T (&o)[9], const T* p) {
#pragma unroll
  for (int i = 0; i < 9; ++i) o[i] = p[i];
}
template <typename T> __device__ __forceinline__ void st9(T* p, const T (&o)[9]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) p[i] = o[i];
}

// skew(v) = [[0,-v2,v1],[v2,0,-v0],[-v1,v0,0]]  (tensornet.py:16-34)
template <typename T> __device__ __forceinline__ void skew(T (&m)[9], T x, T y, T z) {
  m[0] = T(0); m[1] = -z; m[2] = y;
  m[3] = z; m[4] = T(0); m[5] = -x;
  m[6] = -y; m[7] = x; m[8] = T(0);
}
// sym(v) = v v^T - |v|^2/3 Id  (tensornet.py:37-44)
template <typename T> __device__ __forceinline__ void symm(T (&m)[9], T x, T y, T z) {
  const T tr = (x * x + y * y + z * z) / T(3);
  m[0] = x * x - tr; m[1] = x * y; m[2] = x * z;
  m[3] = y * x; m[4] = y * y - tr; m[5] = y * z;
  m[6] = z * x; m[7] = z * y; m[8] = z * z - tr;
}
// d<G, skew(v)>/dv
template <typename T> __device__ __forceinline__ void dskew(const T (&g)[9], T& dx, T& dy, T& dz) {
  dx = g[7] - g[5];
  dy = g[2] - g[6];
  dz = g[3] - g[1];
}
// d<G, sym(v)>/dv = (G + G^T) v - 2 v tr(G) / 3
template <typename T>
__device__ __forceinline__ void dsymm(const T (&g)[9], T x, T y, T z, T& dx, T& dy, T& dz) {
  const T tr = (g[0] + g[4] + g[8]) * (T(2) / T(3));
  dx = (g[0] + g[0]) * x + (g[1] + g[3]) * y + (g[2] + g[6]) * z - tr * x;
  dy = (g[3] + g[1]) * x + (g[4] + g[4]) * y + (g[5] + g[7]) * z - tr * y;
  dz = (g[6] + g[2]) * x + (g[7] + g[5]) * y + (g[8] + g[8]) * z - tr * z;
}
template <typename T> struct Args;
// Multiplicity of atom 0's self loop.  With a device pair count (static_shapes under HIP-graph
// capture) it is computed here: 1 + (reference padding capacity - pairs found), a uniform scalar load.
template <typename T> __device__ __forceinline__ T mult0_of(const Args<T>& A);

template <typename T> __device__ __forceinline__ T dot9(const T (&a)[9], const T (&b)[9]) {
  T s = T(0);
#pragma unroll
  for (int i = 0; i < 9; ++i) s += a[i] * b[i];
  return s;
}

template <typename T> struct Args {
  int n, H, nblk, cap;
  T mult0;
  const int32_t* npd;  // device num_pairs: mult0 = 1 + max(0, padcap - *npd) (HIP-graph capturable)
  int padcap;
  const int32_t* row_ptr;
  const int32_t* src;
  // embedding
  const T* P; const T* Q;   // [N][H]
  const T* W; int ldw;      // [E][3H] (W1 | W2 | W3), pre-cutoff
  const T* C;               // [E]
  const T* u;               // [E][3]
  T* I; T* A; T* S;         // [N][H][9]
  const T* gI; const T* gA; const T* gS;
  T* gP; T* gQ; T* gW; T* gC; T* gu;
  // message
  const T* ea; int ldea;    // [E][3H] interleaved (h, c)
  const T* Ti; const T* Ta; const T* Ts;  // [N][H][9]
  T* msg;
  const T* gmsg;
  T* gea; T* gTi; T* gTa; T* gTs;
};

template <typename T> __device__ __forceinline__ T mult0_of(const Args<T>& A) {
  if (A.npd == nullptr) return A.mult0;
  const int pad = A.padcap - __builtin_amdgcn_readfirstlane(A.npd[0]);
  return T(1 + (pad > 0 ? pad : 0));
}

__device__ __forceinline__ void wave_node(int nblk, int& node, int& ch0) {
  const int w = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  node = w / nblk;
  ch0 = (w % nblk) * TMD_WAVE;
}

// ---------------------------------------------------------------- embedding forward
template <typename T>
__global__ __launch_bounds__(256) void k_embed_fwd(Args<T> A) {
  int n, ch0;
  wave_node(A.nblk, n, ch0);
  if (n >= A.n) return;
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  const T Pn = A.P[(size_t)n * A.H + hc];
  T aI = T(0), aA[9], aS[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) { aA[i] = T(0); aS[i] = T(0); }
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int k = b; k < e; ++k) {
    const int m = A.src[k];
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    const T zc = (Pn + A.Q[(size_t)m * A.H + hc]) * A.C[k] * mult;
    const T* wr = A.W + (size_t)k * A.ldw;
    const T w1 = wr[hc], w2 = wr[A.H + hc], w3 = wr[2 * A.H + hc];
    const T ux = -A.u[3 * k], uy = -A.u[3 * k + 1], uz = -A.u[3 * k + 2];
    T sk[9], sy[9];
    skew(sk, ux, uy, uz);
    symm(sy, ux, uy, uz);
    aI += zc * w1;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      aA[i] += zc * w2 * sk[i];
      aS[i] += zc * w3 * sy[i];
    }
  }
  if (on) {
    const size_t o = ((size_t)n * A.H + h) * 9;
    T mI[9] = {aI, T(0), T(0), T(0), aI, T(0), T(0), T(0), aI};
    st9(A.I + o, mI);
    st9(A.A + o, aA);
    st9(A.S + o, aS);
  }
}

// ---------------------------------------------------------------- embedding backward
// destination pass: gP[n], gW[e'], gC[e'], gu[e'].  One wave per node covering all NB channel
// blocks, so the per-edge channel sums (gC, gu) finish inside the wave: plain stores, deterministic.
template <typename T, int NB>
__global__ __launch_bounds__(256) void k_embed_bwd_dst(Args<T> A) {
  const int n = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (n >= A.n) return;
  const int lane = lane_id();
  T gi[NB], gPn[NB];
  T gA[NB][9], gS[NB][9];
  T Pn[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const int h = c * TMD_WAVE + lane;
    const int hc = h < A.H ? h : 0;
    const size_t o = ((size_t)n * A.H + hc) * 9;
    T gI[9];
    ld9(gI, A.gI + o);
    ld9(gA[c], A.gA + o);
    ld9(gS[c], A.gS + o);
    gi[c] = gI[0] + gI[4] + gI[8];
    Pn[c] = A.P[(size_t)n * A.H + hc];
    gPn[c] = T(0);
  }
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int k = b; k < e; ++k) {
    const int m = A.src[k];
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    const T Ck = A.C[k];
    const T ux = -A.u[3 * k], uy = -A.u[3 * k + 1], uz = -A.u[3 * k + 2];
    T sk[9], sy[9];
    skew(sk, ux, uy, uz);
    symm(sy, ux, uy, uz);
    const T* wr = A.W + (size_t)k * A.ldw;
    T* gw = A.gW + (size_t)k * 3 * A.H;
    T gc = T(0), gux = T(0), guy = T(0), guz = T(0);
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      const int h = c * TMD_WAVE + lane;
      const bool on = h < A.H;
      const int hc = on ? h : 0;
      const T z = Pn[c] + A.Q[(size_t)m * A.H + hc];
      const T w1 = wr[hc], w2 = wr[A.H + hc], w3 = wr[2 * A.H + hc];
      const T g1 = gi[c] * mult, g2 = dot9(gA[c], sk) * mult, g3 = dot9(gS[c], sy) * mult;
      gPn[c] += (g1 * w1 + g2 * w2 + g3 * w3) * Ck;
      if (on) {
        gw[h] = g1 * z * Ck;
        gw[A.H + h] = g2 * z * Ck;
        gw[2 * A.H + h] = g3 * z * Ck;
        gc += (g1 * w1 + g2 * w2 + g3 * w3) * z;
        // gradient w.r.t. the row edge's u (= -u(n->m)): chain through the sign flip
        T dax, day, daz, dsx, dsy, dsz;
        dskew(gA[c], dax, day, daz);
        dsymm(gS[c], ux, uy, uz, dsx, dsy, dsz);
        const T a2 = z * w2 * Ck * mult, a3 = z * w3 * Ck * mult;
        gux -= a2 * dax + a3 * dsx;
        guy -= a2 * day + a3 * dsy;
        guz -= a2 * daz + a3 * dsz;
      }
    }
    gc = wave_sum(gc);
    gux = wave_sum(gux);
    guy = wave_sum(guy);
    guz = wave_sum(guz);
    if (lane == 0) {
      A.gC[k] = gc;
      A.gu[3 * k] = gux;
      A.gu[3 * k + 1] = guy;
      A.gu[3 * k + 2] = guz;
    }
  }
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const int h = c * TMD_WAVE + lane;
    if (h < A.H) A.gP[(size_t)n * A.H + h] = gPn[c];
  }
}

// source pass: gQ[m] = sum over reversed edges of the same g_z
template <typename T>
__global__ __launch_bounds__(256) void k_embed_bwd_src(Args<T> A) {
  int m, ch0;
  wave_node(A.nblk, m, ch0);
  if (m >= A.n) return;
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T gQm = T(0);
  const int b = min(A.row_ptr[m], A.cap), e = min(A.row_ptr[m + 1], A.cap);
  for (int k = b; k < e; ++k) {
    const int n = A.src[k];  // row edge n->m; its reverse m->n contributed Q[m] to I/A/S[n]
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    const size_t o = ((size_t)n * A.H + hc) * 9;
    T gI[9], gA[9], gS[9];
    ld9(gI, A.gI + o);
    ld9(gA, A.gA + o);
    ld9(gS, A.gS + o);
    // u of the reversed edge's own row edge (m->n as seen from row n) is -u(k); the embedding
    // used skew/sym of -(that) = u(k)
    const T ux = A.u[3 * k], uy = A.u[3 * k + 1], uz = A.u[3 * k + 2];
    T sk[9], sy[9];
    skew(sk, ux, uy, uz);
    symm(sy, ux, uy, uz);
    const T* wr = A.W + (size_t)k * A.ldw;
    const T w1 = wr[hc], w2 = wr[A.H + hc], w3 = wr[2 * A.H + hc];
    const T g = (gI[0] + gI[4] + gI[8]) * w1 + dot9(gA, sk) * w2 + dot9(gS, sy) * w3;
    gQm += g * A.C[k] * mult;
  }
  if (on) A.gQ[(size_t)m * A.H + h] = gQm;
}

// ---------------------------------------------------------------- message passing
template <typename T>
__global__ __launch_bounds__(256) void k_msg_fwd(Args<T> A) {
  int n, ch0;
  wave_node(A.nblk, n, ch0);
  if (n >= A.n) return;
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T acc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] = T(0);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int k = b; k < e; ++k) {
    const int m = A.src[k];
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    const T* er = A.ea + (size_t)k * A.ldea + 3 * hc;
    const T f0 = er[0] * mult, f1 = er[1] * mult, f2 = er[2] * mult;
    const size_t o = ((size_t)m * A.H + hc) * 9;
    T ti[9], ta[9], ts[9];
    ld9(ti, A.Ti + o);
    ld9(ta, A.Ta + o);
    ld9(ts, A.Ts + o);
#pragma unroll
    for (int i = 0; i < 9; ++i) acc[i] += f0 * ti[i] + f1 * ta[i] + f2 * ts[i];
  }
  if (on) st9(A.msg + ((size_t)n * A.H + h) * 9, acc);
}

// destination pass: gea[e'] = <gmsg[n], {I,A,S}[m]>
template <typename T>
__global__ __launch_bounds__(256) void k_msg_bwd_dst(Args<T> A) {
  int n, ch0;
  wave_node(A.nblk, n, ch0);
  if (n >= A.n) return;
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T g[9];
  ld9(g, A.gmsg + ((size_t)n * A.H + hc) * 9);
  const int b = min(A.row_ptr[n], A.cap), e = min(A.row_ptr[n + 1], A.cap);
  for (int k = b; k < e; ++k) {
    const int m = A.src[k];
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    const size_t o = ((size_t)m * A.H + hc) * 9;
    T ti[9], ta[9], ts[9];
    ld9(ti, A.Ti + o);
    ld9(ta, A.Ta + o);
    ld9(ts, A.Ts + o);
    if (on) {
      T* gr = A.gea + (size_t)k * 3 * A.H + 3 * h;
      gr[0] = dot9(g, ti) * mult;
      gr[1] = dot9(g, ta) * mult;
      gr[2] = dot9(g, ts) * mult;
    }
  }
}

// source pass: g{I,A,S}[m] = sum over reversed edges ea * gmsg[n]
template <typename T>
__global__ __launch_bounds__(256) void k_msg_bwd_src(Args<T> A) {
  int m, ch0;
  wave_node(A.nblk, m, ch0);
  if (m >= A.n) return;
  const int h = ch0 + lane_id();
  const bool on = h < A.H;
  const int hc = on ? h : 0;
  T ai[9], aa[9], as[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) { ai[i] = T(0); aa[i] = T(0); as[i] = T(0); }
  const int b = min(A.row_ptr[m], A.cap), e = min(A.row_ptr[m + 1], A.cap);
  for (int k = b; k < e; ++k) {
    const int n = A.src[k];
    const T mult = (m == n && n == 0) ? mult0_of(A) : T(1);
    const T* er = A.ea + (size_t)k * A.ldea + 3 * hc;
    const T f0 = er[0] * mult, f1 = er[1] * mult, f2 = er[2] * mult;
    T g[9];
    ld9(g, A.gmsg + ((size_t)n * A.H + hc) * 9);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      ai[i] += f0 * g[i];
      aa[i] += f1 * g[i];
      as[i] += f2 * g[i];
    }
  }
  if (on) {
    const size_t o = ((size_t)m * A.H + h) * 9;
    st9(A.gTi + o, ai);
    st9(A.gTa + o, aa);
    st9(A.gTs + o, as);
  }
}

template <typename T>
static int launch(void (*k)(Args<T>), const Args<T>& A, hipStream_t st) {
  if (A.n <= 0) return kOk;
  const long long waves = (long long)A.n * A.nblk;
  const int tb = 256, wpb = tb / TMD_WAVE;
  hipLaunchKernelGGL(k, dim3((unsigned)((waves + wpb - 1) / wpb)), dim3(tb), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static Args<T> base(int n, int H, const int32_t* row_ptr, const int32_t* src, int cap, double mult0,
                    const int32_t* npd, int padcap) {
  Args<T> A{};
  A.n = n; A.H = H; A.nblk = (H + TMD_WAVE - 1) / TMD_WAVE; A.cap = cap; A.mult0 = (T)mult0;
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
                                   const void* cutoff, const void* unit, void* I, void* A, void* S,
                                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                                 pad_capacity);
    a.P = (const T*)P; a.Q = (const T*)Q; a.W = (const T*)W; a.ldw = ld_w;
    a.C = (const T*)cutoff; a.u = (const T*)unit; a.I = (T*)I; a.A = (T*)A; a.S = (T*)S;
    return tn::launch<T>(tn::k_embed_fwd<T>, a, st);
  })
}

extern "C" int tmdnet_tn_embed_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                   const int32_t* src, int max_pairs, double self0_mult,
                                   const int32_t* pad_pairs, int pad_capacity,
                                   const void* P, const void* Q, const void* W, int ld_w,
                                   const void* cutoff, const void* unit, const void* gI,
                                   const void* gA, const void* gS, void* gP, void* gQ, void* gW,
                                   void* gcut, void* gunit, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                                 pad_capacity);
    a.P = (const T*)P; a.Q = (const T*)Q; a.W = (const T*)W; a.ldw = ld_w;
    a.C = (const T*)cutoff; a.u = (const T*)unit;
    a.gI = (const T*)gI; a.gA = (const T*)gA; a.gS = (const T*)gS;
    a.gP = (T*)gP; a.gQ = (T*)gQ; a.gW = (T*)gW; a.gC = (T*)gcut; a.gu = (T*)gunit;
    int rc;
    {
      auto a1 = a;
      a1.nblk = 1;  // wave per node, all channel blocks inside the wave
      if (a.nblk == 1) rc = tn::launch<T>(tn::k_embed_bwd_dst<T, 1>, a1, st);
      else if (a.nblk == 2) rc = tn::launch<T>(tn::k_embed_bwd_dst<T, 2>, a1, st);
      else if (a.nblk <= 4) rc = tn::launch<T>(tn::k_embed_bwd_dst<T, 4>, a1, st);
      else return kUnsupported;
    }
    if (rc) return rc;
    return tn::launch<T>(tn::k_embed_bwd_src<T>, a, st);
  })
}

extern "C" int tmdnet_tn_message_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                     const int32_t* src, int max_pairs, double self0_mult,
                                   const int32_t* pad_pairs, int pad_capacity,
                                     const void* edge_attr, int ld_ea, const void* I, const void* A,
                                     const void* S, void* msg, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                                 pad_capacity);
    a.ea = (const T*)edge_attr; a.ldea = ld_ea;
    a.Ti = (const T*)I; a.Ta = (const T*)A; a.Ts = (const T*)S; a.msg = (T*)msg;
    return tn::launch<T>(tn::k_msg_fwd<T>, a, st);
  })
}

extern "C" int tmdnet_tn_message_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                     const int32_t* src, int max_pairs, double self0_mult,
                                   const int32_t* pad_pairs, int pad_capacity,
                                     const void* edge_attr, int ld_ea, const void* I, const void* A,
                                     const void* S, const void* grad_msg, void* g_edge_attr,
                                     void* gI, void* gA, void* gS, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TN_DISPATCH(dtype, {
    auto a = tn::base<T>(n_nodes, hidden, row_ptr, src, max_pairs, self0_mult, pad_pairs,
                                 pad_capacity);
    a.ea = (const T*)edge_attr; a.ldea = ld_ea;
    a.Ti = (const T*)I; a.Ta = (const T*)A; a.Ts = (const T*)S;
    a.gmsg = (const T*)grad_msg; a.gea = (T*)g_edge_attr;
    a.gTi = (T*)gI; a.gTa = (T*)gA; a.gTs = (T*)gS;
    int rc = tn::launch<T>(tn::k_msg_bwd_dst<T>, a, st);
    if (rc) return rc;
    return tn::launch<T>(tn::k_msg_bwd_src<T>, a, st);
  })
}
