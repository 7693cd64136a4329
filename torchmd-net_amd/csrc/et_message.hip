// Equivariant-Transformer edge message + aggregation, and the neighbour-embedding aggregation.
//
// Reference: EquivariantMultiHeadAttention.forward/message/aggregate (models/torchmd_et.py:272-347),
// NeighborEmbedding.forward/message (models/utils.py:73-108).  The reference gathers q_i, k_j, v_j,
// vec_j into E x (heads, d) and E x (3, heads, d) tensors, multiplies them elementwise and
// scatter-adds with atomics (torch_scatter).  Here:
//   * one wave64 owns one destination atom t; its q[t] (and, backward, dL/dx[t], dL/dvec[t]) sit in
//     registers; the wave streams t's CSR row of edges (pre-activation dk/dv rows are read
//     coalesced, 4*H values per edge) and gathers k/v/vec rows of the sources (L2 / Infinity-Cache
//     resident for spatially ordered atoms);
//   * heads are aligned lane groups: the q.k.dk dot product is a group_sum over d/VEC lanes;
//   * x (H) and vec (3H) accumulate in registers and are written ONCE: no atomics, deterministic;
//   * the backward is two such passes: a destination pass (gq, per-edge grads) and a source pass
//     that walks the same CSR rows as reversed edges (valid for the symmetric lists the model
//     builds: dk, dv, cutoff are functions of |r| only and unit vectors flip sign), giving
//     gk, gv, gvec without a transpose scatter or atomics.
#include <cstdlib>

#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace et {

template <typename T, int V> struct Vec;
template <> struct Vec<float, 1> { using t = float; };
template <> struct Vec<float, 2> { using t = float2; };
template <> struct Vec<float, 4> { using t = float4; };
template <> struct Vec<double, 1> { using t = double; };
template <> struct Vec<double, 2> { using t = double2; };
template <> struct Vec<double, 4> { using t = double4; };

template <typename T, int V> __device__ __forceinline__ void ldv(T (&o)[V], const T* p);
template <typename T, int V> __device__ __forceinline__ void ldv_(T (&o)[V], const T* p) {
  using VT = typename Vec<T, V>::t;
  const VT x = *reinterpret_cast<const VT*>(p);
  if constexpr (V == 1) { o[0] = x; }
  else if constexpr (V == 2) { o[0] = x.x; o[1] = x.y; }
  else { o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w; }
}
template <typename T, int V> __device__ __forceinline__ void ldv(T (&o)[V], const T* p) {
  if constexpr (V == 8) {
    T a[4], b[4];
    ldv_<T, 4>(a, p);
    ldv_<T, 4>(b, p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = a[i]; o[4 + i] = b[i]; }
  } else {
    ldv_<T, V>(o, p);
  }
}
template <typename T, int V> __device__ __forceinline__ void stv(T* p, const T (&o)[V]);
template <typename T, int V> __device__ __forceinline__ void stv_(T* p, const T (&o)[V]) {
  using VT = typename Vec<T, V>::t;
  VT x;
  if constexpr (V == 1) { x = o[0]; }
  else if constexpr (V == 2) { x.x = o[0]; x.y = o[1]; }
  else { x.x = o[0]; x.y = o[1]; x.z = o[2]; x.w = o[3]; }
  *reinterpret_cast<VT*>(p) = x;
}
template <typename T, int V> __device__ __forceinline__ void stv(T* p, const T (&o)[V]) {
  if constexpr (V == 8) {
    T a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = o[i]; b[i] = o[4 + i]; }
    stv_<T, 4>(p, a);
    stv_<T, 4>(p + 4, b);
  } else {
    stv_<T, V>(p, o);
  }
}
// store, or (acc: the buffer already holds cotangents injected by the second order) add to it
template <typename T, int V> __device__ __forceinline__ void stv_acc(T* p, const T (&o)[V], bool acc) {
  if (acc) {
    T q[V];
    ldv<T, V>(q, p);
#pragma unroll
    for (int i = 0; i < V; ++i) q[i] += o[i];
    stv<T, V>(p, q);
  } else {
    stv<T, V>(p, o);
  }
}
template <typename T, int V> __device__ __forceinline__ void zero(T (&o)[V]) {
#pragma unroll
  for (int i = 0; i < V; ++i) o[i] = T(0);
}

template <typename T> struct Args {
  int n, H, d, L, lph, cap;
  int xcd;      // XCD-contiguous block remap (on: +10-15 % on C5-scale graphs)
  int HC;       // channels per channel group (H / CS)
  const int32_t* row_ptr;
  const int32_t* src;
  const int32_t* order;
  const T* q; int ldq;
  const T* k; int ldk;
  const T* v; int ldv;
  const T* vec;
  const T* pk; int ldpk;
  const T* pv; int ldpv;
  const int32_t* prow;  // row of pk / pv holding edge e's projection (pair-shared rows); NULL: row e
  const T* dpk;         // "dr mode" (backward): d pk / d r, d pv / d r rows (layout of pk / pv); the
  const T* dpv;         // projection gradient is contracted with them into gr[e] instead of stored
  T* gr;                // [E] accumulated d/d r (dr mode)
  const T* C;
  const T* u;
  // forward outputs
  T* xo; T* veco;
  // backward inputs / outputs
  const T* gx; const T* gvec;
  T* gq; T* gk; T* gv; T* gveci; T* gpk; T* gpv; T* gC; T* gu;
  int acc;  // TMDNET_ACC_* flags of the backward
  int planar;  // TMDNET_ET_V_PLANAR: v / pv rows are [x | v1 | v2] H-blocks (else per-head [x|v1|v2] d-blocks)
  int vst;     // distance between the x, v1, v2 parts of a v / pv row: H (planar) or d
  int act_kv;  // ActCode of the dk / dv projections (reference `activation`) and of the attention
  int act_at;  // (`attn_activation`), torchmd_et.py:285-291, 316: TMDNET_ET_ACT bits of the flags
};

// SiLU of a pre-activation row segment already in registers (or 1 / 0 when the projection is
// absent).  Loads and activations are kept apart on purpose: every per-edge load of an edge is
// issued before the first activation, so an edge costs one memory round trip, not one per load.
// `code`: the ActCode (SiLU: one branch for the whole segment, the math unchanged).
template <typename T, int V>
__device__ __forceinline__ void act(const T (&x)[V], bool has, T (&s)[V], T (&ds)[V], int code) {
  if (code == kActSilu) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      if (has) {
        Silu<T> f(x[i]);
        s[i] = f.s;
        ds[i] = f.d(x[i]);
      } else {
        s[i] = T(1);
        ds[i] = T(0);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    if (has) {
      ActF<T> f(x[i], code);
      s[i] = f.s;
      ds[i] = f.d(x[i]);
    } else {
      s[i] = T(1);
      ds[i] = T(0);
    }
  }
}
// Branch-free optional load: an absent projection reads a valid dummy row (result ignored).
template <typename T> __device__ __forceinline__ const T* opt(const T* p, size_t off, const T* dummy) {
  return p ? p + off : dummy;
}

// Work decomposition shared by the three kernels.
//   * a 256-thread block = 4 waves; S waves cooperate on one node (S in {1, 2, 4}), so a block owns
//     4/S nodes; the S partial results are summed through LDS at the end;
//   * inside a wave, groups of L lanes ("edge slots") each stream their own edge: a lane owns V
//     contiguous channels (16-byte loads at H = 128, fp32), so one wave instruction covers 64/L
//     edges (2 with L = 32);
//   * CS channel groups: each wave covers H/CS channels of its node (heads are independent);
//   * row bounds and the node index are wave-uniform (readfirstlane): scalar loads.

// XCD-contiguous remap (common.h xcd_remap): the source rows a node range's waves gather
// (neighbours of nearby nodes) are shared in that XCD's L2.
__device__ __forceinline__ int xcd_block(int b, int nwg, int xcd) { return xcd ? xcd_remap(b, nwg) : b; }
struct Geo {
  int node;  // node owned by this wave (-1: idle wave of a partially filled block)
  int sub;   // wave index within the node's group [0, S)
  int es;    // edge slot of this lane (lanes [es*L, (es+1)*L) stream one edge)
  int el;    // lane within the edge slot
  int cg;    // channel group of this wave [0, CS)
};

// Logical block -> (channel group, node block).  With the XCD-contiguous remap the CS channel
// groups of one node range run on DIFFERENT XCDs, so each XCD's L2 holds only its channel slice of
// the gathered source rows (the per-XCD working set shrinks CS-fold).
template <int S, int CS, bool ORD, int WPB = 4>  // WPB: waves per block
__device__ __forceinline__ Geo geo(int n, int L, const int32_t* order, int xcd, int blk, int nwg) {
  Geo g;
  const int wid = threadIdx.x >> 6;
  const int npb = WPB / S;
  const int nbn = (n + npb - 1) / npb;
  const int lb = xcd_block(blk, nwg, xcd);
  g.cg = CS > 1 ? __builtin_amdgcn_readfirstlane(lb / nbn) : 0;
  const int w = __builtin_amdgcn_readfirstlane((CS > 1 ? lb % nbn : lb) * npb + wid / S);
  g.sub = __builtin_amdgcn_readfirstlane(wid % S);
  g.node = w < n ? (ORD ? __builtin_amdgcn_readfirstlane(order[w]) : w) : -1;
  const int lane = lane_id();
  g.es = lane / L;
  g.el = lane % L;
  return g;
}

template <typename T, int V> __device__ __forceinline__ void xor_slots(T (&a)[V], int L) {
  for (int o = L; o < TMD_WAVE; o <<= 1)
#pragma unroll
    for (int i = 0; i < V; ++i) a[i] += __shfl_xor(a[i], o);
}

// Sum NV per-lane values over the S waves of a node through LDS; the result lands in wave sub==0.
template <typename T, int S, int NV>
__device__ __forceinline__ void reduce_waves(T (&a)[NV], int sub, T* lds) {
  if constexpr (S > 1) {
    const int wid = threadIdx.x >> 6, lane = lane_id();
    const int base = (wid - sub) * 64 * NV;  // group's slab
    if (sub > 0) {
#pragma unroll
      for (int i = 0; i < NV; ++i) lds[base + (sub * NV + i) * 64 + lane] = a[i];
    }
    __syncthreads();
    if (sub == 0) {
#pragma unroll
      for (int s2 = 1; s2 < S; ++s2)
#pragma unroll
        for (int i = 0; i < NV; ++i) a[i] += lds[base + (s2 * NV + i) * 64 + lane];
    }
  }
}

// Row traversal.  The per-edge scalars (source index, cutoff, unit vector) are fetched once per chunk
// of 64 edges by one coalesced load per lane and handed to the edge slots by cross-lane permutes, so
// an edge's gathers depend on ONE memory round trip, not two.  The chunk and slot loops are
// wave-uniform (permutes need every lane active); a slot past the end of the row skips the body.
// The per-edge STREAM (dk/dv rows, read once) is software-pipelined PD edges ahead: `ld(k, st)` loads edge k's stream rows into registers; `body(k, s, C, u0, u1, u2, st, pre)`
// issues its source gathers, then calls `pre()` -- which issues the NEXT edge's stream loads -- and
// only then consumes data.  Loads retire in issue order, so waiting for this edge's gathers leaves
// the next edges' stream in flight (a counted vmcnt).  PD = 1 is used: C5 fwd 1.44 -> 1.35-1.41 ms;
// PD = 2 measured equal in interleaved runs (tools/kbench.py) at 18 more VGPRs.
// The prefetch is unconditional (clamped to the chunk's last edge) so the wait count is static.
template <typename T, int S, int PD, typename St, typename LD, typename F>
__device__ __forceinline__ void edge_chunks_pf(const Args<T>& A, int b, int e, int EPW, const Geo& G,
                                               LD&& ld, F&& body) {
  const int lane = lane_id();
  St cur, nxt, nx2;
  const int step = EPW * S;
  for (int c = b; c < e; c += TMD_WAVE) {
    const int n = min(TMD_WAVE, e - c);
    int s_r = 0, p_r = c + lane;
    T C_r = T(0), u0_r = T(0), u1_r = T(0), u2_r = T(0);
    if (lane < n) {
      const int k = c + lane;
      s_r = A.src[k];
      TMD_DCHECK(s_r >= 0 && s_r < A.n);
      if (A.prow) p_r = A.prow[k];
      C_r = A.C[k];
      u0_r = A.u[3 * k];
      u1_r = A.u[3 * k + 1];
      u2_r = A.u[3 * k + 2];
    }
    int j0 = EPW * G.sub;
    if (j0 < n) {  // PD edges of stream in flight ahead of the one being consumed (ld takes ROWS)
      ld(__shfl(p_r, min(j0 + G.es, n - 1)), cur);
      if constexpr (PD == 2) ld(__shfl(p_r, min(j0 + step + G.es, n - 1)), nxt);
    }
    for (; j0 < n; j0 += step) {
      const int j = j0 + G.es;
      const int jj = j < n ? j : n - 1;
      const int s = __shfl(s_r, jj);
      const T Ce = __shfl(C_r, jj), u0 = __shfl(u0_r, jj), u1 = __shfl(u1_r, jj), u2 = __shfl(u2_r, jj);
      const int kn = __shfl(p_r, min(j0 + PD * step + G.es, n - 1));  // next edge's stream row
      auto pre = [&]() { ld(kn, PD == 2 ? nx2 : nxt); };
      if (j < n) body(c + j, s, Ce, u0, u1, u2, cur, pre);
      else pre();
      cur = nxt;
      if constexpr (PD == 2) nxt = nx2;
    }
  }
}

// The same traversal without the stream prefetch: body(k, s, C, u0, u1, u2, row) issues every load of
// the edge itself (fewer live registers: the merged backward's occupancy is worth more than the
// pipelining).
template <typename T, int S, typename F>
__device__ __forceinline__ void edge_chunks(const Args<T>& A, int b, int e, int EPW, const Geo& G, F&& body) {
  const int lane = lane_id();
  const int step = EPW * S;
  for (int c = b; c < e; c += TMD_WAVE) {
    const int n = min(TMD_WAVE, e - c);
    int s_r = 0, p_r = c + lane;
    T C_r = T(0), u0_r = T(0), u1_r = T(0), u2_r = T(0);
    if (lane < n) {
      const int k = c + lane;
      s_r = A.src[k];
      TMD_DCHECK(s_r >= 0 && s_r < A.n);
      if (A.prow) p_r = A.prow[k];
      C_r = A.C[k];
      u0_r = A.u[3 * k];
      u1_r = A.u[3 * k + 1];
      u2_r = A.u[3 * k + 2];
    }
    for (int j0 = EPW * G.sub; j0 < n; j0 += step) {
      const int j = j0 + G.es;
      const int jj = j < n ? j : n - 1;
      const int s = __shfl(s_r, jj), row = __shfl(p_r, jj);
      const T Ce = __shfl(C_r, jj), u0 = __shfl(u0_r, jj), u1 = __shfl(u1_r, jj), u2 = __shfl(u2_r, jj);
      if (j < n) body(c + j, s, Ce, u0, u1, u2, row);
    }
  }
}

// ------------------------------------------------------------------ forward
// ORD: nodes visited in the caller's `order` (cell order for large periodic systems, so the waves in
// flight gather from a compact spatial window of source rows).
template <typename T, int V, int S, int CS, bool ORD, bool GA = true>
__global__ __launch_bounds__(256) void k_fwd(Args<T> A) {
  const int AKV = GA ? A.act_kv : kActSilu, AAT = GA ? A.act_at : kActSilu;  // GA: runtime codes
  __shared__ T lds[S > 1 ? 4 * 64 * 4 * V : 1];
  const Geo G = geo<S, CS, ORD>(A.n, A.L, A.order, A.xcd, blockIdx.x, gridDim.x);
  const int t = G.node;
  const bool on = true;
  const int EPW = TMD_WAVE / A.L;  // edges per wave instruction
  const int c0 = G.cg * A.HC + G.el * V;
  const int hh = c0 / A.d, cc = c0 % A.d;
  const int vo = A.planar ? c0 : hh * 3 * A.d + cc;
  const bool hk = A.pk != nullptr, hv = A.pv != nullptr, hw = A.vec != nullptr;
  const int pvd = hv ? A.vst : 0, vcd = hw ? A.H : 0;  // branch-free optional loads
  (void)vcd;
  T ax[V], a0[V], a1[V], a2[V];
  zero(ax); zero(a0); zero(a1); zero(a2);
  if (t >= 0) {
    T q[V];
    ldv<T, V>(q, A.q + (size_t)t * A.ldq + c0);
    const int b = min(A.row_ptr[t], A.cap), e = min(A.row_ptr[t + 1], A.cap);
    const T* dummy = A.q + (size_t)t * A.ldq;  // valid row for absent optional inputs
    struct St { T k[V], x[V], a[V], b[V]; };  // one edge's dk/dv stream (pre-activations)
    auto ld = [&](int k, St& st) {
      ldv<T, V>(st.k, opt(A.pk, (size_t)k * A.ldpk + c0, dummy + c0));
      const T* pvs = opt(A.pv, (size_t)k * A.ldpv + vo, dummy);
      ldv<T, V>(st.x, pvs);
      ldv<T, V>(st.a, pvs + pvd);
      ldv<T, V>(st.b, pvs + 2 * pvd);
    };
    auto body = [&](int k, int s, T Ce, T u0, T u1, T u2, const St& st, auto&& pre) {
      (void)k;
      // source gathers (k, v, vec) for this edge, then the next edge's stream, then the math
      T kk[V], vx[V], v1[V], v2[V], w0[V], w1[V], w2[V];
      ldv<T, V>(kk, A.k + (size_t)s * A.ldk + c0);
      const T* vs = A.v + (size_t)s * A.ldv + vo;
      ldv<T, V>(vx, vs);
      ldv<T, V>(v1, vs + A.vst);
      ldv<T, V>(v2, vs + 2 * A.vst);
      const T* vecs = hw ? A.vec + (size_t)s * 3 * A.H + c0 : dummy + c0;
      ldv<T, V>(w0, vecs);
      ldv<T, V>(w1, vecs + vcd);
      ldv<T, V>(w2, vecs + 2 * vcd);
      pre();
      if (!hw) { zero(w0); zero(w1); zero(w2); }
      T dk[V], dvx[V], dv1[V], dv2[V], dd[V];
      act<T, V>(st.k, hk, dk, dd, AKV);
      act<T, V>(st.x, hv, dvx, dd, AKV);
      act<T, V>(st.a, hv, dv1, dd, AKV);
      act<T, V>(st.b, hv, dv2, dd, AKV);
      T part = T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) part += q[i] * kk[i] * dk[i];
      part = group_sum(part, A.lph);
      const ActF<T> sa(part, AAT);
      const T a = sa.s * Ce;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        ax[i] += vx[i] * dvx[i] * a;
        const T v1e = v1[i] * dv1[i], v2e = v2[i] * dv2[i];
        a0[i] += w0[i] * v1e + v2e * u0;
        a1[i] += w1[i] * v1e + v2e * u1;
        a2[i] += w2[i] * v1e + v2e * u2;
      }
    };
    edge_chunks_pf<T, S, 1, St>(A, b, e, EPW, G, ld, body);
  }
  xor_slots(ax, A.L); xor_slots(a0, A.L); xor_slots(a1, A.L); xor_slots(a2, A.L);
  T all[4 * V];
#pragma unroll
  for (int i = 0; i < V; ++i) { all[i] = ax[i]; all[V + i] = a0[i]; all[2 * V + i] = a1[i]; all[3 * V + i] = a2[i]; }
  reduce_waves<T, S, 4 * V>(all, G.sub, lds);
  if (t >= 0 && G.sub == 0 && on && G.es == 0) {
#pragma unroll
    for (int i = 0; i < V; ++i) { ax[i] = all[i]; a0[i] = all[V + i]; a1[i] = all[2 * V + i]; a2[i] = all[3 * V + i]; }
    stv<T, V>(A.xo + (size_t)t * A.H + c0, ax);
    T* vo_ = A.veco + (size_t)t * 3 * A.H + c0;
    stv<T, V>(vo_, a0);
    stv<T, V>(vo_ + A.H, a1);
    stv<T, V>(vo_ + 2 * A.H, a2);
  }
}

// ------------------------------------------------------------------ backward, destination pass
// Static-capacity edge lists: rows [row_ptr[n], cap) of gpk / gpv belong to no CSR row.  They are
// zeroed here (spread over the grid) so the weight-gradient GEMMs over all `cap` rows see zeros
// without a memset of the whole buffer.
template <typename T>
__device__ __forceinline__ void zero_pad_rows(const Args<T>& A, int blk, int nwg) {
  const int e0 = min(A.row_ptr[A.n], A.cap);
  if (e0 >= A.cap) return;
  const long long rows = A.cap - e0;
  const long long tid = (long long)blk * blockDim.x + threadIdx.x, nth = (long long)nwg * blockDim.x;
  if (A.gpk) {
    for (long long i = tid; i < rows * A.H; i += nth)
      A.gpk[(size_t)(e0 + i / A.H) * A.ldpk + i % A.H] = T(0);
  }
  if (A.gpv) {
    const int w = 3 * A.H;
    for (long long i = tid; i < rows * w; i += nth)
      A.gpv[(size_t)(e0 + i / w) * A.ldpv + i % w] = T(0);
  }
  if (A.gC)
    for (long long i = tid; i < rows; i += nth) A.gC[e0 + i] = T(0);
  if (A.gu)
    for (long long i = tid; i < rows * 3; i += nth) A.gu[3 * (size_t)e0 + i] = T(0);
  if (A.gr)
    for (long long i = tid; i < rows; i += nth) A.gr[e0 + i] = T(0);
}

// AG: TMDNET_ACC_GRADS in the training form -- the injected per-edge projection cotangents are loaded
// with the edge's other loads (not read back after the math: one memory round trip per edge fewer)
template <typename T, int V, int S, int CS, bool DR, bool AG = false, bool GA = true>
__device__ __forceinline__ void bwd_dst_body(const Args<T>& A, int blk, int nwg) {
  const int AKV = GA ? A.act_kv : kActSilu, AAT = GA ? A.act_at : kActSilu;  // GA: runtime codes
  __shared__ T lds[S > 1 ? 4 * 64 * V : 1];
  const Geo G = geo<S, CS, false>(A.n, A.L, nullptr, A.xcd, blk, nwg);
  const int t = G.node;
  const bool on = true;
  const int EPW = TMD_WAVE / A.L;  // edges per wave instruction
  const int c0 = G.cg * A.HC + G.el * V;
  const int hh = c0 / A.d, cc = c0 % A.d;
  const int vo = A.planar ? c0 : hh * 3 * A.d + cc;
  const bool hk = A.pk != nullptr, hv = A.pv != nullptr, hw = A.vec != nullptr;
  const int pvd = hv ? A.vst : 0, vcd = hw ? A.H : 0;  // branch-free optional loads
  (void)vcd;
  const bool head_leader = on && (G.el % A.lph) == 0;
  T gq[V];
  zero(gq);
  if (t >= 0) {
    T q[V], gx[V], g0[V], g1[V], g2[V];
    ldv<T, V>(q, A.q + (size_t)t * A.ldq + c0);
    ldv<T, V>(gx, A.gx + (size_t)t * A.H + c0);
    const T* gvt = A.gvec + (size_t)t * 3 * A.H + c0;
    ldv<T, V>(g0, gvt);
    ldv<T, V>(g1, gvt + A.H);
    ldv<T, V>(g2, gvt + 2 * A.H);
    const int b = min(A.row_ptr[t], A.cap), e = min(A.row_ptr[t + 1], A.cap);
    const T* dummy = A.q + (size_t)t * A.ldq;
    const bool acc_edge = (A.acc & TMDNET_ACC_EDGE) && G.el == 0;
    // dr mode (DR): the edge's (pair) row index rides along; d pk / d r, d pv / d r are loaded in
    // the body with the source-row gathers (prefetching them too costs occupancy: 183 vs 157 VGPRs)
    struct St { T k[V], x[V], a[V], b[V]; int row; };
    auto ld = [&](int k, St& st) {
      ldv<T, V>(st.k, opt(A.pk, (size_t)k * A.ldpk + c0, dummy + c0));
      const T* pvs = opt(A.pv, (size_t)k * A.ldpv + vo, dummy);
      ldv<T, V>(st.x, pvs);
      ldv<T, V>(st.a, pvs + pvd);
      ldv<T, V>(st.b, pvs + 2 * pvd);
      st.row = k;
    };
    auto body = [&](int k, int s, T Ce, T u0, T u1, T u2, const St& st, auto&& pre) {
      T oc = T(0), ou0 = T(0), ou1 = T(0), ou2 = T(0), orr = T(0);  // accumulate mode: issued with the loads
      if (acc_edge) {
        oc = A.gC[k];
        ou0 = A.gu[3 * k];
        ou1 = A.gu[3 * k + 1];
        ou2 = A.gu[3 * k + 2];
        if constexpr (DR) orr = A.gr[k];
      }
      T kk[V], vx[V], v1[V], v2[V], w0[V], w1[V], w2[V];
      ldv<T, V>(kk, A.k + (size_t)s * A.ldk + c0);
      const T* vs = A.v + (size_t)s * A.ldv + vo;
      ldv<T, V>(vx, vs);
      ldv<T, V>(v1, vs + A.vst);
      ldv<T, V>(v2, vs + 2 * A.vst);
      const T* vecs = hw ? A.vec + (size_t)s * 3 * A.H + c0 : dummy + c0;
      ldv<T, V>(w0, vecs);
      ldv<T, V>(w1, vecs + vcd);
      ldv<T, V>(w2, vecs + 2 * vcd);
      T ik[AG ? V : 1], ix[AG ? V : 1], i1[AG ? V : 1], i2[AG ? V : 1];  // injected cotangents (AG)
      if constexpr (AG) {
        if (hk) ldv<T, V>(ik, A.gpk + (size_t)k * A.ldpk + c0); else zero(ik);
        if (hv) {
          const T* gp = A.gpv + (size_t)k * A.ldpv + vo;
          ldv<T, V>(ix, gp); ldv<T, V>(i1, gp + A.vst); ldv<T, V>(i2, gp + 2 * A.vst);
        } else {
          zero(ix); zero(i1); zero(i2);
        }
      }
      T dpk_[DR ? V : 1], dpx_[DR ? V : 1], dp1_[DR ? V : 1], dp2_[DR ? V : 1];
      if constexpr (DR) {
        ldv<T, V>(dpk_, opt(A.dpk, (size_t)st.row * A.ldpk + c0, dummy + c0));
        const T* dps = opt(A.dpv, (size_t)st.row * A.ldpv + vo, dummy);
        ldv<T, V>(dpx_, dps);
        ldv<T, V>(dp1_, dps + pvd);
        ldv<T, V>(dp2_, dps + 2 * pvd);
      }
      pre();
      if (!hw) { zero(w0); zero(w1); zero(w2); }
      const T (&pk)[V] = st.k;
      const T (&px)[V] = st.x;
      const T (&p1)[V] = st.a;
      const T (&p2)[V] = st.b;
      T dk[V], ddk[V], dvx[V], dv1[V], dv2[V], ddx[V], dd1[V], dd2[V];
      act<T, V>(pk, hk, dk, ddk, AKV);
      act<T, V>(px, hv, dvx, ddx, AKV);
      act<T, V>(p1, hv, dv1, dd1, AKV);
      act<T, V>(p2, hv, dv2, dd2, AKV);
      T part = T(0), ga = T(0), gu0 = T(0), gu1 = T(0), gu2 = T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        part += q[i] * kk[i] * dk[i];
        ga += gx[i] * vx[i] * dvx[i];
        const T v2e = v2[i] * dv2[i];
        gu0 += g0[i] * v2e;
        gu1 += g1[i] * v2e;
        gu2 += g2[i] * v2e;
      }
      part = group_sum(part, A.lph);
      ga = group_sum(ga, A.lph);
      const ActF<T> sa(part, AAT);
      const T a = sa.s * Ce;
      const T gs = ga * Ce * sa.d(part);
      T gpk[V], gpx[V], gp1[V], gp2[V];
#pragma unroll
      for (int i = 0; i < V; ++i) {
        gq[i] += gs * kk[i] * dk[i];
        gpk[i] = gs * q[i] * kk[i] * ddk[i];
        gpx[i] = gx[i] * a * vx[i] * ddx[i];
        const T gv1e = g0[i] * w0[i] + g1[i] * w1[i] + g2[i] * w2[i];
        gp1[i] = gv1e * v1[i] * dd1[i];
        const T gv2e = g0[i] * u0 + g1[i] * u1 + g2[i] * u2;
        gp2[i] = gv2e * v2[i] * dd2[i];
      }
      const T gc = group_sum(head_leader ? ga * sa.s : T(0), A.L);
      gu0 = group_sum(gu0, A.L);
      gu1 = group_sum(gu1, A.L);
      gu2 = group_sum(gu2, A.L);
      T grr = T(0);
      if constexpr (DR) {  // d/dr through the projections: <g_pk, d pk/dr> + <g_pv, d pv/dr>
#pragma unroll
        for (int i = 0; i < V; ++i)
          grr += (hk ? gpk[i] * dpk_[i] : T(0)) +
                 (hv ? gpx[i] * dpx_[i] + gp1[i] * dp1_[i] + gp2[i] * dp2_[i] : T(0));
        grr = group_sum(grr, A.L);
        if (on && (A.gpk || A.gpv)) {  // the recorded force pass also keeps the projection gradient
          if (hk && A.gpk) stv<T, V>(A.gpk + (size_t)k * A.ldpk + c0, gpk);
          if (hv && A.gpv) {
            T* gp = A.gpv + (size_t)k * A.ldpv + vo;
            stv<T, V>(gp, gpx);
            stv<T, V>(gp + A.vst, gp1);
            stv<T, V>(gp + 2 * A.vst, gp2);
          }
        }
      } else {
        if (on) {
          if constexpr (AG) {
#pragma unroll
            for (int i = 0; i < V; ++i) { gpk[i] += ik[i]; gpx[i] += ix[i]; gp1[i] += i1[i]; gp2[i] += i2[i]; }
          }
          const bool ag = !AG && (A.acc & TMDNET_ACC_GRADS);
          if (hk) stv_acc<T, V>(A.gpk + (size_t)k * A.ldpk + c0, gpk, ag);
          if (hv) {
            T* gp = A.gpv + (size_t)k * A.ldpv + vo;
            stv_acc<T, V>(gp, gpx, ag);
            stv_acc<T, V>(gp + A.vst, gp1, ag);
            stv_acc<T, V>(gp + 2 * A.vst, gp2, ag);
          }
        }
      }
      if (G.el == 0) {
        A.gC[k] = oc + gc;
        A.gu[3 * k] = ou0 + gu0;
        A.gu[3 * k + 1] = ou1 + gu1;
        A.gu[3 * k + 2] = ou2 + gu2;
        if constexpr (DR) A.gr[k] = orr + grr;
      }
    };
    edge_chunks_pf<T, S, 1, St>(A, b, e, EPW, G, ld, body);
  }
  xor_slots(gq, A.L);
  reduce_waves<T, S, V>(gq, G.sub, lds);
  if (t >= 0 && G.sub == 0 && on && G.es == 0)
    stv_acc<T, V>(A.gq + (size_t)t * A.ldq + c0, gq, A.acc & TMDNET_ACC_GRADS);
  zero_pad_rows(A, blk, nwg);
}

// ------------------------------------------------------------------ backward, source pass
// A wave group owns node j as SOURCE.  Row j lists edges m->j; each is read as its reverse j->m
// (same dk/dv/cutoff, unit vector negated), m being the destination whose q/gx/gvec are gathered.
template <typename T, int V, int S, int CS, bool GA = true>
__device__ __forceinline__ void bwd_src_body(const Args<T>& A, int blk, int nwg) {
  const int AKV = GA ? A.act_kv : kActSilu, AAT = GA ? A.act_at : kActSilu;  // GA: runtime codes
  __shared__ T lds[S > 1 ? 4 * 64 * 7 * V : 1];
  const Geo G = geo<S, CS, false>(A.n, A.L, nullptr, A.xcd, blk, nwg);
  const int j = G.node;
  const bool on = true;
  const int EPW = TMD_WAVE / A.L;  // edges per wave instruction
  const int c0 = G.cg * A.HC + G.el * V;
  const int hh = c0 / A.d, cc = c0 % A.d;
  const int vo = A.planar ? c0 : hh * 3 * A.d + cc;
  const bool hk = A.pk != nullptr, hv = A.pv != nullptr, hw = A.vec != nullptr;
  const int pvd = hv ? A.vst : 0, vcd = hw ? A.H : 0;  // branch-free optional loads
  (void)vcd;
  T gk[V], gvx[V], gv1[V], gv2[V], gw0[V], gw1[V], gw2[V];
  zero(gk); zero(gvx); zero(gv1); zero(gv2); zero(gw0); zero(gw1); zero(gw2);
  if (j >= 0) {
    T kk[V], vx[V], v1[V], v2[V], w0[V], w1[V], w2[V];
    ldv<T, V>(kk, A.k + (size_t)j * A.ldk + c0);
    const T* vj = A.v + (size_t)j * A.ldv + vo;
    ldv<T, V>(vx, vj);
    ldv<T, V>(v1, vj + A.vst);
    ldv<T, V>(v2, vj + 2 * A.vst);
    if (hw) {
      const T* vecj = A.vec + (size_t)j * 3 * A.H + c0;
      ldv<T, V>(w0, vecj);
      ldv<T, V>(w1, vecj + A.H);
      ldv<T, V>(w2, vecj + 2 * A.H);
    } else {
      zero(w0); zero(w1); zero(w2);
    }
    const int b = min(A.row_ptr[j], A.cap), e = min(A.row_ptr[j + 1], A.cap);
    const T* dummy = A.k + (size_t)j * A.ldk;
    struct St { T k[V], x[V], a[V], b[V]; };
    auto ld = [&](int k, St& st) {
      ldv<T, V>(st.k, opt(A.pk, (size_t)k * A.ldpk + c0, dummy + c0));
      const T* pvs = opt(A.pv, (size_t)k * A.ldpv + vo, dummy);
      ldv<T, V>(st.x, pvs);
      ldv<T, V>(st.a, pvs + pvd);
      ldv<T, V>(st.b, pvs + 2 * pvd);
    };
    auto body = [&](int k, int m, T Ce, T u0, T u1, T u2, const St& st, auto&& pre) {
      u0 = -u0; u1 = -u1; u2 = -u2;  // the reversed edge j->m
      (void)k;
      T qm[V], gxm[V], g0[V], g1[V], g2[V];
      ldv<T, V>(qm, A.q + (size_t)m * A.ldq + c0);
      ldv<T, V>(gxm, A.gx + (size_t)m * A.H + c0);
      const T* gvm = A.gvec + (size_t)m * 3 * A.H + c0;
      ldv<T, V>(g0, gvm);
      ldv<T, V>(g1, gvm + A.H);
      ldv<T, V>(g2, gvm + 2 * A.H);
      pre();
      const T (&pk)[V] = st.k;
      const T (&px)[V] = st.x;
      const T (&p1)[V] = st.a;
      const T (&p2)[V] = st.b;
      T dk[V], ddk[V], dvx[V], dv1[V], dv2[V], dd[V];
      act<T, V>(pk, hk, dk, ddk, AKV);
      act<T, V>(px, hv, dvx, dd, AKV);
      act<T, V>(p1, hv, dv1, dd, AKV);
      act<T, V>(p2, hv, dv2, dd, AKV);
      T part = T(0), ga = T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        part += qm[i] * kk[i] * dk[i];
        ga += gxm[i] * vx[i] * dvx[i];
      }
      part = group_sum(part, A.lph);
      ga = group_sum(ga, A.lph);
      const ActF<T> sa(part, AAT);
      const T a = sa.s * Ce;
      const T gs = ga * Ce * sa.d(part);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        gk[i] += gs * qm[i] * dk[i];
        gvx[i] += gxm[i] * a * dvx[i];
        const T gv1e = g0[i] * w0[i] + g1[i] * w1[i] + g2[i] * w2[i];
        gv1[i] += gv1e * dv1[i];
        const T gv2e = g0[i] * u0 + g1[i] * u1 + g2[i] * u2;
        gv2[i] += gv2e * dv2[i];
        const T v1e = v1[i] * dv1[i];
        gw0[i] += g0[i] * v1e;
        gw1[i] += g1[i] * v1e;
        gw2[i] += g2[i] * v1e;
      }
    };
    edge_chunks_pf<T, S, 1, St>(A, b, e, EPW, G, ld, body);
  }
  xor_slots(gk, A.L); xor_slots(gvx, A.L); xor_slots(gv1, A.L); xor_slots(gv2, A.L); xor_slots(gw0, A.L); xor_slots(gw1, A.L); xor_slots(gw2, A.L);
  T all[7 * V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    all[i] = gk[i]; all[V + i] = gvx[i]; all[2 * V + i] = gv1[i]; all[3 * V + i] = gv2[i];
    all[4 * V + i] = gw0[i]; all[5 * V + i] = gw1[i]; all[6 * V + i] = gw2[i];
  }
  reduce_waves<T, S, 7 * V>(all, G.sub, lds);
  if (j >= 0 && G.sub == 0 && on && G.es == 0) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      gk[i] = all[i]; gvx[i] = all[V + i]; gv1[i] = all[2 * V + i]; gv2[i] = all[3 * V + i];
      gw0[i] = all[4 * V + i]; gw1[i] = all[5 * V + i]; gw2[i] = all[6 * V + i];
    }
    const bool ag = A.acc & TMDNET_ACC_GRADS;
    stv_acc<T, V>(A.gk + (size_t)j * A.ldk + c0, gk, ag);
    T* gvj = A.gv + (size_t)j * A.ldv + vo;
    stv_acc<T, V>(gvj, gvx, ag);
    stv_acc<T, V>(gvj + A.vst, gv1, ag);
    stv_acc<T, V>(gvj + 2 * A.vst, gv2, ag);
    if (A.gveci != nullptr) {
      if (A.acc & TMDNET_ACC_VEC_RESIDUAL) {  // gvec_in = grad_vec (residual path) + message part
        const T* gr = A.gvec + (size_t)j * 3 * A.H + c0;
        T r0[V], r1[V], r2[V];
        ldv<T, V>(r0, gr);
        ldv<T, V>(r1, gr + A.H);
        ldv<T, V>(r2, gr + 2 * A.H);
#pragma unroll
        for (int i = 0; i < V; ++i) { gw0[i] += r0[i]; gw1[i] += r1[i]; gw2[i] += r2[i]; }
      }
      T* gwj = A.gveci + (size_t)j * 3 * A.H + c0;
      stv_acc<T, V>(gwj, gw0, ag);
      stv_acc<T, V>(gwj + A.H, gw1, ag);
      stv_acc<T, V>(gwj + 2 * A.H, gw2, ag);
    }
  }
}

// (fp32 dr variants: 3 waves / SIMD asked for -- they sit a few VGPRs above the 168 that allow it;
// 12 B/lane spill, measured faster than 2 waves)
template <typename T, int V, bool DR>
constexpr int bwd_min_waves() { return (DR && sizeof(T) == 4 && V <= 4) ? 3 : 1; }

template <typename T, int V, int S, int CS, bool DR, bool AG = false, bool GA = true>
__global__ __launch_bounds__(256, (bwd_min_waves<T, V, DR>())) void k_bwd_dst(Args<T> A) {
  bwd_dst_body<T, V, S, CS, DR, AG, GA>(A, blockIdx.x, gridDim.x);
}
template <typename T, int V, int S, int CS, bool GA = true>
__global__ __launch_bounds__(256) void k_bwd_src(Args<T> A) {
  bwd_src_body<T, V, S, CS, GA>(A, blockIdx.x, gridDim.x);
}
// Both passes in ONE grid (they only read the same inputs): blocks [0, split) run the destination
// pass, [split, 2 split) the source pass.  Used for small systems, where one pass alone leaves most
// of the chip idle and the launch gap between the two passes is a visible share of the layer.
template <typename T, int V, int S, int CS, bool DR, bool AG = false, bool GA = true>
__global__ __launch_bounds__(256, (bwd_min_waves<T, V, DR>())) void k_bwd_both(Args<T> A) {
  const int split = (int)gridDim.x / 2;
  if ((int)blockIdx.x < split) bwd_dst_body<T, V, S, CS, DR, AG, GA>(A, blockIdx.x, split);
  else bwd_src_body<T, V, S, CS, GA>(A, blockIdx.x - split, split);
}

// ------------------------------------------------------------------ backward, merged pass (dr mode)
// Both roles of a node in ONE pass over its CSR row: for the edge e = (t <- s) the destination role
// (gq[t], and e's g_cut / g_unit / g_r) and, from the same pair row, the source role of its reverse
// s <- t (gk[t], gv[t], gvec_in[t]) -- the pair row (dk / dv pre-activations) is fetched once per
// edge instead of once per pass (the two-pass backward reads it twice per direction, four times per
// pair: 3.4x its distinct bytes at C5), and the per-edge activations are formed once.  Each edge
// gathers both of its source's row sets (k, v, vec for the destination role; q, gx, gvec for the
// source role).  The node's own vectors (q, gx, gvec | k, v, vec) are staged in LDS once per node
// and re-read per edge (48 fewer VGPRs than holding them in registers).
template <typename T, int V, int S, int PD, bool GA = true>
__device__ __forceinline__ void bwd_merged_body(const Args<T>& A, int blk, int nwg) {
  const int AKV = GA ? A.act_kv : kActSilu, AAT = GA ? A.act_at : kActSilu;  // GA: runtime codes
  constexpr int NA = 8 * V;            // accumulators summed over a node's S waves
  extern __shared__ __attribute__((aligned(16))) char dyn_lds[];  // max(4/S nodes x 12 H, reduction)
  T* lds = reinterpret_cast<T*>(dyn_lds);
  const int HM = A.H;
  const Geo G = geo<S, 1, false>(A.n, A.L, nullptr, A.xcd, blk, nwg);
  const int t = G.node;
  const int EPW = TMD_WAVE / A.L;
  const int c0 = G.el * V;
  const int hh = c0 / A.d, cc = c0 % A.d;
  const int vo = A.planar ? c0 : hh * 3 * A.d + cc;
  const bool hk = A.pk != nullptr, hv = A.pv != nullptr, hw = A.vec != nullptr;
  const int pvd = hv ? A.vst : 0, vcd = hw ? A.H : 0;
  const bool head_leader = (G.el % A.lph) == 0;
  // node vectors: [q | gx | g0 | g1 | g2 | k | vx | v1 | v2 | w0 | w1 | w2] x H of this wave's node
  T* nv = lds + ((threadIdx.x >> 6) / S) * 12 * HM;
  if (t >= 0 && G.sub == 0 && G.es == 0) {
    T a[V];
    const T* src[12];
    const T* gvt = A.gvec + (size_t)t * 3 * A.H;
    const T* vt = A.v + (size_t)t * A.ldv;
    const T* wt = A.vec + (size_t)t * 3 * A.H;
    src[0] = A.q + (size_t)t * A.ldq + c0; src[1] = A.gx + (size_t)t * A.H + c0;
    src[2] = gvt + c0; src[3] = gvt + A.H + c0; src[4] = gvt + 2 * A.H + c0;
    src[5] = A.k + (size_t)t * A.ldk + c0;
    src[6] = vt + vo; src[7] = vt + vo + A.vst; src[8] = vt + vo + 2 * A.vst;
    src[9] = hw ? wt + c0 : src[0]; src[10] = hw ? wt + A.H + c0 : src[0]; src[11] = hw ? wt + 2 * A.H + c0 : src[0];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
      ldv<T, V>(a, src[r]);
      if (r >= 9 && !hw) zero(a);
      stv<T, V>(nv + r * HM + c0, a);
    }
  }
  __syncthreads();
  T gq[V], gk[V], gvx[V], gv1[V], gv2[V], gw0[V], gw1[V], gw2[V];
  zero(gq); zero(gk); zero(gvx); zero(gv1); zero(gv2); zero(gw0); zero(gw1); zero(gw2);
  if (t >= 0) {
    const int b = min(A.row_ptr[t], A.cap), e = min(A.row_ptr[t + 1], A.cap);
    const T* dummy = A.q + (size_t)t * A.ldq;
    const bool acc_edge = (A.acc & TMDNET_ACC_EDGE) && G.el == 0;
    struct St { T k[V], x[V], a[V], b[V]; int row; };
    auto ld = [&](int k, St& st) {
      ldv<T, V>(st.k, opt(A.pk, (size_t)k * A.ldpk + c0, dummy + c0));
      const T* pvs = opt(A.pv, (size_t)k * A.ldpv + vo, dummy);
      ldv<T, V>(st.x, pvs);
      ldv<T, V>(st.a, pvs + pvd);
      ldv<T, V>(st.b, pvs + 2 * pvd);
      st.row = k;
    };
    auto body = [&](int k, int s, T Ce, T u0, T u1, T u2, const St& st, auto&& pre) {
      T oc = T(0), ou0 = T(0), ou1 = T(0), ou2 = T(0), orr = T(0);
      if (acc_edge) {
        oc = A.gC[k]; ou0 = A.gu[3 * k]; ou1 = A.gu[3 * k + 1]; ou2 = A.gu[3 * k + 2]; orr = A.gr[k];
      }
      // the source's rows: k, v, vec (destination role) and q, gx, gvec (source role of the reverse)
      T kk[V], vx[V], v1[V], v2[V], w0[V], w1[V], w2[V], qs[V], gxs[V], h0[V], h1[V], h2[V];
      ldv<T, V>(kk, A.k + (size_t)s * A.ldk + c0);
      const T* vs = A.v + (size_t)s * A.ldv + vo;
      ldv<T, V>(vx, vs);
      ldv<T, V>(v1, vs + A.vst);
      ldv<T, V>(v2, vs + 2 * A.vst);
      const T* vecs = hw ? A.vec + (size_t)s * 3 * A.H + c0 : dummy + c0;
      ldv<T, V>(w0, vecs);
      ldv<T, V>(w1, vecs + vcd);
      ldv<T, V>(w2, vecs + 2 * vcd);
      ldv<T, V>(qs, A.q + (size_t)s * A.ldq + c0);
      ldv<T, V>(gxs, A.gx + (size_t)s * A.H + c0);
      const T* gvs = A.gvec + (size_t)s * 3 * A.H + c0;
      ldv<T, V>(h0, gvs);
      ldv<T, V>(h1, gvs + A.H);
      ldv<T, V>(h2, gvs + 2 * A.H);
      T dpk_[V], dpx_[V], dp1_[V], dp2_[V];
      ldv<T, V>(dpk_, opt(A.dpk, (size_t)st.row * A.ldpk + c0, dummy + c0));
      const T* dps = opt(A.dpv, (size_t)st.row * A.ldpv + vo, dummy);
      ldv<T, V>(dpx_, dps);
      ldv<T, V>(dp1_, dps + pvd);
      ldv<T, V>(dp2_, dps + 2 * pvd);
      pre();
      if (!hw) { zero(w0); zero(w1); zero(w2); }
      T dk[V], ddk[V], dvx[V], dv1[V], dv2[V], ddx[V], dd1[V], dd2[V];
      act<T, V>(st.k, hk, dk, ddk, AKV);
      act<T, V>(st.x, hv, dvx, ddx, AKV);
      act<T, V>(st.a, hv, dv1, dd1, AKV);
      act<T, V>(st.b, hv, dv2, dd2, AKV);
      // ---- destination role: e = (t <- s), the node's q / gx / gvec from LDS
      {
        T q[V], gx[V], g0[V], g1[V], g2[V];
        ldv<T, V>(q, nv + 0 * HM + c0);
        ldv<T, V>(gx, nv + 1 * HM + c0);
        ldv<T, V>(g0, nv + 2 * HM + c0);
        ldv<T, V>(g1, nv + 3 * HM + c0);
        ldv<T, V>(g2, nv + 4 * HM + c0);
        T part = T(0), ga = T(0), gu0 = T(0), gu1 = T(0), gu2 = T(0);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          part += q[i] * kk[i] * dk[i];
          ga += gx[i] * vx[i] * dvx[i];
          const T v2e = v2[i] * dv2[i];
          gu0 += g0[i] * v2e;
          gu1 += g1[i] * v2e;
          gu2 += g2[i] * v2e;
        }
        part = group_sum(part, A.lph);
        ga = group_sum(ga, A.lph);
        const ActF<T> sa(part, AAT);
        const T a = sa.s * Ce;
        const T gs = ga * Ce * sa.d(part);
        T grr = T(0);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          gq[i] += gs * kk[i] * dk[i];
          const T gpk = gs * q[i] * kk[i] * ddk[i];
          const T gpx = gx[i] * a * vx[i] * ddx[i];
          const T gp1 = (g0[i] * w0[i] + g1[i] * w1[i] + g2[i] * w2[i]) * v1[i] * dd1[i];
          const T gp2 = (g0[i] * u0 + g1[i] * u1 + g2[i] * u2) * v2[i] * dd2[i];
          grr += (hk ? gpk * dpk_[i] : T(0)) + (hv ? gpx * dpx_[i] + gp1 * dp1_[i] + gp2 * dp2_[i] : T(0));
        }
        const T gc = group_sum(head_leader ? ga * sa.s : T(0), A.L);
        gu0 = group_sum(gu0, A.L);
        gu1 = group_sum(gu1, A.L);
        gu2 = group_sum(gu2, A.L);
        grr = group_sum(grr, A.L);
        if (G.el == 0) {
          A.gC[k] = oc + gc;
          A.gu[3 * k] = ou0 + gu0;
          A.gu[3 * k + 1] = ou1 + gu1;
          A.gu[3 * k + 2] = ou2 + gu2;
          A.gr[k] = orr + grr;
        }
      }
      // ---- source role: the reverse edge s <- t (unit vector negated), the node's k / v / vec from LDS
      {
        T kt[V], vxt[V], v1t[V], w0t[V], w1t[V], w2t[V];
        ldv<T, V>(kt, nv + 5 * HM + c0);
        ldv<T, V>(vxt, nv + 6 * HM + c0);
        ldv<T, V>(v1t, nv + 7 * HM + c0);
        ldv<T, V>(w0t, nv + 9 * HM + c0);
        ldv<T, V>(w1t, nv + 10 * HM + c0);
        ldv<T, V>(w2t, nv + 11 * HM + c0);
        T part = T(0), ga = T(0);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          part += qs[i] * kt[i] * dk[i];
          ga += gxs[i] * vxt[i] * dvx[i];
        }
        part = group_sum(part, A.lph);
        ga = group_sum(ga, A.lph);
        const ActF<T> sa(part, AAT);
        const T a = sa.s * Ce;
        const T gs = ga * Ce * sa.d(part);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          gk[i] += gs * qs[i] * dk[i];
          gvx[i] += gxs[i] * a * dvx[i];
          gv1[i] += (h0[i] * w0t[i] + h1[i] * w1t[i] + h2[i] * w2t[i]) * dv1[i];
          gv2[i] -= (h0[i] * u0 + h1[i] * u1 + h2[i] * u2) * dv2[i];
          const T v1e = v1t[i] * dv1[i];
          gw0[i] += h0[i] * v1e;
          gw1[i] += h1[i] * v1e;
          gw2[i] += h2[i] * v1e;
        }
      }
    };
    if constexpr (PD == 1) {
      edge_chunks_pf<T, S, 1, St>(A, b, e, EPW, G, ld, body);
    } else {
      edge_chunks<T, S>(A, b, e, EPW, G, [&](int k, int s, T Ce, T u0, T u1, T u2, int row) {
        St st;
        ld(row, st);
        body(k, s, Ce, u0, u1, u2, st, [] {});
      });
    }
  }
  xor_slots(gq, A.L); xor_slots(gk, A.L); xor_slots(gvx, A.L); xor_slots(gv1, A.L);
  xor_slots(gv2, A.L); xor_slots(gw0, A.L); xor_slots(gw1, A.L); xor_slots(gw2, A.L);
  T all[NA];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    all[i] = gq[i]; all[V + i] = gk[i]; all[2 * V + i] = gvx[i]; all[3 * V + i] = gv1[i];
    all[4 * V + i] = gv2[i]; all[5 * V + i] = gw0[i]; all[6 * V + i] = gw1[i]; all[7 * V + i] = gw2[i];
  }
  __syncthreads();  // the node vectors are dead: their LDS is the reduction's
  reduce_waves<T, S, NA>(all, G.sub, lds);
  if (t >= 0 && G.sub == 0 && G.es == 0) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      gq[i] = all[i]; gk[i] = all[V + i]; gvx[i] = all[2 * V + i]; gv1[i] = all[3 * V + i];
      gv2[i] = all[4 * V + i]; gw0[i] = all[5 * V + i]; gw1[i] = all[6 * V + i]; gw2[i] = all[7 * V + i];
    }
    const bool ag = A.acc & TMDNET_ACC_GRADS;
    stv_acc<T, V>(A.gq + (size_t)t * A.ldq + c0, gq, ag);
    stv_acc<T, V>(A.gk + (size_t)t * A.ldk + c0, gk, ag);
    T* gvj = A.gv + (size_t)t * A.ldv + vo;
    stv_acc<T, V>(gvj, gvx, ag);
    stv_acc<T, V>(gvj + A.vst, gv1, ag);
    stv_acc<T, V>(gvj + 2 * A.vst, gv2, ag);
    if (A.gveci != nullptr) {
      if (A.acc & TMDNET_ACC_VEC_RESIDUAL) {
        T r0[V], r1[V], r2[V];  // (the node's gvec: its LDS copy was overwritten by the reduction)
        const T* gr = A.gvec + (size_t)t * 3 * A.H + c0;
        ldv<T, V>(r0, gr);
        ldv<T, V>(r1, gr + A.H);
        ldv<T, V>(r2, gr + 2 * A.H);
#pragma unroll
        for (int i = 0; i < V; ++i) { gw0[i] += r0[i]; gw1[i] += r1[i]; gw2[i] += r2[i]; }
      }
      T* gwj = A.gveci + (size_t)t * 3 * A.H + c0;
      stv_acc<T, V>(gwj, gw0, ag);
      stv_acc<T, V>(gwj + A.H, gw1, ag);
      stv_acc<T, V>(gwj + 2 * A.H, gw2, ag);
    }
  }
  zero_pad_rows(A, blk, nwg);
}

template <typename T, int V, int S, int PD, bool GA = true>
__global__ __launch_bounds__(256, 2) void k_bwd_merged(Args<T> A) {
  bwd_merged_body<T, V, S, PD, GA>(A, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------ second-order backward
// VJP of tmdnet_et_message_bwd (needed when forces are differentiated again: force-matching
// training, reference model.py:286-298 with create_graph=True).  With gg* the cotangents of the
// first backward's outputs (gq, gk, gv, gvec_in, gpk, gpv, gcut, gunit), per edge e = (t <- s) and
// head h (part = q.k.dk, ga = gx.vx.dvx, sil/sd/sdd = silu and its derivatives of part):
//   S = sum_c ggq k dk + ggk q dk + ggpk q k dk'        X = sum_c ggvx gx dvx + ggpvx gx vx dvx'
//   P = C ga sdd S + C sd X + ggC ga sd                   G = C sd S + ggC sil
//   d/dq   += P k dk + gs (ggk dk + ggpk k dk')           (gs = ga C sd, a = sil C)
//   d/dk_s += P q dk + gs (ggq dk + ggpk q dk')
//   d/dpk   = P q k dk' + gs ((ggq k + ggk q) dk' + ggpk q k dk'')
//   d/dgx  += G vx dvx + a (ggvx dvx + ggpvx vx dvx')
//   d/dvx_s+= G gx dvx + a ggpvx gx dvx'
//   d/dpvx  = G gx vx dvx' + a (ggvx gx dvx' + ggpvx gx vx dvx'')
//   d/dC    = sum_h ga sd S + sil X
// and for the vector channels (G1 = sum_a gvec_a w_a, G2 = sum_a gvec_a u_a, U = sum_a ggu_a gvec_a,
// B1 = ggv1 dv1 + ggpv1 v1 dv1', B2 = ggv2 dv2 + ggpv2 v2 dv2'):
//   d/dgvec_a += w_a B1 + u_a B2 + ggw_a v1 dv1 + ggu_a v2 dv2       d/dw_a,s += gvec_a B1
//   d/dv1_s   += G1 ggpv1 dv1' + sum_a ggw_a gvec_a dv1              d/du_a    = sum_c gvec_a B2
//   d/dpv1     = G1 (ggv1 dv1' + ggpv1 v1 dv1'') + sum_a ggw_a gvec_a v1 dv1'
//   d/dv2_s   += G2 ggpv2 dv2' + U dv2
//   d/dpv2     = G2 (ggv2 dv2' + ggpv2 v2 dv2'') + U v2 dv2'
// One destination-row pass: destination-node terms accumulate in registers, per-edge terms are
// stored.  The source-node terms (k, v, vec) of edge e are either stored as a row of the per-edge
// scratch src[e] = [k (H) | v (3H, the v row layout) | vec (3H)] and summed per source node by
// k_bwd2_src over the reversed edges (deterministic, no atomics, no zero fills), or -- without a
// transpose map / scratch -- added with atomics into zero-initialised buffers.
template <typename T> struct Args2 {
  Args<T> a;                                       // primal inputs (q, k, v, vec, pk, pv, C, u) + gx, gvec
  const T* ggq; const T* ggk; const T* ggv; const T* ggw;   // node cotangents ([N][H], [N][H], [N][3H], [N][3][H])
  int ldggq, ldggk, ldggv;                                  // (row strides)
  const T* ggpk; int ldggpk; const T* ggpv; int ldggpv;     // edge cotangents
  const T* ggsc;  // non-NULL: the edge cotangents are the PAIR rows ggpk / ggpv[pk_rows[e]] scaled by ggsc[e]
                  // (force-matching: the cotangent of g_r times the pair rows' d(dk,dv)/dr)
  const T* ggC; const T* ggu;
  T* o_gx; T* o_gvec; T* o_q; T* o_k; T* o_v; T* o_vec;       // node outputs
  int ldoq, ldok, ldov;
  T* o_pk; T* o_pv; T* o_C; T* o_u;                          // edge outputs ([E][H], [E][3H], [E], [E][3])
  int ldopk, ldopv;
  T* o_src;               // per-edge source terms [E][7H] (NULL: atomics)
  const int32_t* tr;      // transpose map (k_bwd2_src)
  int acc_edge, acc_gvec; // accumulate o_C / o_u (and o_gvec) into the caller's buffers
};

// (S = 8: one node per 512-thread block -- the kernel's ~190 VGPRs allow two waves per SIMD, so a
// block of 8 waves fills a CU and a node's edges spread over 8 waves instead of 4)
template <typename T, int V, int S>
// (capping the registers for more waves per SIMD spills: 4 waves/SIMD 63 -> 142 us, 3 -> 84 us per
// layer at ET-QM9; measured and not kept)
__global__ __launch_bounds__(S > 4 ? 64 * S : 256) void k_bwd2(Args2<T> B) {
  constexpr int WPB = S > 4 ? S : 4;
  __shared__ T lds[S > 1 ? WPB * 64 * 5 * V : 1];
  const Args<T>& A = B.a;
  const Geo G = geo<S, 1, false, WPB>(A.n, A.L, nullptr, A.xcd, blockIdx.x, gridDim.x);
  const int t = G.node;
  {  // static-capacity padding rows [row_ptr[n], cap) of the per-edge outputs: zero (no memset)
    const int e0 = min(A.row_ptr[A.n], A.cap);
    const long long rows = A.cap - e0;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
    if (rows > 0) {
      if (B.o_pk)
        for (long long i = tid; i < rows * A.H; i += nth)
          B.o_pk[(size_t)(e0 + i / A.H) * B.ldopk + i % A.H] = T(0);
      if (B.o_pv)
        for (long long i = tid; i < rows * 3 * A.H; i += nth)
          B.o_pv[(size_t)(e0 + i / (3 * A.H)) * B.ldopv + i % (3 * A.H)] = T(0);
      if (!B.acc_edge) {  // accumulating: the caller's padding rows stay as they are (zero)
        for (long long i = tid; i < rows; i += nth) B.o_C[e0 + i] = T(0);
        for (long long i = tid; i < rows * 3; i += nth) B.o_u[3 * (size_t)e0 + i] = T(0);
      }
    }
  }
  if (S == 1 && t < 0) return;
  const int EPW = TMD_WAVE / A.L;
  const int c0 = G.el * V;
  const int hh = c0 / A.d, cc = c0 % A.d;
  const int vo = A.planar ? c0 : hh * 3 * A.d + cc;
  const bool hk = A.pk != nullptr, hv = A.pv != nullptr, hw = A.vec != nullptr;
  const bool head_leader = (G.el % A.lph) == 0;
  T q[V], gx[V], g0[V], g1[V], g2[V], ggq[V];
  T oq[V], ogx[V], og0[V], og1[V], og2[V];
  zero(oq); zero(ogx); zero(og0); zero(og1); zero(og2);
  if (t >= 0) {
  ldv<T, V>(q, A.q + (size_t)t * A.ldq + c0);
  ldv<T, V>(gx, A.gx + (size_t)t * A.H + c0);
  ldv<T, V>(g0, A.gvec + (size_t)t * 3 * A.H + c0);
  ldv<T, V>(g1, A.gvec + (size_t)t * 3 * A.H + A.H + c0);
  ldv<T, V>(g2, A.gvec + (size_t)t * 3 * A.H + 2 * A.H + c0);
  ldv<T, V>(ggq, B.ggq + (size_t)t * B.ldggq + c0);
  const int b = min(A.row_ptr[t], A.cap), e = min(A.row_ptr[t + 1], A.cap);
  const int step = EPW * S;
  // the per-edge scalars one edge ahead: the next edge's loads are in flight while this edge's rows
  // are gathered (one memory round trip per edge instead of two)
  int sn = 0, krn = 0;
  T Cn = T(0), u0n = T(0), u1n = T(0), u2n = T(0), gCn = T(0), g0n = T(0), g1n = T(0), g2n = T(0), scn = T(1);
  auto scalars = [&](int kk_) {
    sn = A.src[kk_];
    krn = A.prow ? A.prow[kk_] : kk_;  // pair-shared projection rows
    if (B.ggsc) scn = B.ggsc[kk_];
    Cn = A.C[kk_];
    u0n = A.u[3 * kk_]; u1n = A.u[3 * kk_ + 1]; u2n = A.u[3 * kk_ + 2];
    gCn = B.ggC[kk_];
    g0n = B.ggu[3 * kk_]; g1n = B.ggu[3 * kk_ + 1]; g2n = B.ggu[3 * kk_ + 2];
  };
  if (b + EPW * G.sub + G.es < e) scalars(b + EPW * G.sub + G.es);
  for (int k = b + EPW * G.sub + G.es; k < e; k += step) {
    const int s = sn, kr = krn;
    const T gsc = scn;
    const int kg = B.ggsc ? kr : k;  // row of the edge cotangents
    TMD_DCHECK(s >= 0 && s < A.n);
    const T Ce = Cn;
    const T u0 = u0n, u1 = u1n, u2 = u2n;
    const T ggC = gCn;
    const T gu0 = g0n, gu1 = g1n, gu2 = g2n;
    if (k + step < e) scalars(k + step);
    T pC = T(0), pu0 = T(0), pu1 = T(0), pu2 = T(0);  // accumulated edge outputs: read with the loads
    if (B.acc_edge && G.el == 0) {
      pC = B.o_C[k];
      pu0 = B.o_u[3 * k]; pu1 = B.o_u[3 * k + 1]; pu2 = B.o_u[3 * k + 2];
    }
    T kk[V], ggk[V], vx[V], v1[V], v2[V], ggvx[V], ggv1[V], ggv2[V], w0[V], w1[V], w2[V];
    T ggw0[V], ggw1[V], ggw2[V], rk[V], rx[V], r1[V], r2[V], ggpk[V], ggpx[V], ggp1[V], ggp2[V];
    ldv<T, V>(kk, A.k + (size_t)s * A.ldk + c0);
    ldv<T, V>(ggk, B.ggk + (size_t)s * B.ldggk + c0);
    const T* vs = A.v + (size_t)s * A.ldv + vo;
    ldv<T, V>(vx, vs); ldv<T, V>(v1, vs + A.vst); ldv<T, V>(v2, vs + 2 * A.vst);
    const T* gvs = B.ggv + (size_t)s * B.ldggv + vo;
    ldv<T, V>(ggvx, gvs); ldv<T, V>(ggv1, gvs + A.vst); ldv<T, V>(ggv2, gvs + 2 * A.vst);
    if (hw) {
      const T* ws = A.vec + (size_t)s * 3 * A.H + c0;
      ldv<T, V>(w0, ws); ldv<T, V>(w1, ws + A.H); ldv<T, V>(w2, ws + 2 * A.H);
    } else {
      zero(w0); zero(w1); zero(w2);
    }
    const T* gws = B.ggw + (size_t)s * 3 * A.H + c0;
    ldv<T, V>(ggw0, gws); ldv<T, V>(ggw1, gws + A.H); ldv<T, V>(ggw2, gws + 2 * A.H);
    if (hk) {
      ldv<T, V>(rk, A.pk + (size_t)kr * A.ldpk + c0);
      ldv<T, V>(ggpk, B.ggpk + (size_t)kg * B.ldggpk + c0);
    } else {
      zero(rk); zero(ggpk);
    }
    if (hv) {
      const T* ps = A.pv + (size_t)kr * A.ldpv + vo;
      ldv<T, V>(rx, ps); ldv<T, V>(r1, ps + A.vst); ldv<T, V>(r2, ps + 2 * A.vst);
      const T* gps = B.ggpv + (size_t)kg * B.ldggpv + vo;
      ldv<T, V>(ggpx, gps); ldv<T, V>(ggp1, gps + A.vst); ldv<T, V>(ggp2, gps + 2 * A.vst);
    } else {
      zero(rx); zero(r1); zero(r2); zero(ggpx); zero(ggp1); zero(ggp2);
    }
    if (B.ggsc) {
#pragma unroll
      for (int i = 0; i < V; ++i) { ggpk[i] *= gsc; ggpx[i] *= gsc; ggp1[i] *= gsc; ggp2[i] *= gsc; }
    }
    // activations with first and second derivatives (an absent projection is the constant 1)
    T dk[V], dk1[V], dk2[V], dx[V], dx1[V], dx2[V], d1[V], d11[V], d12[V], d2[V], d21[V], d22[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int ca = A.act_kv;
      if (hk) { ActF<T> f(rk[i], ca); dk[i] = f.s; dk1[i] = f.d(rk[i]); dk2[i] = f.dd(rk[i]); }
      else { dk[i] = T(1); dk1[i] = T(0); dk2[i] = T(0); }
      if (hv) {
        ActF<T> fx(rx[i], ca); dx[i] = fx.s; dx1[i] = fx.d(rx[i]); dx2[i] = fx.dd(rx[i]);
        ActF<T> f1(r1[i], ca); d1[i] = f1.s; d11[i] = f1.d(r1[i]); d12[i] = f1.dd(r1[i]);
        ActF<T> f2(r2[i], ca); d2[i] = f2.s; d21[i] = f2.d(r2[i]); d22[i] = f2.dd(r2[i]);
      } else {
        dx[i] = d1[i] = d2[i] = T(1); dx1[i] = d11[i] = d21[i] = T(0); dx2[i] = d12[i] = d22[i] = T(0);
      }
    }
    T part = T(0), ga = T(0), Sh = T(0), Xh = T(0);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      part += q[i] * kk[i] * dk[i];
      ga += gx[i] * vx[i] * dx[i];
      Sh += ggq[i] * kk[i] * dk[i] + ggk[i] * q[i] * dk[i] + ggpk[i] * q[i] * kk[i] * dk1[i];
      Xh += ggvx[i] * gx[i] * dx[i] + ggpx[i] * gx[i] * vx[i] * dx1[i];
    }
    part = group_sum(part, A.lph);
    ga = group_sum(ga, A.lph);
    Sh = group_sum(Sh, A.lph);
    Xh = group_sum(Xh, A.lph);
    const ActF<T> sa(part, A.act_at);
    const T sil = sa.s, sd = sa.d(part), sdd = sa.dd(part);
    const T gs = ga * Ce * sd, a = sil * Ce;
    const T P = Ce * ga * sdd * Sh + Ce * sd * Xh + ggC * ga * sd;
    const T Gm = Ce * sd * Sh + ggC * sil;
    const T gC = group_sum(head_leader ? ga * sd * Sh + sil * Xh : T(0), A.L);
    T ok_[V], opk[V], ovx[V], opx[V], ov1[V], op1[V], ov2[V], op2[V], ow0[V], ow1[V], ow2[V];
    T gua0 = T(0), gua1 = T(0), gua2 = T(0);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      oq[i] += P * kk[i] * dk[i] + gs * (ggk[i] * dk[i] + ggpk[i] * kk[i] * dk1[i]);
      ok_[i] = P * q[i] * dk[i] + gs * (ggq[i] * dk[i] + ggpk[i] * q[i] * dk1[i]);
      opk[i] = P * q[i] * kk[i] * dk1[i] +
               gs * ((ggq[i] * kk[i] + ggk[i] * q[i]) * dk1[i] + ggpk[i] * q[i] * kk[i] * dk2[i]);
      ogx[i] += Gm * vx[i] * dx[i] + a * (ggvx[i] * dx[i] + ggpx[i] * vx[i] * dx1[i]);
      ovx[i] = Gm * gx[i] * dx[i] + a * ggpx[i] * gx[i] * dx1[i];
      opx[i] = Gm * gx[i] * vx[i] * dx1[i] + a * (ggvx[i] * gx[i] * dx1[i] + ggpx[i] * gx[i] * vx[i] * dx2[i]);
      const T G1 = g0[i] * w0[i] + g1[i] * w1[i] + g2[i] * w2[i];
      const T G2 = g0[i] * u0 + g1[i] * u1 + g2[i] * u2;
      const T U = gu0 * g0[i] + gu1 * g1[i] + gu2 * g2[i];
      const T Wg = ggw0[i] * g0[i] + ggw1[i] * g1[i] + ggw2[i] * g2[i];
      const T B1 = ggv1[i] * d1[i] + ggp1[i] * v1[i] * d11[i];
      const T B2 = ggv2[i] * d2[i] + ggp2[i] * v2[i] * d21[i];
      const T v1e = v1[i] * d1[i], v2e = v2[i] * d2[i];
      og0[i] += w0[i] * B1 + u0 * B2 + ggw0[i] * v1e + gu0 * v2e;
      og1[i] += w1[i] * B1 + u1 * B2 + ggw1[i] * v1e + gu1 * v2e;
      og2[i] += w2[i] * B1 + u2 * B2 + ggw2[i] * v1e + gu2 * v2e;
      ow0[i] = g0[i] * B1; ow1[i] = g1[i] * B1; ow2[i] = g2[i] * B1;
      gua0 += g0[i] * B2; gua1 += g1[i] * B2; gua2 += g2[i] * B2;
      ov1[i] = G1 * ggp1[i] * d11[i] + Wg * d1[i];
      op1[i] = G1 * (ggv1[i] * d11[i] + ggp1[i] * v1[i] * d12[i]) + Wg * v1[i] * d11[i];
      ov2[i] = G2 * ggp2[i] * d21[i] + U * d2[i];
      op2[i] = G2 * (ggv2[i] * d21[i] + ggp2[i] * v2[i] * d22[i]) + U * v2[i] * d21[i];
    }
    gua0 = group_sum(gua0, A.L);
    gua1 = group_sum(gua1, A.L);
    gua2 = group_sum(gua2, A.L);
    // per-edge outputs
    if (hk) stv<T, V>(B.o_pk + (size_t)k * B.ldopk + c0, opk);
    if (hv) {
      T* op = B.o_pv + (size_t)k * B.ldopv + vo;
      stv<T, V>(op, opx); stv<T, V>(op + A.vst, op1); stv<T, V>(op + 2 * A.vst, op2);
    }
    if (G.el == 0) {
      B.o_C[k] = pC + gC;
      B.o_u[3 * k] = pu0 + gua0; B.o_u[3 * k + 1] = pu1 + gua1; B.o_u[3 * k + 2] = pu2 + gua2;
    }
    if (B.o_src) {  // source-node terms as this edge's scratch row (summed by k_bwd2_src)
      T* sr = B.o_src + (size_t)k * 7 * A.H;
      stv<T, V>(sr + c0, ok_);
      T* sv = sr + A.H + vo;
      stv<T, V>(sv, ovx); stv<T, V>(sv + A.vst, ov1); stv<T, V>(sv + 2 * A.vst, ov2);
      T* sw = sr + 4 * A.H + c0;
      stv<T, V>(sw, ow0); stv<T, V>(sw + A.H, ow1); stv<T, V>(sw + 2 * A.H, ow2);
    } else {  // source-node outputs (atomics)
#pragma unroll
      for (int i = 0; i < V; ++i) {
        atomicAdd(B.o_k + (size_t)s * B.ldok + c0 + i, ok_[i]);
        T* ov = B.o_v + (size_t)s * B.ldov + vo + i;
        atomicAdd(ov, ovx[i]); atomicAdd(ov + A.vst, ov1[i]); atomicAdd(ov + 2 * A.vst, ov2[i]);
        if (B.o_vec) {
          T* ow = B.o_vec + (size_t)s * 3 * A.H + c0 + i;
          atomicAdd(ow, ow0[i]); atomicAdd(ow + A.H, ow1[i]); atomicAdd(ow + 2 * A.H, ow2[i]);
        }
      }
    }
  }
  }  // t >= 0
  xor_slots(oq, A.L); xor_slots(ogx, A.L); xor_slots(og0, A.L); xor_slots(og1, A.L); xor_slots(og2, A.L);
  T all[5 * V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    all[i] = oq[i]; all[V + i] = ogx[i]; all[2 * V + i] = og0[i]; all[3 * V + i] = og1[i]; all[4 * V + i] = og2[i];
  }
  reduce_waves<T, S, 5 * V>(all, G.sub, lds);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    oq[i] = all[i]; ogx[i] = all[V + i]; og0[i] = all[2 * V + i]; og1[i] = all[3 * V + i]; og2[i] = all[4 * V + i];
  }
  if (t >= 0 && G.sub == 0 && G.es == 0) {
    stv<T, V>(B.o_q + (size_t)t * B.ldoq + c0, oq);
    stv<T, V>(B.o_gx + (size_t)t * A.H + c0, ogx);
    T* og = B.o_gvec + (size_t)t * 3 * A.H + c0;
    if (B.acc_gvec) {
      T p0[V], p1[V], p2[V];
      ldv<T, V>(p0, og); ldv<T, V>(p1, og + A.H); ldv<T, V>(p2, og + 2 * A.H);
#pragma unroll
      for (int i = 0; i < V; ++i) { og0[i] += p0[i]; og1[i] += p1[i]; og2[i] += p2[i]; }
    }
    stv<T, V>(og, og0); stv<T, V>(og + A.H, og1); stv<T, V>(og + 2 * A.H, og2);
  }
}

// Source pass of the second order: node j's k / v / vec terms are the sum of the scratch rows of the
// edges leaving j, i.e. the reverses tr[e'] of the edges e' of row j.  One 256-thread block per node,
// 4 columns per thread (7H / 4 = 224 threads at H = 128: every column group in one pass), the row's
// edges unrolled by 4 so their loads are in flight together (one wave per node covering the columns in
// 3.5 passes left the chip at ~3 waves per CU: 26 us per ET-QM9 layer).  A capacity-truncated
// list (a step the capacity check discards) leaves tr[e] = -1 where the reverse was cut off: no term.
template <typename T>
__global__ __launch_bounds__(256) void k_bwd2_src(Args2<T> B) {
  using V4 = T __attribute__((ext_vector_type(4)));
  const Args<T>& A = B.a;
  const int j = blockIdx.x;
  if (j >= A.n) return;
  const int W = 7 * A.H, b = min(A.row_ptr[j], A.cap), e = min(A.row_ptr[j + 1], A.cap);
  for (int c = 4 * threadIdx.x; c < W; c += 4 * blockDim.x) {
    V4 acc = {T(0), T(0), T(0), T(0)};
    int i = b;
    for (; i + 4 <= e; i += 4) {
      V4 r[4];
      int tk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        tk[u] = B.tr[i + u];
        TMD_DCHECK(tk[u] < A.cap);
        // unconditional load (row 0 for a cut-off reverse, dropped below): the four stay in flight together
        r[u] = *reinterpret_cast<const V4*>(B.o_src + (size_t)max(tk[u], 0) * W + c);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (tk[u] >= 0) acc += r[u];
    }
    for (; i < e; ++i) {
      const int k = B.tr[i];
      const V4 r1 = *reinterpret_cast<const V4*>(B.o_src + (size_t)max(k, 0) * W + c);
      if (k >= 0) acc += r1;
    }
    T* dst;
    if (c < A.H) dst = B.o_k + (size_t)j * B.ldok + c;
    else if (c < 4 * A.H) dst = B.o_v + (size_t)j * B.ldov + (c - A.H);
    else if (B.o_vec) dst = B.o_vec + (size_t)j * 3 * A.H + (c - 4 * A.H);
    else continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[u] = acc[u];
  }
}

// ------------------------------------------------------------------ neighbour embedding
template <typename T> struct NbArgs {
  int n, H, L, cap;
  const int32_t* row_ptr;
  const int32_t* src;
  const T* x; int ldx;
  const T* w; int ldw;
  const T* C;
  T* out; int ldo;         // output rows (ldo >= H: e.g. the right half of the combine input)
  const T* xself; T* oself;  // optional row copy xself[t] -> oself[t] (stride ldo): the left half
  const T* gout; int ldg;  // incoming gradient rows
  T* gx; T* gw; T* gC;
  // second order (k_nb_bwd2_*): cotangents of gx / gw / gC (NULL = 0), their VJP outputs, and the
  // transpose map tr[e] = index of the reversed edge
  const T* ggx; const T* ggw; const T* ggC;
  T* dgout; T* dx; T* dw; T* dC;
  const int32_t* tr;
};

// Edge loop of the neighbour-embedding kernels: a row's src / C for up to 64 edges arrive in one
// coalesced load and are broadcast by shuffle; NB_U edges are processed per step so their row loads
// are in flight together (one edge at a time left these kernels latency-bound).
constexpr int NB_U = 4;

// (sub, nsub): this wave takes every nsub-th group of NB_U edges of the row (waves sharing a node)
template <typename T, typename F>
__device__ __forceinline__ void nb_edges(const NbArgs<T>& A, int row, F&& body, int sub = 0, int nsub = 1) {
  const int lane = lane_id();
  const int b = min(A.row_ptr[row], A.cap), e = min(A.row_ptr[row + 1], A.cap);
  for (int base = b; base < e; base += TMD_WAVE) {
    const int cnt = min(TMD_WAVE, e - base);
    const int s_l = lane < cnt ? A.src[base + lane] : -1;
    TMD_DCHECK(lane >= cnt || (s_l >= 0 && s_l < A.n));
    const T c_l = lane < cnt ? A.C[base + lane] : T(0);
    for (int q = sub * NB_U; q < cnt; q += NB_U * nsub) {
      int sq[NB_U];
      T cq[NB_U];
#pragma unroll
      for (int u = 0; u < NB_U; ++u) {
        sq[u] = __shfl(s_l, (q + u) & (TMD_WAVE - 1));
        cq[u] = __shfl(c_l, (q + u) & (TMD_WAVE - 1));
        if (q + u >= cnt) sq[u] = -1;  // past the row end
      }
      body(base + q, sq, cq);
    }
  }
}

template <typename T, int V>
__global__ __launch_bounds__(256) void k_nb_fwd(NbArgs<T> A) {
  const int t = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (t >= A.n) return;
  const int lane = lane_id();
  const bool on = lane < A.L;
  const int c0 = on ? lane * V : 0;
  T acc[V];
  zero(acc);
  nb_edges(A, t, [&](int k0, const int (&sq)[NB_U], const T (&cq)[NB_U]) {
    T xs[NB_U][V], wk[NB_U][V];
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const bool live = sq[u] >= 0 && sq[u] != t;
      const int s = live ? sq[u] : t, k = live ? k0 + u : k0;
      ldv<T, V>(xs[u], A.x + (size_t)s * A.ldx + c0);
      ldv<T, V>(wk[u], A.w + (size_t)k * A.ldw + c0);
      const T ce = live ? cq[u] : T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) wk[u][i] *= ce;
    }
#pragma unroll
    for (int u = 0; u < NB_U; ++u)
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += xs[u][i] * wk[u][i];
  });
  if (on) stv<T, V>(A.out + (size_t)t * A.ldo + c0, acc);
  if (on && A.xself) {  // the combine Linear's [x | x_nb] input in one buffer: no concatenation
    T xv[V];
    ldv<T, V>(xv, A.xself + (size_t)t * A.H + c0);
    stv<T, V>(A.oself + (size_t)t * A.ldo + c0, xv);
  }
}

// destination pass: gw[e] = gout[t] * x[s] * C[e], gC[e] = sum_c gout[t] x[s] w[e]; the static-capacity
// padding slots [row_ptr[n], cap) of gw / gC are zeroed here too (no memset before the launch)
template <typename T, int V>
__global__ __launch_bounds__(256) void k_nb_bwd_dst(NbArgs<T> A) {
  {
    const int e0 = min(A.row_ptr[A.n], A.cap);
    const long long rows = A.cap - e0;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
    for (long long i = tid; i < rows * A.H; i += nth) A.gw[(size_t)e0 * A.H + i] = T(0);
    for (long long i = tid; i < rows; i += nth) A.gC[e0 + i] = T(0);
  }
  // four waves per node, each a quarter of the row's edges (the outputs are per edge: no reduction;
  // one wave per node left a QM9 batch at ~3 waves per CU)
  const int t = blockIdx.x, sub = threadIdx.x / TMD_WAVE, nsub = blockDim.x / TMD_WAVE;
  if (t >= A.n) return;
  const int lane = lane_id();
  const bool on = lane < A.L;
  const int c0 = on ? lane * V : 0;
  T go[V];
  ldv<T, V>(go, A.gout + (size_t)t * A.ldg + c0);
  nb_edges(A, t, [&](int k0, const int (&sq)[NB_U], const T (&cq)[NB_U]) {
    T xs[NB_U][V], wk[NB_U][V], gc[NB_U];
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const bool valid = sq[u] >= 0;
      const bool live = valid && sq[u] != t;
      const int s = live ? sq[u] : t, k = valid ? k0 + u : k0;
      ldv<T, V>(xs[u], A.x + (size_t)s * A.ldx + c0);
      ldv<T, V>(wk[u], A.w + (size_t)k * A.ldw + c0);
    }
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const bool valid = sq[u] >= 0;
      const bool live = valid && sq[u] != t;
      const T ce = live ? cq[u] : T(0);
      T gw[V];
      gc[u] = T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        gw[i] = go[i] * xs[u][i] * ce;
        gc[u] += go[i] * xs[u][i] * wk[u][i];
      }
      if (!live) gc[u] = T(0);
      if (on && valid) stv<T, V>(A.gw + (size_t)(k0 + u) * A.H + c0, gw);
    }
#pragma unroll
    for (int u = 0; u < NB_U; ++u) gc[u] = wave_sum(on ? gc[u] : T(0));
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < NB_U; ++u)
        if (sq[u] >= 0) A.gC[k0 + u] = gc[u];
    }
  }, sub, nsub);
}

// source pass: gx[j] = sum_{reverse edges j->m} gout[m] * w[e] * C[e]
template <typename T, int V>
__global__ __launch_bounds__(256) void k_nb_bwd_src(NbArgs<T> A) {
  const int j = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (j >= A.n) return;
  const int lane = lane_id();
  const bool on = lane < A.L;
  const int c0 = on ? lane * V : 0;
  T acc[V];
  zero(acc);
  nb_edges(A, j, [&](int k0, const int (&sq)[NB_U], const T (&cq)[NB_U]) {
    T gm[NB_U][V], wk[NB_U][V];
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const bool live = sq[u] >= 0 && sq[u] != j;
      const int m = live ? sq[u] : j, k = live ? k0 + u : k0;
      ldv<T, V>(gm[u], A.gout + (size_t)m * A.ldg + c0);
      ldv<T, V>(wk[u], A.w + (size_t)k * A.ldw + c0);
      const T ce = live ? cq[u] : T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) wk[u][i] *= ce;
    }
#pragma unroll
    for (int u = 0; u < NB_U; ++u)
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += gm[u][i] * wk[u][i];
  });
  if (on) stv<T, V>(A.gx + (size_t)j * A.H + c0, acc);
}

// Second order of the neighbour embedding (force-matching training; the forward is trilinear in
// (x, w, C), so its backward's VJP for cotangents (ggx, ggw, ggC) of (gx, gw, gC) is):
//   d_gout[t] = sum_{e in row t} ggx[s] w_e C_e + x[s] (ggw_e C_e + ggC_e w_e)
//   d_w[e]    = C_e ggx[s] gout[t] + ggC_e gout[t] x[s]
//   d_C[e]    = sum_c gout[t] (ggx[s] w_e + ggw_e x[s])                       (destination pass)
//   d_x[s]    = sum_{e: src_e = s} gout[dst_e] (ggw_e C_e + ggC_e w_e)         (source pass: the
//               edges leaving s are the reverses tr[e'] of the edges e' of row s)
// Self loops (and padding) contribute nothing, as in the forward.
template <typename T, int V>
__global__ __launch_bounds__(256) void k_nb_bwd2_dst(NbArgs<T> A) {
  const int t = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (t >= A.n) return;
  const int lane = lane_id();
  const bool on = lane < A.L;
  const int c0 = on ? lane * V : 0;
  T go[V], acc[V];
  ldv<T, V>(go, A.gout + (size_t)t * A.ldg + c0);
  zero(acc);
  nb_edges(A, t, [&](int k0, const int (&sq)[NB_U], const T (&cq)[NB_U]) {
    T xs[NB_U][V], wk[NB_U][V], gxs[NB_U][V], gwk[NB_U][V], gck[NB_U], dc[NB_U];
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const bool valid = sq[u] >= 0;
      const bool live = valid && sq[u] != t;
      const int s = live ? sq[u] : t, k = valid ? k0 + u : k0;
      ldv<T, V>(xs[u], A.x + (size_t)s * A.ldx + c0);
      ldv<T, V>(wk[u], A.w + (size_t)k * A.ldw + c0);
      if (A.ggx) ldv<T, V>(gxs[u], A.ggx + (size_t)s * A.H + c0); else zero(gxs[u]);
      if (A.ggw) ldv<T, V>(gwk[u], A.ggw + (size_t)k * A.H + c0); else zero(gwk[u]);
      gck[u] = (A.ggC && live) ? A.ggC[k] : T(0);
    }
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const bool valid = sq[u] >= 0;
      const bool live = valid && sq[u] != t;
      const T ce = live ? cq[u] : T(0), gc = gck[u];
      T dw[V];
      dc[u] = T(0);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        acc[i] += ce * (gxs[u][i] * wk[u][i] + xs[u][i] * gwk[u][i]) + gc * xs[u][i] * wk[u][i];
        dw[i] = live ? go[i] * (ce * gxs[u][i] + gc * xs[u][i]) : T(0);
        dc[u] += go[i] * (gxs[u][i] * wk[u][i] + gwk[u][i] * xs[u][i]);
      }
      if (!live) dc[u] = T(0);
      if (on && valid && A.dw) stv<T, V>(A.dw + (size_t)(k0 + u) * A.H + c0, dw);
    }
    if (A.dC) {
#pragma unroll
      for (int u = 0; u < NB_U; ++u) dc[u] = wave_sum(on ? dc[u] : T(0));
      if (lane == 0) {
#pragma unroll
        for (int u = 0; u < NB_U; ++u)
          if (sq[u] >= 0) A.dC[k0 + u] = dc[u];
      }
    }
  });
  if (on && A.dgout) stv<T, V>(A.dgout + (size_t)t * A.H + c0, acc);
}

template <typename T, int V>
__global__ __launch_bounds__(256) void k_nb_bwd2_src(NbArgs<T> A) {
  const int j = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (j >= A.n) return;
  const int lane = lane_id();
  const bool on = lane < A.L;
  const int c0 = on ? lane * V : 0;
  T acc[V];
  zero(acc);
  nb_edges(A, j, [&](int k0, const int (&sq)[NB_U], const T (&cq)[NB_U]) {
    T gm[NB_U][V], wk[NB_U][V], gwk[NB_U][V], ck[NB_U], gck[NB_U];
#pragma unroll
    for (int u = 0; u < NB_U; ++u) {
      const int kt = sq[u] >= 0 ? A.tr[k0 + u] : -1;  // the edge j -> m
      const bool live = kt >= 0 && sq[u] != j;
      const int m = live ? sq[u] : j;
      const int k = live ? kt : k0;
      TMD_DCHECK(!live || k < A.cap);
      ldv<T, V>(gm[u], A.gout + (size_t)m * A.ldg + c0);
      ldv<T, V>(wk[u], A.w + (size_t)k * A.ldw + c0);
      if (A.ggw) ldv<T, V>(gwk[u], A.ggw + (size_t)k * A.H + c0); else zero(gwk[u]);
      ck[u] = live ? A.C[k] : T(0);
      gck[u] = (live && A.ggC) ? A.ggC[k] : T(0);
    }
#pragma unroll
    for (int u = 0; u < NB_U; ++u)
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += gm[u][i] * (gwk[u][i] * ck[u] + gck[u] * wk[u][i]);
  });
  if (on) stv<T, V>(A.dx + (size_t)j * A.H + c0, acc);
}

// ------------------------------------------------------------------ host helpers
static inline int pick_vec(int H) {
  if (H % 256 == 0) return 4;
  if (H % 128 == 0) return 2;
  return 1;
}

template <typename T>
static bool aligned(const void* p, int ld, int V) {
  if (!p) return true;
  return ((uintptr_t)p % (sizeof(T) * V)) == 0 && (ld % V) == 0;
}

template <typename T, template <typename, int> class K, typename AT>
static int launch_v(int V, int n, AT A, hipStream_t st) {
  const int tb = 256, wpb = tb / TMD_WAVE;
  dim3 g((n + wpb - 1) / wpb);
  if (n <= 0) return kOk;
  if (V == 1) hipLaunchKernelGGL((K<T, 1>::fn), g, dim3(tb), 0, st, A);
  else if (V == 2) hipLaunchKernelGGL((K<T, 2>::fn), g, dim3(tb), 0, st, A);
  else hipLaunchKernelGGL((K<T, 4>::fn), g, dim3(tb), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// ET launch: V = H/32 channels per lane (half-wave per edge), S waves per node (small systems get
// S = 4 so that e.g. a 678-atom QM9 batch still puts ~2.7k waves on the 256 CUs).
static inline int et_waves_per_node(int n, int bytes_per_lane_vec) {
  if (bytes_per_lane_vec > 32) return 1;
  static const int env_s = [] { const char* e = getenv("TMDNET_ET_S"); return e ? atoi(e) : 0; }();  // tuning, read once
  if (env_s > 0) return env_s >= 4 ? 4 : env_s >= 2 ? 2 : 1;
  if (n < 4096) return 4;
  if (n < 8192) return 2;
  return 1;
}

template <typename T, int V, int S, int KIND, bool ORD, bool GA>
static int et_launch_k(const Args<T>& A, dim3 g, dim3 b, int nbn, hipStream_t st);

template <typename T, int V, int S, int KIND, bool ORD>
static int et_launch_vs(Args<T> A, hipStream_t st) {
  // channel groups: split heads across XCDs for large systems (L2 working-set), not for the
  // destination pass (its per-edge channel sums would need a cross-group combine)
  // channel groups (CS = 2 / 4) are supported by the kernels but measured neutral (+-1 %) on the
  // C5 water box (tools/kbench.py), so one group is used.
  int cs = 1;
  if (KIND == 1 || A.H % (cs * V) || (A.H / cs / V) & (A.H / cs / V - 1) || A.H / cs / V < A.lph ||
      A.H / cs / V > 64)
    cs = 1;
  A.HC = A.H / cs;
  A.L = A.HC / V;
  if (A.L > 64 || (A.L & (A.L - 1))) return kUnsupported;
  const int nbn = (A.n + (4 / S) - 1) / (4 / S);
  const dim3 g(nbn * cs), b(256);
  // SiLU / SiLU (the configs' activations) runs kernels with the codes as compile-time constants: the
  // runtime-code form splits every per-edge activation into its own basic block (C2: k_bwd_both
  // 226 -> 264 us, k_fwd 83 -> 90 us per step when it was the only form)
  if (A.act_kv == kActSilu && A.act_at == kActSilu)
    return et_launch_k<T, V, S, KIND, ORD, false>(A, g, b, nbn, st);
  return et_launch_k<T, V, S, KIND, ORD, true>(A, g, b, nbn, st);
}

template <typename T, int V, int S, int KIND, bool ORD, bool GA>
static int et_launch_k(const Args<T>& A, dim3 g, dim3 b, int nbn, hipStream_t st) {
  if (KIND == 0) hipLaunchKernelGGL((k_fwd<T, V, S, 1, ORD, GA>), g, b, 0, st, A);
  else if (KIND == 1) hipLaunchKernelGGL((k_bwd_dst<T, V, S, 1, false, false, GA>), g, b, 0, st, A);
  else if (KIND == 2) hipLaunchKernelGGL((k_bwd_src<T, V, S, 1, GA>), g, b, 0, st, A);
  else if (KIND == 3) hipLaunchKernelGGL((k_bwd_both<T, V, S, 1, false, false, GA>), dim3(2 * nbn), b, 0, st, A);
  else if (KIND == 4) hipLaunchKernelGGL((k_bwd_dst<T, V, S, 1, true, false, GA>), g, b, 0, st, A);
  else if (KIND == 5) hipLaunchKernelGGL((k_bwd_both<T, V, S, 1, true, false, GA>), dim3(2 * nbn), b, 0, st, A);
  else if (KIND == 6) hipLaunchKernelGGL((k_bwd_both<T, V, S, 1, false, true, GA>), dim3(2 * nbn), b, 0, st, A);
  else if (KIND == 8 || KIND == 9) {
    // dynamic LDS: the node vectors of the block's 4 / S nodes, or the cross-wave reduction
    const size_t node = (size_t)(4 / S) * 12 * A.H, red = S > 1 ? 4 * 64 * 8 * V : 1;
    const size_t bytes = (node > red ? node : red) * sizeof(T);
    if (KIND == 8) hipLaunchKernelGGL((k_bwd_merged<T, V, S, 1, GA>), dim3(nbn), b, bytes, st, A);
    else hipLaunchKernelGGL((k_bwd_merged<T, V, S, 0, GA>), dim3(nbn), b, bytes, st, A);
  }
  else hipLaunchKernelGGL((k_bwd_dst<T, V, S, 1, false, true, GA>), g, b, 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// below this many nodes the two backward passes share one grid (k_bwd_both)
static constexpr int kBwdFuseNodes = 16384;

// size switches of the backward's launch forms, settable at run time (tmdnet_set_tuning: tests force the
// large-system forms on small graphs); first read from TMDNET_ET_FUSE / TMDNET_ET_MERGED_MIN
static int g_tune[3] = {-1, -1, -1};
static int tune_get(int key) {
  int& v = g_tune[key];
  if (v < 0) {
    const char* e = getenv(key == TMDNET_TUNE_ET_BOTH_MAX_NODES ? "TMDNET_ET_FUSE" : "TMDNET_ET_MERGED_MIN");
    v = e ? atoi(e) : kBwdFuseNodes;
  }
  return v;
}

template <typename T, int V, int KIND, bool ORD>
static int et_launch_v(const Args<T>& A, hipStream_t st) {
  int S = et_waves_per_node(A.n, (int)sizeof(T) * V);
  // the forward keeps 4 waves per node at every size: on the C5 probe (pair rows) 1.158 vs 1.196 ms at 1
  // wave (r04, tools/pair_probe.py; fewer nodes in flight per XCD, so more of each pair row's second read
  // hits L2); the backward passes are faster at 1 there (3.25 vs 3.52 ms)
  static const bool env_s_set = getenv("TMDNET_ET_S") != nullptr;
  if (KIND == 0 && !env_s_set && (int)sizeof(T) * V <= 32) S = 4;
  static const int bwd_s = getenv("TMDNET_ET_BWD_S") ? atoi(getenv("TMDNET_ET_BWD_S")) : 0;  // tuning
  if (KIND != 0 && bwd_s && (int)sizeof(T) * V <= 32) S = bwd_s >= 4 ? 4 : bwd_s >= 2 ? 2 : 1;
  if (S == 4) return et_launch_vs<T, V, (sizeof(T) * V <= 32 ? 4 : 1), KIND, ORD>(A, st);
  if (S == 2) return et_launch_vs<T, V, (sizeof(T) * V <= 32 ? 2 : 1), KIND, ORD>(A, st);
  return et_launch_vs<T, V, 1, KIND, ORD>(A, st);
}

template <typename T, int KIND, bool ORD>
static int et_launch(int V, const Args<T>& A, hipStream_t st) {
  if (A.n <= 0) return kOk;
  switch (V) {
    case 1: return et_launch_v<T, 1, KIND, ORD>(A, st);
    case 2: return et_launch_v<T, 2, KIND, ORD>(A, st);
    case 4: return et_launch_v<T, 4, KIND, ORD>(A, st);
    case 8: return et_launch_v<T, 8, KIND, ORD>(A, st);
  }
  return kUnsupported;
}

template <typename T, int V> struct KNbFwd { static constexpr auto fn = k_nb_fwd<T, V>; };
template <typename T, int V> struct KNbDst { static constexpr auto fn = k_nb_bwd_dst<T, V>; };
template <typename T, int V> struct KNbSrc { static constexpr auto fn = k_nb_bwd_src<T, V>; };
template <typename T, int V> struct KNb2Dst { static constexpr auto fn = k_nb_bwd2_dst<T, V>; };
template <typename T, int V> struct KNb2Src { static constexpr auto fn = k_nb_bwd2_src<T, V>; };

template <typename T>
static int setup(Args<T>& A, int n, int H, int heads, const int32_t* row_ptr, const int32_t* src,
                 int cap, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv_,
                 const void* vec, const void* pk, int ldpk, const void* pv, int ldpv, const void* C,
                 const void* u, const int32_t* order, int& V, const int32_t* prow = nullptr) {
  if (H <= 0 || heads <= 0 || H % heads) return kBadArgument;
  if (H % 32 == 0) V = H / 32;  // channels per lane, one edge per half-wave
  else if (H < 32) V = 1;       // fewer channels than half-wave lanes: idle lanes
  else return kUnsupported;

  if (V != 1 && V != 2 && V != 4 && V != 8) return kUnsupported;
  const int d = H / heads;
  if (d % V) return kUnsupported;
  const int lph = d / V;
  if (lph & (lph - 1)) return kUnsupported;  // a head must be a power-of-two lane group
  const int VA = V > 4 ? 4 : V;               // vector width of one load
  if (!aligned<T>(q, ldq, VA) || !aligned<T>(k, ldk, VA) || !aligned<T>(v, ldv_, VA) ||
      !aligned<T>(pk, ldpk, VA) || !aligned<T>(pv, ldpv, VA) || !aligned<T>(vec, H, VA))
    return kBadArgument;
  A = Args<T>{};
  A.n = n; A.H = H; A.d = d; A.L = H / V; A.HC = H; A.lph = lph; A.cap = cap;
  A.planar = 0; A.vst = d;
  A.row_ptr = row_ptr; A.src = src; A.order = order;
  A.xcd = 1;
  A.q = (const T*)q; A.ldq = ldq; A.k = (const T*)k; A.ldk = ldk; A.v = (const T*)v; A.ldv = ldv_;
  A.vec = (const T*)vec; A.pk = (const T*)pk; A.ldpk = ldpk; A.pv = (const T*)pv; A.ldpv = ldpv;
  A.prow = prow;
  A.C = (const T*)C; A.u = (const T*)u;
  return kOk;
}

// the activation codes of a call's flags (TMDNET_ET_ACT bits 8-11 / 12-15)
template <typename T>
static int set_acts(Args<T>& A, int flags) {
  A.act_kv = (flags >> 8) & 15;
  A.act_at = (flags >> 12) & 15;
  return (A.act_kv > kActSigmoid || A.act_at > kActSigmoid) ? kBadArgument : kOk;
}

template <typename T>
static int fwd(int n, int H, int heads, const int32_t* row_ptr, const int32_t* src, int cap,
               const void* q, int ldq, const void* k, int ldk, const void* v, int ldv_,
               const void* vec, const void* pk, int ldpk, const void* pv, int ldpv, const void* C,
               const void* u, void* xo, void* veco, int flags, const int32_t* prow, const int32_t* order,
               hipStream_t st) {
  Args<T> A;
  int V;
  int rc = setup<T>(A, n, H, heads, row_ptr, src, cap, q, ldq, k, ldk, v, ldv_, vec, pk, ldpk, pv,
                    ldpv, C, u, order, V, prow);
  if (rc) return rc;
  if ((rc = set_acts(A, flags))) return rc;
  if (flags & TMDNET_ET_V_PLANAR) { A.planar = 1; A.vst = H; }
  A.xo = (T*)xo;
  A.veco = (T*)veco;
  return order ? et_launch<T, 0, true>(V, A, st) : et_launch<T, 0, false>(V, A, st);
}

template <typename T>
static int bwd(int n, int H, int heads, const int32_t* row_ptr, const int32_t* src, int cap,
               const void* q, int ldq, const void* k, int ldk, const void* v, int ldv_,
               const void* vec, const void* pk, int ldpk, const void* pv, int ldpv, const void* C,
               const void* u, const void* gx, const void* gvec, void* gq, void* gk, void* gv,
               void* gveci, void* gpk, void* gpv, void* gC, void* gu, const void* dpk, const void* dpv,
               void* gr, int acc, const int32_t* prow, const int32_t* order, hipStream_t st) {
  Args<T> A;
  int V;
  int rc = setup<T>(A, n, H, heads, row_ptr, src, cap, q, ldq, k, ldk, v, ldv_, vec, pk, ldpk, pv,
                    ldpv, C, u, order, V, prow);
  if (rc) return rc;
  A.gx = (const T*)gx; A.gvec = (const T*)gvec;
  A.gq = (T*)gq; A.gk = (T*)gk; A.gv = (T*)gv; A.gveci = (T*)gveci;
  A.gpk = (T*)gpk; A.gpv = (T*)gpv; A.gC = (T*)gC; A.gu = (T*)gu;
  A.dpk = (const T*)dpk; A.dpv = (const T*)dpv; A.gr = (T*)gr;
  A.acc = acc;
  if ((rc = set_acts(A, acc))) return rc;
  static const int bwd_v = getenv("TMDNET_ET_BWD_V") ? atoi(getenv("TMDNET_ET_BWD_V")) : 0;  // tuning
  if (bwd_v && bwd_v < V && H % (32 * bwd_v) == 0 && H / bwd_v <= 64 && (A.d / bwd_v) > 0 &&
      A.d % bwd_v == 0 && !((A.d / bwd_v) & (A.d / bwd_v - 1))) {
    V = bwd_v;
    A.lph = A.d / V;
  }
  if (acc & TMDNET_ET_V_PLANAR) { A.planar = 1; A.vst = H; }
  const bool dr = gr != nullptr;
  if (dr && ((A.pk && !dpk) || (A.pv && !dpv))) return kBadArgument;
  if (!dr && ((A.pk && !gpk) || (A.pv && !gpv))) return kBadArgument;
  const int fuse_nodes = tune_get(TMDNET_TUNE_ET_BOTH_MAX_NODES);
  const bool ag = !dr && (acc & TMDNET_ACC_GRADS) && (A.pk || A.pv);  // injected projection cotangents
  // dr mode: both roles in one pass over the rows (k_bwd_merged)
  // (tuning: TMDNET_ET_MERGED=0 off, 1 stream-prefetching variant, 2 loads per edge in the body).
  // Large graphs only: C5 2.97 vs 3.38 ms per layer (the two passes); at C2 the two passes in one
  // grid (k_bwd_both, twice the waves at 167 vs 222 VGPRs) win, 51 vs 69 us.
  static const int merged = getenv("TMDNET_ET_MERGED") ? atoi(getenv("TMDNET_ET_MERGED")) : 1;
  const int merged_min = tune_get(TMDNET_TUNE_ET_MERGED_MIN_NODES);
  if (dr && merged && n >= merged_min && !(acc & TMDNET_ET_TWO_PASS) && !A.gpk && !A.gpv)
    return merged == 2 ? et_launch<T, 9, false>(V, A, st) : et_launch<T, 8, false>(V, A, st);
  if (n < fuse_nodes)
    return dr ? et_launch<T, 5, false>(V, A, st) : ag ? et_launch<T, 6, false>(V, A, st) : et_launch<T, 3, false>(V, A, st);
  rc = dr ? et_launch<T, 4, false>(V, A, st) : ag ? et_launch<T, 7, false>(V, A, st) : et_launch<T, 1, false>(V, A, st);
  if (rc) return rc;
  return et_launch<T, 2, false>(V, A, st);
}

struct Bwd2Ex {  // the strides / accumulation / source-pass extras of tmdnet_et_message_bwd2_ex
  int ldggq, ldggk, ldggv, ldoq, ldok, ldov, ldopk, ldopv;
  const int32_t* tr;
  void* scratch;
  const int32_t* prow;  // pk / pv row of every edge (pair-shared rows); NULL: row e
  const void* ggsc;     // per-edge scale of pair-row edge cotangents (Args2::ggsc)
};

template <typename T>
static int bwd2(int n, int H, int heads, const int32_t* row_ptr, const int32_t* src, int cap,
                const void* q, int ldq, const void* k, int ldk, const void* v, int ldv_,
                const void* vec, const void* pk, int ldpk, const void* pv, int ldpv, const void* C,
                const void* u, const void* gx, const void* gvec, const void* ggq, const void* ggk,
                const void* ggv, const void* ggw, const void* ggpk, int ldggpk, const void* ggpv,
                int ldggpv, const void* ggC, const void* ggu, void* o_gx, void* o_gvec, void* o_q,
                void* o_k, void* o_v, void* o_vec, void* o_pk, void* o_pv, void* o_C, void* o_u,
                int flags, hipStream_t st, const Bwd2Ex* ex = nullptr) {
  Args2<T> B{};
  int V;
  int rc = setup<T>(B.a, n, H, heads, row_ptr, src, cap, q, ldq, k, ldk, v, ldv_, vec, pk, ldpk, pv,
                    ldpv, C, u, nullptr, V);
  if (rc) return rc;
  // narrower lanes than the first-order kernels (V = H/64: one edge per wave instruction): this
  // kernel keeps ~22 row segments of an edge live
  if (H % 64 == 0) V = H / 64;
  const int d = H / heads;
  if ((V != 1 && V != 2 && V != 4) || d % V || ((d / V) & (d / V - 1))) return kUnsupported;
  B.a.L = H / V;
  B.a.lph = d / V;
  if (B.a.L > 64 || (B.a.L & (B.a.L - 1))) return kUnsupported;
  if (!aligned<T>(ggpk, ldggpk, V) || !aligned<T>(ggpv, ldggpv, V)) return kBadArgument;
  if ((rc = set_acts(B.a, flags))) return rc;
  if (flags & TMDNET_ET_V_PLANAR) { B.a.planar = 1; B.a.vst = H; }
  B.a.gx = (const T*)gx; B.a.gvec = (const T*)gvec;
  B.ggq = (const T*)ggq; B.ggk = (const T*)ggk; B.ggv = (const T*)ggv; B.ggw = (const T*)ggw;
  B.ggpk = (const T*)ggpk; B.ldggpk = ldggpk; B.ggpv = (const T*)ggpv; B.ldggpv = ldggpv;
  B.ggC = (const T*)ggC; B.ggu = (const T*)ggu;
  B.o_gx = (T*)o_gx; B.o_gvec = (T*)o_gvec; B.o_q = (T*)o_q; B.o_k = (T*)o_k; B.o_v = (T*)o_v;
  B.o_vec = (T*)o_vec; B.o_pk = (T*)o_pk; B.o_pv = (T*)o_pv; B.o_C = (T*)o_C; B.o_u = (T*)o_u;
  B.ldggq = B.ldok = B.ldoq = H; B.ldggk = H; B.ldggv = B.ldov = 3 * H; B.ldopk = H; B.ldopv = 3 * H;
  if (ex) {
    auto pick = [](int x, int dflt) { return x ? x : dflt; };
    B.ldggq = pick(ex->ldggq, H); B.ldggk = pick(ex->ldggk, H); B.ldggv = pick(ex->ldggv, 3 * H);
    B.ldoq = pick(ex->ldoq, H); B.ldok = pick(ex->ldok, H); B.ldov = pick(ex->ldov, 3 * H);
    B.ldopk = pick(ex->ldopk, H); B.ldopv = pick(ex->ldopv, 3 * H);
    if (B.ldggq < H || B.ldggk < H || B.ldggv < 3 * H || B.ldoq < H || B.ldok < H || B.ldov < 3 * H ||
        B.ldopk < H || B.ldopv < 3 * H)
      return kBadArgument;
    if (!aligned<T>(ggq, B.ldggq, V) || !aligned<T>(ggk, B.ldggk, V) || !aligned<T>(ggv, B.ldggv, V) ||
        !aligned<T>(o_q, B.ldoq, V) || !aligned<T>(o_pk, B.ldopk, V) || !aligned<T>(o_pv, B.ldopv, V))
      return kBadArgument;
    if ((ex->tr == nullptr) != (ex->scratch == nullptr)) return kBadArgument;
    if (ex->scratch) {
      // the source pass stores 4-wide rows: 16-byte aligned node rows and scratch
      if (H % 4 || B.ldok % 4 || B.ldov % 4 || ((uintptr_t)o_k % (4 * sizeof(T))) ||
          ((uintptr_t)o_v % (4 * sizeof(T))) || ((uintptr_t)ex->scratch % (4 * sizeof(T))))
        return kBadArgument;
      B.tr = ex->tr;
      B.o_src = (T*)ex->scratch;
    }
    B.a.prow = ex->prow;
    if (ex->ggsc && !ex->prow) return kBadArgument;
    B.ggsc = (const T*)ex->ggsc;
  }
  B.acc_edge = (flags & TMDNET_BWD2_ACC_EDGE) ? 1 : 0;
  B.acc_gvec = (flags & TMDNET_BWD2_ACC_GVEC) ? 1 : 0;
  if (n <= 0) return kOk;
  // waves per node (small systems: fill the chip); TMDNET_BWD2_S overrides (tuning)
  static const int s_env = getenv("TMDNET_BWD2_S") ? atoi(getenv("TMDNET_BWD2_S")) : 0;
  int S = n < 2048 ? 8 : (n < 4096 ? 4 : (n < 8192 ? 2 : 1));
  if (s_env == 1 || s_env == 2 || s_env == 4 || s_env == 8) S = s_env;
  if (S == 8 && V != 2) S = 4;
  const dim3 g(S == 8 ? n : (n + 4 / S - 1) / (4 / S)), b(S == 8 ? 512 : 256);
#define TMD_L2(VV, SS) hipLaunchKernelGGL((k_bwd2<T, VV, SS>), g, b, 0, st, B)
  if (V == 1) { if (S == 4) TMD_L2(1, 4); else if (S == 2) TMD_L2(1, 2); else TMD_L2(1, 1); }
  else if (V == 2) {
    if (S == 8) TMD_L2(2, 8); else if (S == 4) TMD_L2(2, 4); else if (S == 2) TMD_L2(2, 2); else TMD_L2(2, 1);
  }
  else { if (S == 4) TMD_L2(4, 4); else if (S == 2) TMD_L2(4, 2); else TMD_L2(4, 1); }
#undef TMD_L2
  if (hipGetLastError() != hipSuccess) return kLaunchFailed;
  if (B.o_src) hipLaunchKernelGGL(k_bwd2_src<T>, dim3(n), dim3(256), 0, st, B);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static int nb_setup(NbArgs<T>& A, int n, int H, const int32_t* row_ptr, const int32_t* src, int cap,
                    const void* x, int ldx, const void* w, int ldw, const void* C, int& V) {
  V = pick_vec(H);
  if (H / V > TMD_WAVE || H % V) return kUnsupported;
  if (!aligned<T>(x, ldx, V) || !aligned<T>(w, ldw, V)) return kBadArgument;
  A = NbArgs<T>{};
  A.n = n; A.H = H; A.L = H / V; A.cap = cap; A.row_ptr = row_ptr; A.src = src;
  A.x = (const T*)x; A.ldx = ldx; A.w = (const T*)w; A.ldw = ldw; A.C = (const T*)C;
  return kOk;
}

}  // namespace et
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_et_message_fwd(int dtype, int n_nodes, int hidden, int heads,
                                     const int32_t* row_ptr, const int32_t* src, int max_pairs,
                                     const void* q, int ld_q, const void* k, int ld_k, const void* v,
                                     int ld_v, const void* vec_in, const void* pk, int ld_pk,
                                     const void* pv, int ld_pv, const void* cutoff, const void* unit,
                                     void* x_out, void* vec_out, int flags, const int32_t* pk_rows,
                                     const int32_t* order, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return et::fwd<float>(n_nodes, hidden, heads, row_ptr, src, max_pairs, q, ld_q, k, ld_k, v, ld_v,
                          vec_in, pk, ld_pk, pv, ld_pv, cutoff, unit, x_out, vec_out, flags, pk_rows, order, st);
  if (dtype == TMDNET_F64)
    return et::fwd<double>(n_nodes, hidden, heads, row_ptr, src, max_pairs, q, ld_q, k, ld_k, v, ld_v,
                           vec_in, pk, ld_pk, pv, ld_pv, cutoff, unit, x_out, vec_out, flags, pk_rows, order,
                           st);
  return kUnsupported;
}

extern "C" int tmdnet_et_message_bwd(int dtype, int n_nodes, int hidden, int heads,
                                     const int32_t* row_ptr, const int32_t* src, int max_pairs,
                                     const void* q, int ld_q, const void* k, int ld_k, const void* v,
                                     int ld_v, const void* vec_in, const void* pk, int ld_pk,
                                     const void* pv, int ld_pv, const void* cutoff, const void* unit,
                                     const void* grad_x, const void* grad_vec, void* gq, void* gk,
                                     void* gv, void* gvec_in, void* gpk, void* gpv, void* gcut,
                                     void* gunit, const void* dpk, const void* dpv, void* gdist,
                                     int accumulate, const int32_t* pk_rows, const int32_t* order,
                                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return et::bwd<float>(n_nodes, hidden, heads, row_ptr, src, max_pairs, q, ld_q, k, ld_k, v, ld_v,
                          vec_in, pk, ld_pk, pv, ld_pv, cutoff, unit, grad_x, grad_vec, gq, gk, gv,
                          gvec_in, gpk, gpv, gcut, gunit, dpk, dpv, gdist, accumulate, pk_rows, order, st);
  if (dtype == TMDNET_F64)
    return et::bwd<double>(n_nodes, hidden, heads, row_ptr, src, max_pairs, q, ld_q, k, ld_k, v, ld_v,
                           vec_in, pk, ld_pk, pv, ld_pv, cutoff, unit, grad_x, grad_vec, gq, gk, gv,
                           gvec_in, gpk, gpv, gcut, gunit, dpk, dpv, gdist, accumulate, pk_rows, order, st);
  return kUnsupported;
}

extern "C" int tmdnet_et_message_bwd2(
    int dtype, int n_nodes, int hidden, int heads, const int32_t* row_ptr, const int32_t* src,
    int max_pairs, const void* q, int ld_q, const void* k, int ld_k, const void* v, int ld_v,
    const void* vec_in, const void* pk, int ld_pk, const void* pv, int ld_pv, const void* cutoff,
    const void* unit, const void* grad_x, const void* grad_vec, const void* gg_q, const void* gg_k,
    const void* gg_v, const void* gg_vec, const void* gg_pk, int ld_ggpk, const void* gg_pv,
    int ld_ggpv, const void* gg_cut, const void* gg_unit, void* d_grad_x, void* d_grad_vec,
    void* d_q, void* d_k, void* d_v, void* d_vec, void* d_pk, void* d_pv, void* d_cut,
    void* d_unit, int flags, void* stream) {
  hipStream_t st = (hipStream_t)stream;
#define TMD_BWD2(T)                                                                              \
  return et::bwd2<T>(n_nodes, hidden, heads, row_ptr, src, max_pairs, q, ld_q, k, ld_k, v, ld_v, \
                     vec_in, pk, ld_pk, pv, ld_pv, cutoff, unit, grad_x, grad_vec, gg_q, gg_k,   \
                     gg_v, gg_vec, gg_pk, ld_ggpk, gg_pv, ld_ggpv, gg_cut, gg_unit, d_grad_x,    \
                     d_grad_vec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_cut, d_unit, flags, st)
  if (dtype == TMDNET_F32) TMD_BWD2(float);
  if (dtype == TMDNET_F64) TMD_BWD2(double);
#undef TMD_BWD2
  return kUnsupported;
}

extern "C" int tmdnet_et_message_bwd2_ex(
    int dtype, int n_nodes, int hidden, int heads, const int32_t* row_ptr, const int32_t* src,
    const int32_t* transpose, int max_pairs, const void* q, int ld_q, const void* k, int ld_k,
    const void* v, int ld_v, const void* vec_in, const void* pk, int ld_pk, const void* pv, int ld_pv,
    const void* cutoff, const void* unit, const void* grad_x, const void* grad_vec, const void* gg_q,
    int ld_ggq, const void* gg_k, int ld_ggk, const void* gg_v, int ld_ggv, const void* gg_vec,
    const void* gg_pk, int ld_ggpk, const void* gg_pv, int ld_ggpv, const void* gg_cut,
    const void* gg_unit, void* d_grad_x, void* d_grad_vec, void* d_q, int ld_dq, void* d_k, int ld_dk,
    void* d_v, int ld_dv, void* d_vec, void* d_pk, int ld_dpk, void* d_pv, int ld_dpv, void* d_cut,
    void* d_unit, void* edge_scratch, const int32_t* pk_rows, const void* gg_pkv_scale, int flags, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const et::Bwd2Ex ex{ld_ggq, ld_ggk, ld_ggv, ld_dq, ld_dk, ld_dv, ld_dpk, ld_dpv, transpose, edge_scratch, pk_rows,
                      gg_pkv_scale};
#define TMD_BWD2(T)                                                                              \
  return et::bwd2<T>(n_nodes, hidden, heads, row_ptr, src, max_pairs, q, ld_q, k, ld_k, v, ld_v, \
                     vec_in, pk, ld_pk, pv, ld_pv, cutoff, unit, grad_x, grad_vec, gg_q, gg_k,   \
                     gg_v, gg_vec, gg_pk, ld_ggpk, gg_pv, ld_ggpv, gg_cut, gg_unit, d_grad_x,    \
                     d_grad_vec, d_q, d_k, d_v, d_vec, d_pk, d_pv, d_cut, d_unit, flags, st, &ex)
  if (dtype == TMDNET_F32) TMD_BWD2(float);
  if (dtype == TMDNET_F64) TMD_BWD2(double);
#undef TMD_BWD2
  return kUnsupported;
}

template <typename T>
static int nb_fwd_t(int n, int H, const int32_t* row_ptr, const int32_t* src, int cap, const void* x,
                    int ldx, const void* w, int ldw, const void* C, void* out, int ldo, const void* xself,
                    void* oself, hipStream_t st) {
  et::NbArgs<T> A;
  int V;
  int rc = et::nb_setup<T>(A, n, H, row_ptr, src, cap, x, ldx, w, ldw, C, V);
  if (rc) return rc;
  if (!out) return kBadArgument;
  A.out = (T*)out;
  A.ldo = ldo ? ldo : H;
  if (A.ldo < H || !et::aligned<T>(out, A.ldo, V)) return kBadArgument;
  if ((xself == nullptr) != (oself == nullptr) || !et::aligned<T>(xself, H, V) ||
      !et::aligned<T>(oself, A.ldo, V))
    return kBadArgument;
  A.xself = (const T*)xself;
  A.oself = (T*)oself;
  return et::launch_v<T, et::KNbFwd>(V, n, A, st);
}

template <typename T>
static int nb_bwd_t(int n, int H, const int32_t* row_ptr, const int32_t* src, int cap, const void* x,
                    int ldx, const void* w, int ldw, const void* C, const void* gout, int ldg, void* gx,
                    void* gw, void* gC, hipStream_t st) {
  et::NbArgs<T> A;
  int V;
  int rc = et::nb_setup<T>(A, n, H, row_ptr, src, cap, x, ldx, w, ldw, C, V);
  if (rc) return rc;
  if (!gout) return kBadArgument;
  A.gout = (const T*)gout;
  A.ldg = ldg ? ldg : H;
  if (A.ldg < H || !et::aligned<T>(gout, A.ldg, V)) return kBadArgument;
  A.gx = (T*)gx; A.gw = (T*)gw; A.gC = (T*)gC;
  if (!gw || !gC) return kBadArgument;
  if (n > 0) {  // one 4-wave block per node (k_nb_bwd_dst)
    if (V == 1) hipLaunchKernelGGL((et::k_nb_bwd_dst<T, 1>), dim3(n), dim3(256), 0, st, A);
    else if (V == 2) hipLaunchKernelGGL((et::k_nb_bwd_dst<T, 2>), dim3(n), dim3(256), 0, st, A);
    else hipLaunchKernelGGL((et::k_nb_bwd_dst<T, 4>), dim3(n), dim3(256), 0, st, A);
    rc = hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
  }
  if (rc) return rc;
  return gx ? et::launch_v<T, et::KNbSrc>(V, n, A, st) : kOk;  // gx NULL: the source pass is skipped
}

extern "C" int tmdnet_nbr_embed_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                    const int32_t* src, int max_pairs, const void* x, int ld_x,
                                    const void* w, int ld_w, const void* cutoff, void* out, int ld_out,
                                    const void* x_self, void* out_self, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) return nb_fwd_t<float>(n_nodes, hidden, row_ptr, src, max_pairs, x, ld_x, w, ld_w, cutoff, out, ld_out, x_self, out_self, st);
  if (dtype == TMDNET_F64) return nb_fwd_t<double>(n_nodes, hidden, row_ptr, src, max_pairs, x, ld_x, w, ld_w, cutoff, out, ld_out, x_self, out_self, st);
  return kUnsupported;
}

extern "C" int tmdnet_nbr_embed_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                    const int32_t* src, int max_pairs, const void* x, int ld_x,
                                    const void* w, int ld_w, const void* cutoff, const void* grad_out,
                                    int ld_grad_out, void* gx, void* gw, void* gcut, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) return nb_bwd_t<float>(n_nodes, hidden, row_ptr, src, max_pairs, x, ld_x, w, ld_w, cutoff, grad_out, ld_grad_out, gx, gw, gcut, st);
  if (dtype == TMDNET_F64) return nb_bwd_t<double>(n_nodes, hidden, row_ptr, src, max_pairs, x, ld_x, w, ld_w, cutoff, grad_out, ld_grad_out, gx, gw, gcut, st);
  return kUnsupported;
}

template <typename T>
static int nb_bwd2_t(int n, int H, const int32_t* row_ptr, const int32_t* src, const int32_t* tr, int cap,
                     const void* x, int ldx, const void* w, int ldw, const void* C, const void* gout, int ldg,
                     const void* ggx, const void* ggw, const void* ggC, void* dgout, void* dx, void* dw, void* dC,
                     hipStream_t st) {
  et::NbArgs<T> A;
  int V;
  int rc = et::nb_setup<T>(A, n, H, row_ptr, src, cap, x, ldx, w, ldw, C, V);
  if (rc) return rc;
  if (!gout || !C || (dx && !tr)) return kBadArgument;
  A.gout = (const T*)gout;
  A.ldg = ldg ? ldg : H;
  if (A.ldg < H || !et::aligned<T>(gout, A.ldg, V) || !et::aligned<T>(ggx, H, V) || !et::aligned<T>(ggw, H, V))
    return kBadArgument;
  A.ggx = (const T*)ggx; A.ggw = (const T*)ggw; A.ggC = (const T*)ggC;
  A.dgout = (T*)dgout; A.dx = (T*)dx; A.dw = (T*)dw; A.dC = (T*)dC; A.tr = tr;
  if (dgout || dw || dC) {
    rc = et::launch_v<T, et::KNb2Dst>(V, n, A, st);
    if (rc) return rc;
  }
  if (dx) return et::launch_v<T, et::KNb2Src>(V, n, A, st);
  return kOk;
}

extern "C" int tmdnet_nbr_embed_bwd2(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                     const int32_t* src, const int32_t* transpose, int max_pairs,
                                     const void* x, int ld_x, const void* w, int ld_w, const void* cutoff,
                                     const void* grad_out, int ld_grad_out, const void* gg_x, const void* gg_w,
                                     const void* gg_cut, void* d_grad_out, void* d_x, void* d_w, void* d_cut,
                                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
#define TMD_NB2(T)                                                                                              \
  return nb_bwd2_t<T>(n_nodes, hidden, row_ptr, src, transpose, max_pairs, x, ld_x, w, ld_w, cutoff, grad_out, \
                      ld_grad_out, gg_x, gg_w, gg_cut, d_grad_out, d_x, d_w, d_cut, st)
  if (dtype == TMDNET_F32) TMD_NB2(float);
  if (dtype == TMDNET_F64) TMD_NB2(double);
#undef TMD_NB2
  return kUnsupported;
}

extern "C" const char* tmdnet_build_info(void) {
  return "torchmd-net_amd libtmdnet_hip (gfx950, wave64 CSR edge kernels)";
}

extern "C" int tmdnet_set_tuning(int key, int value) {
  if (key != TMDNET_TUNE_ET_BOTH_MAX_NODES && key != TMDNET_TUNE_ET_MERGED_MIN_NODES) return -1;
  const int prev = et::tune_get(key);
  et::g_tune[key] = value < 0 ? 0 : value;
  return prev;
}
