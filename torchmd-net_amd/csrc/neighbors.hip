// Neighbour-list build for gfx950 (CDNA4, wave64).
//
// Replaces the reference op `torchmdnet_neighbors::get_neighbor_pairs`
//   schema:      torchmdnet/neighbors/neighbors.cpp:3-5
//   CUDA impls:  neighbors_cuda_brute.cuh:21-101, neighbors_cuda_shared.cuh:13-106,
//                neighbors_cuda_cell.cuh:90-378, output contract common.cuh:64-116
//   CPU oracle:  neighbors_cpu.cpp:19-95
//
// Design (MI355X-first, not a translation):
//  * The reference appends pairs with one global atomicAdd per pair (common.cuh:108), so its
//    output order is nondeterministic.  Here the list is built in two passes -- a count pass and a
//    fill pass -- with one wave64 per destination atom, and wave ballots + mbcnt lane prefixes give
//    every lane its write slot.  The result is a DETERMINISTIC destination-grouped CSR:
//      row t = all edges e with neighbors[1][e] == t, in ascending candidate order,
//    plus the reference's (2, max_pairs) / (max_pairs, 3) / (max_pairs) / (1) view of it.
//  * Batched small molecules (the QM9/SPICE regime) restrict each destination's candidates to its
//    own molecule segment when `batch` is sorted (checked on device, no host sync); unsorted
//    batches fall back to scanning every atom.
//  * The cell strategy bins atoms (rect PBC, reference cell geometry), stable-radix-sorts them by
//    cell (deterministic within-cell order), then runs the same count/fill pair over the 27 cells.
//  * An optional transpose map T (T[e] = index of the reversed edge) lets the backward pass be a
//    segmented CSR reduction with no atomics:  dpos[n] = sum_{e in row n} g[T(e)] - g[e].
#include "common.h"
#include "tmdnet.h"
#include <hipcub/hipcub.hpp>

namespace tmd {
namespace nl {

template <typename T> struct V3 { T x, y, z; };

template <typename T> __device__ __forceinline__ V3<T> load3(const T* p, int i) {
  return {p[3 * i + 0], p[3 * i + 1], p[3 * i + 2]};
}

// Triclinic minimum image, reference common.cuh:183-194 (brute/shared): scale by round(),
// c then b then a.  `round` is half-away-from-zero (odd-symmetric), so the reversed edge's delta is
// the exact negation of the forward one.
template <typename T> struct Tric {
  T a0, b0, b1, c0, c1, c2;
  __device__ __forceinline__ V3<T> apply(V3<T> d) const {
    T s3 = round(d.z / c2);
    d.x -= s3 * c0; d.y -= s3 * c1; d.z -= s3 * c2;
    T s2 = round(d.y / b1);
    d.x -= s2 * b0; d.y -= s2 * b1;
    T s1 = round(d.x / a0);
    d.x -= s1 * a0;
    return d;
  }
};

// Rectangular minimum image used by the reference cell list (common.cuh:143-148).
template <typename T> __device__ __forceinline__ V3<T> rect_apply(V3<T> p, V3<T> L) {
  p.x = p.x - floor(p.x / L.x + T(0.5)) * L.x;
  p.y = p.y - floor(p.y / L.y + T(0.5)) * L.y;
  p.z = p.z - floor(p.z / L.z + T(0.5)) * L.z;
  return p;
}

template <typename T> struct Params {
  const T* pos;
  const int64_t* batch;
  int n;
  int periodic;
  int rect;  // 1 = cell-list rect PBC convention, 0 = triclinic round()
  Tric<T> box;
  V3<T> L;
  T cl2, cu2;
  int loop, transpose;
  const int* unsorted;  // brute/shared: k_segments' per-block descent flags (nonzero somewhere: unsorted)
  int n_unsorted;       // ... their count
};

// Directed edge s -> t (neighbors[0]=s, neighbors[1]=t): delta = pos[s] - pos[t] (minimum image).
template <typename T>
__device__ __forceinline__ V3<T> edge_delta(const Params<T>& P, V3<T> ps, V3<T> pt) {
  V3<T> d{ps.x - pt.x, ps.y - pt.y, ps.z - pt.z};
  if (P.periodic) d = P.rect ? rect_apply(d, P.L) : P.box.apply(d);
  return d;
}

// Is s a neighbour (source) of destination t?  Self pairs only when loop (kept regardless of the
// lower cutoff, as every reference strategy does); without include_transpose only s > t (the
// reference emits (max, min) pairs: neighbors_cpu.cpp:62, _cell.cuh:264-274).
template <typename T>
__device__ __forceinline__ bool accept(const Params<T>& P, int s, int t, int64_t bt, V3<T> pt,
                                       V3<T>& d, T& d2) {
  if (s == t) {
    d = {T(0), T(0), T(0)};
    d2 = T(0);
    return P.loop != 0;
  }
  if (!P.transpose && s < t) return false;
  if (P.batch[s] != bt) return false;
  d = edge_delta(P, load3(P.pos, s), pt);
  d2 = d.x * d.x + d.y * d.y + d.z * d.z;
  return d2 < P.cu2 && d2 >= P.cl2;
}

// ---------------------------------------------------------------- batch segments (no host sync)
// seg[2t], seg[2t+1] = candidate range of destination t, by binary search as if `batch` were sorted;
// in the same pass every thread checks its neighbour pair and each block stores whether it saw a descent
// in flag[block] (written unconditionally: no zero fill before the launch).  The pair kernels OR the block
// flags and fall back to all candidates [0, n) when any is set (the reference accepts unsorted batches),
// so the searched ranges are only used when they are valid.
__global__ __launch_bounds__(256) void k_segments(const int64_t* __restrict__ batch, int n, int* __restrict__ flag,
                                                  int* __restrict__ seg) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = t < n ? batch[t] : 0;
  const int desc = __syncthreads_or(t + 1 < n && b > batch[t + 1]);
  if (threadIdx.x == 0) flag[blockIdx.x] = desc;
  if (t >= n) return;
  int lo = 0, hi = t;  // first index with batch == b
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (batch[m] < b) lo = m + 1; else hi = m;
  }
  seg[2 * t] = lo;
  lo = t + 1;
  hi = n;  // first index with batch > b
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (batch[m] <= b) lo = m + 1; else hi = m;
  }
  seg[2 * t + 1] = lo;
}


// ---------------------------------------------------------------- all-pairs (brute / shared)
// One wave64 per destination; 64 candidates per iteration; ballot counts/compacts.
// Count pass with `ccounts`: also the number of canonical sources (s >= t) per row -- the pair
// numbering of the sorted rows (see k_transpose) needs nothing else.
template <typename T, bool FILL>
__global__ __launch_bounds__(256) void k_pairs(Params<T> P, const int* __restrict__ seg,
                                               int* __restrict__ counts, const int* __restrict__ row_ptr,
                                               int cap, int32_t* __restrict__ nb, T* __restrict__ dlt,
                                               T* __restrict__ dist, int* __restrict__ ccounts) {
  const int t = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (t >= P.n) return;
  const int lane = lane_id();
  int uf = 0;  // unsorted batch (a descent flagged by any k_segments block): every atom is a candidate
  for (int i = lane; i < P.n_unsorted; i += TMD_WAVE) uf |= P.unsorted[i];
  const bool all = __any(uf);
  const int lo = all ? 0 : seg[2 * t], hi = all ? P.n : seg[2 * t + 1];
  const V3<T> pt = load3(P.pos, t);
  const int64_t bt = P.batch[t];
  int off = FILL ? row_ptr[t] : 0;
  int coff = 0;
  for (int base = lo; base < hi; base += TMD_WAVE) {
    const int s = base + lane;
    V3<T> d;
    T d2;
    const bool ok = s < hi && accept(P, s, t, bt, pt, d, d2);
    const unsigned long long m = __ballot(ok);
    if (!FILL && ccounts) coff += __popcll(__ballot(ok && s >= t));
    if (FILL) {
      const int slot = off + lane_prefix(m);
      if (ok && slot < cap) {
        nb[slot] = s;
        nb[cap + slot] = t;
        dlt[3 * slot + 0] = d.x;
        dlt[3 * slot + 1] = d.y;
        dlt[3 * slot + 2] = d.z;
        dist[slot] = sqrt(d2);
      }
    }
    off += __popcll(m);
  }
  if (!FILL && lane == 0) {
    counts[t] = off;
    if (ccounts) ccounts[t] = coff;
  }
}

// ---------------------------------------------------------------- exclusive scan (one block)
// counts[0..n) -> row_ptr[0..n], num_pairs[0] = total.  n is at most a few million atoms; one
// 1024-thread block with per-thread serial chunks is a few microseconds at these sizes.
// (`ccounts` non-NULL: the canonical counts are scanned the same way into pair_ptr[0..n].)
__device__ __forceinline__ void block_scan(long long* part, const int* __restrict__ counts, int n,
                                           int* __restrict__ out, int* __restrict__ total) {
  const int tid = threadIdx.x;
  const int chunk = (n + 1023) / 1024;
  const int b = tid * chunk;
  const int e = min(n, b + chunk);
  long long s = 0;
  for (int i = b; i < e; ++i) s += counts[i];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    long long v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  long long run = part[tid] - s;
  for (int i = b; i < e; ++i) {
    out[i] = (int)run;
    run += counts[i];
  }
  if (tid == 1023) {
    out[n] = (int)part[1023];
    if (total) total[0] = (int)part[1023];
  }
}

__global__ __launch_bounds__(1024) void k_scan(const int* __restrict__ counts, int n, int* __restrict__ row_ptr,
                                               int* __restrict__ num_pairs, const int* __restrict__ ccounts,
                                               int* __restrict__ pair_ptr) {
  __shared__ long long part[1024];
  block_scan(part, counts, n, row_ptr, num_pairs);
  if (ccounts) {
    __syncthreads();
    block_scan(part, ccounts, n, pair_ptr, nullptr);
  }
}

// ---------------------------------------------------------------- transpose map + padding
// One pass over the capacity: slots past the pairs found get the reference padding (-1 / 0,
// common.cuh:70-76) when `pad` (replaces three capacity-sized memsets), found slots their transpose.
//
// Pair numbering (Pairs::prow non-NULL, sorted rows only; the same numbers as tmdnet_pair_index):
// the canonical edge of a pair is the direction with src >= dst, numbered row by row in CSR order;
// in a row sorted by source the canonical edges are its suffix, so edge e's number is closed-form:
// row r = min(src, dst), k = e if canonical else T(e),  pid = pair_ptr[r] + k - (row_end(r) - cc[r]).
// Slots past the pair count point at edge 0; a pid outside the slots (capacity-truncated list) reads
// row 0 and is reported by the capacity check.
struct Pairs {
  const int* pair_ptr;  // exclusive scan of the canonical counts, [n + 1]
  const int* cc;        // canonical count per row
  int32_t* prow;        // [cap]   pair row of every edge
  int32_t* pedge;       // [slots] canonical edge of every pair
  int slots, n;
};

template <typename T, bool SORTED_ROWS>
__global__ void k_transpose(int32_t* __restrict__ nb, const int* __restrict__ row_ptr, int cap,
                            const int* __restrict__ num_pairs, int32_t* __restrict__ tr, int pad,
                            T* __restrict__ dlt, T* __restrict__ dist, Pairs PR) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (SORTED_ROWS && PR.prow && e < PR.slots) {
    // canonical edge of pair e, as a gather (every slot written once, always an edge index in [0, cap)):
    // its row r is the last with pair_ptr[r] <= e, its position the (e - pair_ptr[r])-th of the row's
    // canonical suffix.  A pair whose canonical edge fell past a capacity-truncated list gets edge 0 (the
    // build reports the overflow; the scatter form left such slots unwritten -- garbage indices)
    int edge = 0;
    if (e < PR.pair_ptr[PR.n]) {
      int lo = 0, hi = PR.n - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) >> 1;
        if (PR.pair_ptr[m] <= e) lo = m; else hi = m - 1;
      }
      const int k = e - PR.pair_ptr[lo] + min(row_ptr[lo + 1], cap) - PR.cc[lo];
      edge = (k >= 0 && k < cap) ? k : 0;
    }
    PR.pedge[e] = edge;
  }
  if (e >= cap) return;
  if (e >= num_pairs[0]) {  // unwritten slot
    if (pad) {
      nb[e] = -1;
      nb[cap + e] = -1;
      dlt[3 * e] = T(0);
      dlt[3 * e + 1] = T(0);
      dlt[3 * e + 2] = T(0);
      dist[e] = T(0);
    }
    if (tr) tr[e] = -1;
    if (PR.prow) PR.prow[e] = 0;
    return;
  }
  if (!tr) return;
  const int s = nb[e];
  const int t = nb[cap + e];
  int found = -1;
  if (s == t) {
    found = e;
  } else if (s >= 0) {
    int lo = row_ptr[s], hi = min(row_ptr[s + 1], cap);
    if (SORTED_ROWS) {
      while (lo < hi) {
        int m = (lo + hi) >> 1;
        if (nb[m] < t) lo = m + 1; else hi = m;
      }
      if (lo < min(row_ptr[s + 1], cap) && nb[lo] == t) found = lo;
    } else {
      for (int k = lo; k < hi; ++k)
        if (nb[k] == t) { found = k; break; }
    }
  }
  tr[e] = found;
  if (SORTED_ROWS && PR.prow) {
    int pid = 0;
    const bool canon = s >= t;
    const int r = canon ? t : s, k = canon ? e : found;
    if (s >= 0 && k >= 0) {
      pid = PR.pair_ptr[r] + k - (min(row_ptr[r + 1], cap) - PR.cc[r]);
      if (pid < 0 || pid >= PR.slots) pid = 0;
    }
    PR.prow[e] = pid;
  }
}

// ---------------------------------------------------------------- cell list
template <typename T> struct CellGeom {
  V3<T> L;
  T cut;
  int nx, ny, nz;
};

// reference getCell (neighbors_cuda_cell.cuh:38-55): rect wrap, shift by L/2, divide by cutoff,
// fold an index equal to the cell count back to 0.
template <typename T>
__device__ __forceinline__ void cell_of(const CellGeom<T>& G, V3<T> p, int& cx, int& cy, int& cz) {
  p = rect_apply(p, G.L);
  cx = (int)floor((p.x + T(0.5) * G.L.x) / G.cut);
  cy = (int)floor((p.y + T(0.5) * G.L.y) / G.cut);
  cz = (int)floor((p.z + T(0.5) * G.L.z) / G.cut);
  if (cx == G.nx) cx = 0;
  if (cy == G.ny) cy = 0;
  if (cz == G.nz) cz = 0;
}

template <typename T>
__global__ void k_cell_assign(const T* __restrict__ pos, int n, CellGeom<T> G, int* __restrict__ keys,
                              int* __restrict__ vals) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int cx, cy, cz;
  cell_of(G, load3(pos, i), cx, cy, cz);
  keys[i] = cx + G.nx * (cy + G.ny * cz);
  vals[i] = i;
}

__global__ void k_cell_bounds(const int* __restrict__ skeys, int n, int* __restrict__ cstart,
                              int* __restrict__ cend) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = skeys[i];
  if (i == 0 || skeys[i - 1] != c) cstart[c] = i;
  if (i == n - 1 || skeys[i + 1] != c) cend[c] = i + 1;
}

// One thread per atom, visited in cell-sorted order (neighbouring threads share cells).  Candidate
// order inside a row: the 27 cell offsets in the reference order (_cell.cuh:187-195), then the
// stable-sorted (ascending atom index) members of each cell -> deterministic.
template <typename T, bool FILL>
__global__ __launch_bounds__(256) void k_cell_pairs(Params<T> P, CellGeom<T> G,
                                                    const int* __restrict__ skeys,
                                                    const int* __restrict__ svals,
                                                    const int* __restrict__ cstart,
                                                    const int* __restrict__ cend,
                                                    int* __restrict__ counts,
                                                    const int* __restrict__ row_ptr, int cap,
                                                    int32_t* __restrict__ nb, T* __restrict__ dlt,
                                                    T* __restrict__ dist) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.n) return;
  const int t = svals[p];
  const V3<T> pt = load3(P.pos, t);
  const int64_t bt = P.batch[t];
  int cx, cy, cz;
  cell_of(G, pt, cx, cy, cz);
  int off = FILL ? row_ptr[t] : 0;
  for (int k = 0; k < 27; ++k) {
    int jx = cx + k % 3 - 1, jy = cy + (k / 3) % 3 - 1, jz = cz + k / 9 - 1;
    if (jx < 0) jx += G.nx; else if (jx >= G.nx) jx -= G.nx;
    if (jy < 0) jy += G.ny; else if (jy >= G.ny) jy -= G.ny;
    if (jz < 0) jz += G.nz; else if (jz >= G.nz) jz -= G.nz;
    const int c = jx + G.nx * (jy + G.ny * jz);
    const int b = cstart[c];
    if (b < 0) continue;
    const int e = cend[c];
    for (int q = b; q < e; ++q) {
      const int s = svals[q];
      V3<T> d;
      T d2;
      if (!accept(P, s, t, bt, pt, d, d2)) continue;
      if (FILL) {
        if (off < cap) {
          nb[off] = s;
          nb[cap + off] = t;
          dlt[3 * off + 0] = d.x;
          dlt[3 * off + 1] = d.y;
          dlt[3 * off + 2] = d.z;
          dist[off] = sqrt(d2);
        }
      }
      ++off;
    }
  }
  if (!FILL) counts[t] = off;
}

// ---------------------------------------------------------------- backward (segmented, no atomics)
// Reference NeighborAutograd::backward (neighbors_cuda.cu:43-71):
//   g[e] = (r[e]==0) ? 0 : gdelta[e] + delta[e]/r[e] * gr[e];  dpos[src] += g, dpos[dst] -= g.
// With a symmetric list and T:  dpos[n] = sum_{e in row n} g[T(e)] - g[e].
template <typename T>
__device__ __forceinline__ V3<T> edge_grad(int e, const T* gd, const T* gr, const T* gr2, const T* dl, const T* r) {
  const T re = r[e];
  if (re == T(0)) return {T(0), T(0), T(0)};
  T gsum = gr ? gr[e] : T(0);
  if (gr2) gsum += gr2[e];  // the distances' second consumer (the ET stack's dr-mode g_r)
  const T gre = gsum / re;
  V3<T> g{T(0), T(0), T(0)};
  if (gd) g = {gd[3 * e + 0], gd[3 * e + 1], gd[3 * e + 2]};
  g.x += dl[3 * e + 0] * gre;
  g.y += dl[3 * e + 1] * gre;
  g.z += dl[3 * e + 2] * gre;
  return g;
}

// 16 lanes per atom stride over its CSR row; partial sums meet in a 16-lane xor-shuffle reduction
// (fixed order: deterministic).  One thread per atom left ~40 us on a 600-atom batch (serial rows).
constexpr int kNlLanes = 16;

template <typename T>
__device__ __forceinline__ T group_sum16(T v) {
#pragma unroll
  for (int off = kNlLanes / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kNlLanes);
  return v;
}

template <typename T>
__global__ void k_nl_backward(int n, const int* __restrict__ row_ptr, const int32_t* __restrict__ tr,
                              int cap, const T* __restrict__ gd, const T* __restrict__ gr,
                              const T* __restrict__ gr2, const T* __restrict__ dl, const T* __restrict__ r,
                              T* __restrict__ gpos) {
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gt / kNlLanes, lane = gt % kNlLanes;
  V3<T> acc{T(0), T(0), T(0)};
  if (t < n) {
    const int b = min(row_ptr[t], cap), e = min(row_ptr[t + 1], cap);
    for (int k = b + lane; k < e; k += kNlLanes) {
      const V3<T> gm = edge_grad(k, gd, gr, gr2, dl, r);
      acc.x -= gm.x; acc.y -= gm.y; acc.z -= gm.z;
      const int k2 = tr[k];
      if (k2 >= 0) {
        const V3<T> gp = edge_grad(k2, gd, gr, gr2, dl, r);
        acc.x += gp.x; acc.y += gp.y; acc.z += gp.z;
      }
    }
  }
  acc.x = group_sum16(acc.x);
  acc.y = group_sum16(acc.y);
  acc.z = group_sum16(acc.z);
  if (t < n && lane == 0) {
    gpos[3 * t + 0] = acc.x;
    gpos[3 * t + 1] = acc.y;
    gpos[3 * t + 2] = acc.z;
  }
}

// Second order of k_nl_backward (the double backward of NeighborAutograd's index_add pair,
// reference neighbors_cuda.cu:25-89, which the reference differentiates through autograd).  With
// gg = cotangent of gpos and, per edge e = (s -> t), w = gg[s] - gg[t], u = dl/r:
//   d_gd[e] = w,   d_gr[e] = u.w,   d_dl[e] = gr/r (w - u (u.w))      (all 0 when r == 0)
//   d_pos[n] = sum_{e in row n} d_dl[T(e)] - d_dl[e]        (the scatter of k_nl_backward)
// T(e) = (t -> s) sees w(T(e)) = -w(e), so one gather of gg per edge serves both directions.
template <typename T>
__device__ __forceinline__ V3<T> edge_grad2(int e, V3<T> w, const T* gr, const T* dl, const T* r,
                                            T& uw) {
  const T re = r[e];
  if (re == T(0)) {
    uw = T(0);
    return {T(0), T(0), T(0)};
  }
  const T inv = T(1) / re;
  const V3<T> u{dl[3 * e + 0] * inv, dl[3 * e + 1] * inv, dl[3 * e + 2] * inv};
  uw = u.x * w.x + u.y * w.y + u.z * w.z;
  const T c = gr ? gr[e] * inv : T(0);
  return {c * (w.x - u.x * uw), c * (w.y - u.y * uw), c * (w.z - u.z * uw)};
}

template <typename T>
__global__ void k_nl_backward2(int n, const int* __restrict__ row_ptr, const int32_t* __restrict__ src,
                               const int32_t* __restrict__ tr, int cap, const T* __restrict__ gr,
                               const T* __restrict__ dl, const T* __restrict__ r,
                               const T* __restrict__ gg, T* __restrict__ dpos, T* __restrict__ dgd,
                               T* __restrict__ dgr) {
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gt / kNlLanes, lane = gt % kNlLanes;
  V3<T> acc{T(0), T(0), T(0)};
  if (t < n) {
    const int b = min(row_ptr[t], cap), e = min(row_ptr[t + 1], cap);
    const V3<T> gt3{gg[3 * t + 0], gg[3 * t + 1], gg[3 * t + 2]};
    for (int k = b + lane; k < e; k += kNlLanes) {
      const int s = src[k];
      TMD_DCHECK(s >= 0 && s < n);
      const V3<T> w{gg[3 * s + 0] - gt3.x, gg[3 * s + 1] - gt3.y, gg[3 * s + 2] - gt3.z};
      T uw;
      const V3<T> dm = edge_grad2(k, w, gr, dl, r, uw);
      acc.x -= dm.x; acc.y -= dm.y; acc.z -= dm.z;
      if (dgd) {
        const bool live = r[k] != T(0);
        dgd[3 * k + 0] = live ? w.x : T(0);
        dgd[3 * k + 1] = live ? w.y : T(0);
        dgd[3 * k + 2] = live ? w.z : T(0);
      }
      if (dgr) dgr[k] = uw;
      const int k2 = tr[k];
      TMD_DCHECK(k2 >= -1 && k2 < cap);
      if (k2 >= 0) {
        T uw2;
        const V3<T> dp = edge_grad2(k2, V3<T>{-w.x, -w.y, -w.z}, gr, dl, r, uw2);
        acc.x += dp.x; acc.y += dp.y; acc.z += dp.z;
      }
    }
  }
  acc.x = group_sum16(acc.x);
  acc.y = group_sum16(acc.y);
  acc.z = group_sum16(acc.z);
  if (t < n && lane == 0) {
    dpos[3 * t + 0] = acc.x;
    dpos[3 * t + 1] = acc.y;
    dpos[3 * t + 2] = acc.z;
  }
}

// ---------------------------------------------------------------- host side
#define TMD_CHECK(x)                               \
  do {                                             \
    if ((x) != hipSuccess) return kLaunchFailed;   \
  } while (0)

static inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

struct CellDims {
  int nx, ny, nz;
};

static int cell_dims(const double* box, double cut, CellDims& cd) {
  auto f = [&](double l) { int c = (int)(l / cut); return c < 3 ? 3 : c; };
  cd.nx = f(box[0]);
  cd.ny = f(box[4]);
  cd.nz = f(box[8]);
  if (cd.nx > 1024 || cd.ny > 1024 || cd.nz > 1024) return kUnsupported;
  return kOk;
}

static size_t cub_sort_bytes(int n) {
  size_t bytes = 0;
  (void)(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int*)nullptr, (int*)nullptr,
                                     (const int*)nullptr, (int*)nullptr, n, 0, 31, (hipStream_t)0));
  return bytes;
}

struct Layout {
  size_t flag, seg, counts, rowp, cc, pairp, keys, vals, skeys, svals, cstart, cend, cub, total;
  size_t cub_bytes;
  int ncells;
};

static Layout layout(int n, int strategy, const double* box, double cut) {
  Layout L{};
  size_t o = 0;
  L.flag = o; o += align16(sizeof(int) * (size_t)(n > 256 ? (n + 255) / 256 : 1));  // k_segments block flags
  L.seg = o; o += align16(sizeof(int) * 2 * (size_t)n);
  L.counts = o; o += align16(sizeof(int) * ((size_t)n + 1));
  L.rowp = o; o += align16(sizeof(int) * ((size_t)n + 1));
  L.cc = o; o += align16(sizeof(int) * ((size_t)n + 1));
  L.pairp = o; o += align16(sizeof(int) * ((size_t)n + 1));
  if (strategy == TMDNET_NL_CELL) {
    CellDims cd{3, 3, 3};
    cell_dims(box, cut, cd);
    L.ncells = cd.nx * cd.ny * cd.nz;
    L.keys = o; o += align16(sizeof(int) * (size_t)n);
    L.vals = o; o += align16(sizeof(int) * (size_t)n);
    L.skeys = o; o += align16(sizeof(int) * (size_t)n);
    L.svals = o; o += align16(sizeof(int) * (size_t)n);
    L.cstart = o; o += align16(sizeof(int) * (size_t)L.ncells);
    L.cend = o; o += align16(sizeof(int) * (size_t)L.ncells);
    L.cub_bytes = cub_sort_bytes(n);
    L.cub = o; o += align16(L.cub_bytes);
  }
  L.total = o;
  return L;
}

template <typename T>
static int build(int strategy, const T* pos, const int64_t* batch, int n, const double* box,
                 int periodic, double cl, double cu, int cap, int loop, int transpose, int32_t* nb,
                 T* dlt, T* dist, int32_t* num_pairs, int32_t* row_ptr_out, int32_t* tr, int pad,
                 char* ws, size_t ws_bytes, int32_t* prow, int32_t* pedge, int slots, hipStream_t st) {
  if (n <= 0 || cap <= 0 || !(cu > 0)) return kBadArgument;
  if (prow && (!pedge || slots <= 0 || !tr || !transpose || strategy == TMDNET_NL_CELL)) return kBadArgument;
  const Layout Lo = layout(n, strategy, box, cu);
  if (ws_bytes < Lo.total) return kWorkspaceTooSmall;
  int* flag = (int*)(ws + Lo.flag);
  int* seg = (int*)(ws + Lo.seg);
  int* counts = (int*)(ws + Lo.counts);
  int* row_ptr = row_ptr_out ? row_ptr_out : (int*)(ws + Lo.rowp);
  int* cc = prow ? (int*)(ws + Lo.cc) : nullptr;
  int* pairp = prow ? (int*)(ws + Lo.pairp) : nullptr;
  Pairs PR{pairp, cc, prow, pedge, slots, n};

  Params<T> P{};
  P.pos = pos;
  P.batch = batch;
  P.n = n;
  P.periodic = periodic;
  P.rect = strategy == TMDNET_NL_CELL;
  if (periodic || strategy == TMDNET_NL_CELL) {
    P.box = {(T)box[0], (T)box[3], (T)box[4], (T)box[6], (T)box[7], (T)box[8]};
    P.L = {(T)box[0], (T)box[4], (T)box[8]};
  }
  const T clT = (T)cl, cuT = (T)cu;
  P.cl2 = clT * clT;
  P.cu2 = cuT * cuT;
  P.loop = loop;
  P.transpose = transpose;

  const int tb = 256;
  if (strategy == TMDNET_NL_CELL) {
    CellDims cd;
    if (cell_dims(box, cu, cd) != kOk) return kUnsupported;
    CellGeom<T> G{{(T)box[0], (T)box[4], (T)box[8]}, cuT, cd.nx, cd.ny, cd.nz};
    int* keys = (int*)(ws + Lo.keys);
    int* vals = (int*)(ws + Lo.vals);
    int* skeys = (int*)(ws + Lo.skeys);
    int* svals = (int*)(ws + Lo.svals);
    int* cstart = (int*)(ws + Lo.cstart);
    int* cend = (int*)(ws + Lo.cend);
    hipLaunchKernelGGL(k_cell_assign<T>, dim3((n + tb - 1) / tb), dim3(tb), 0, st, pos, n, G, keys, vals);
    size_t cb = Lo.cub_bytes;
    int endbit = 1;
    while ((1 << endbit) < Lo.ncells && endbit < 31) ++endbit;
    if (hipcub::DeviceRadixSort::SortPairs((void*)(ws + Lo.cub), cb, keys, skeys, vals, svals, n, 0,
                                           endbit, st) != hipSuccess)
      return kLaunchFailed;
    TMD_CHECK(hipMemsetAsync(cstart, 0xFF, sizeof(int) * (size_t)Lo.ncells, st));
    hipLaunchKernelGGL(k_cell_bounds, dim3((n + tb - 1) / tb), dim3(tb), 0, st, skeys, n, cstart, cend);
    hipLaunchKernelGGL((k_cell_pairs<T, false>), dim3((n + tb - 1) / tb), dim3(tb), 0, st, P, G, skeys,
                       svals, cstart, cend, counts, row_ptr, cap, nb, dlt, dist);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, counts, n, row_ptr, num_pairs, nullptr, nullptr);
    hipLaunchKernelGGL((k_cell_pairs<T, true>), dim3((n + tb - 1) / tb), dim3(tb), 0, st, P, G, skeys,
                       svals, cstart, cend, counts, row_ptr, cap, nb, dlt, dist);
    if (tr || pad)
      hipLaunchKernelGGL((k_transpose<T, false>), dim3((cap + tb - 1) / tb), dim3(tb), 0, st, nb, row_ptr, cap,
                         num_pairs, tr, pad, dlt, dist, PR);
  } else {
    // (a single-workgroup fusion of the segment search and the count pass measured slower: 25 us
    // against 14 us at 678 atoms -- its binary searches become dependent-load chains on one CU)
    P.unsorted = flag;
    P.n_unsorted = (n + tb - 1) / tb;
    hipLaunchKernelGGL(k_segments, dim3((n + tb - 1) / tb), dim3(tb), 0, st, batch, n, flag, seg);
    const int wpb = tb / TMD_WAVE;
    const dim3 g((n + wpb - 1) / wpb);
    hipLaunchKernelGGL((k_pairs<T, false>), g, dim3(tb), 0, st, P, seg, counts, row_ptr, cap, nb, dlt, dist, cc);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, counts, n, row_ptr, num_pairs, cc, pairp);
    hipLaunchKernelGGL((k_pairs<T, true>), g, dim3(tb), 0, st, P, seg, counts, row_ptr, cap, nb, dlt, dist,
                       nullptr);
    if (tr || pad)
      hipLaunchKernelGGL((k_transpose<T, true>), dim3((max(cap, prow ? slots : 0) + tb - 1) / tb), dim3(tb), 0, st,
                         nb, row_ptr, cap, num_pairs, tr, pad, dlt, dist, PR);
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

}  // namespace nl
}  // namespace tmd

using namespace tmd;

extern "C" size_t tmdnet_nl_workspace_bytes(int n_atoms, int strategy, const double* box9,
                                            double cutoff_upper) {
  double unit[9] = {0};
  return nl::layout(n_atoms, strategy, box9 ? box9 : unit, cutoff_upper).total;
}

static int nl_build_any(int dtype, int strategy, const void* pos, const int64_t* batch, int n_atoms,
                        const double* box9, int use_periodic, double cutoff_lower, double cutoff_upper,
                        int max_pairs, int loop, int include_transpose, int32_t* neighbors, void* deltas,
                        void* distances, int32_t* num_pairs, int32_t* row_ptr, int32_t* transpose_map,
                        int pad_output, void* workspace, size_t workspace_bytes, int32_t* pair_row,
                        int32_t* pair_edge, int n_pair_slots, void* stream) {
  if (strategy != TMDNET_NL_BRUTE && strategy != TMDNET_NL_SHARED && strategy != TMDNET_NL_CELL)
    return kBadArgument;
  double unit[9] = {0};
  const double* box = box9 ? box9 : unit;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return nl::build<float>(strategy, (const float*)pos, batch, n_atoms, box, use_periodic, cutoff_lower,
                            cutoff_upper, max_pairs, loop, include_transpose, neighbors, (float*)deltas,
                            (float*)distances, num_pairs, row_ptr, transpose_map, pad_output, (char*)workspace,
                            workspace_bytes, pair_row, pair_edge, n_pair_slots, st);
  if (dtype == TMDNET_F64)
    return nl::build<double>(strategy, (const double*)pos, batch, n_atoms, box, use_periodic, cutoff_lower,
                             cutoff_upper, max_pairs, loop, include_transpose, neighbors, (double*)deltas,
                             (double*)distances, num_pairs, row_ptr, transpose_map, pad_output,
                             (char*)workspace, workspace_bytes, pair_row, pair_edge, n_pair_slots, st);
  return kUnsupported;
}

extern "C" int tmdnet_nl_build(int dtype, int strategy, const void* pos, const int64_t* batch,
                               int n_atoms, const double* box9, int use_periodic,
                               double cutoff_lower, double cutoff_upper, int max_pairs, int loop,
                               int include_transpose, int32_t* neighbors, void* deltas,
                               void* distances, int32_t* num_pairs, int32_t* row_ptr,
                               int32_t* transpose_map, int pad_output, void* workspace,
                               size_t workspace_bytes, void* stream) {
  return nl_build_any(dtype, strategy, pos, batch, n_atoms, box9, use_periodic, cutoff_lower, cutoff_upper,
                      max_pairs, loop, include_transpose, neighbors, deltas, distances, num_pairs, row_ptr,
                      transpose_map, pad_output, workspace, workspace_bytes, nullptr, nullptr, 0, stream);
}

extern "C" int tmdnet_nl_build_paired(int dtype, int strategy, const void* pos, const int64_t* batch,
                                      int n_atoms, const double* box9, int use_periodic, double cutoff_lower,
                                      double cutoff_upper, int max_pairs, int loop, int include_transpose,
                                      int32_t* neighbors, void* deltas, void* distances, int32_t* num_pairs,
                                      int32_t* row_ptr, int32_t* transpose_map, int pad_output,
                                      void* workspace, size_t workspace_bytes, int32_t* pair_row,
                                      int32_t* pair_edge, int n_pair_slots, void* stream) {
  if (!pair_row || !pair_edge || n_pair_slots <= 0) return kBadArgument;
  return nl_build_any(dtype, strategy, pos, batch, n_atoms, box9, use_periodic, cutoff_lower, cutoff_upper,
                      max_pairs, loop, include_transpose, neighbors, deltas, distances, num_pairs, row_ptr,
                      transpose_map, pad_output, workspace, workspace_bytes, pair_row, pair_edge, n_pair_slots,
                      stream);
}

extern "C" int tmdnet_nl_backward_multi(int dtype, int n_atoms, const int32_t* row_ptr,
                                        const int32_t* transpose_map, int max_pairs, const void* grad_deltas,
                                        const void* grad_distances, const void* grad_distances2, const void* deltas,
                                        const void* distances, void* grad_pos, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int tb = 256;
  dim3 g((unsigned)(((size_t)n_atoms * nl::kNlLanes + tb - 1) / tb));
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(nl::k_nl_backward<float>, g, dim3(tb), 0, st, n_atoms, row_ptr, transpose_map,
                       max_pairs, (const float*)grad_deltas, (const float*)grad_distances,
                       (const float*)grad_distances2, (const float*)deltas, (const float*)distances,
                       (float*)grad_pos);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(nl::k_nl_backward<double>, g, dim3(tb), 0, st, n_atoms, row_ptr, transpose_map,
                       max_pairs, (const double*)grad_deltas, (const double*)grad_distances,
                       (const double*)grad_distances2, (const double*)deltas, (const double*)distances,
                       (double*)grad_pos);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_nl_backward(int dtype, int n_atoms, const int32_t* row_ptr,
                                  const int32_t* transpose_map, int max_pairs,
                                  const void* grad_deltas, const void* grad_distances,
                                  const void* deltas, const void* distances, void* grad_pos,
                                  void* stream) {
  return tmdnet_nl_backward_multi(dtype, n_atoms, row_ptr, transpose_map, max_pairs, grad_deltas, grad_distances,
                                  nullptr, deltas, distances, grad_pos, stream);
}

extern "C" int tmdnet_nl_backward2(int dtype, int n_atoms, const int32_t* row_ptr, const int32_t* src,
                                   const int32_t* transpose_map, int max_pairs,
                                   const void* grad_distances, const void* deltas,
                                   const void* distances, const void* gg_pos, void* d_pos,
                                   void* d_grad_deltas, void* d_grad_distances, void* stream) {
  if (n_atoms <= 0 || max_pairs < 0 || !row_ptr || !src || !transpose_map || !gg_pos || !d_pos)
    return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  const size_t es = dtype == TMDNET_F64 ? 8 : 4;
  // padding slots belong to no CSR row: their gradients are zero
  if (d_grad_deltas) TMD_CHECK(hipMemsetAsync(d_grad_deltas, 0, es * 3 * (size_t)max_pairs, st));
  if (d_grad_distances) TMD_CHECK(hipMemsetAsync(d_grad_distances, 0, es * (size_t)max_pairs, st));
  const int tb = 256;
  dim3 g((unsigned)(((size_t)n_atoms * nl::kNlLanes + tb - 1) / tb));
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(nl::k_nl_backward2<float>, g, dim3(tb), 0, st, n_atoms, row_ptr, src, transpose_map,
                       max_pairs, (const float*)grad_distances, (const float*)deltas,
                       (const float*)distances, (const float*)gg_pos, (float*)d_pos,
                       (float*)d_grad_deltas, (float*)d_grad_distances);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(nl::k_nl_backward2<double>, g, dim3(tb), 0, st, n_atoms, row_ptr, src, transpose_map,
                       max_pairs, (const double*)grad_distances, (const double*)deltas,
                       (const double*)distances, (const double*)gg_pos, (double*)d_pos,
                       (double*)d_grad_deltas, (double*)d_grad_distances);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// ---------------------------------------------------------------- backward over a plain edge list
// The raw op's backward (reference NeighborAutograd::backward, neighbors_cuda.cu:43-71) for any list
// the op returns -- half lists (include_transpose=0) and capacity-truncated ones included, where the
// CSR pass above does not apply: one lane per edge slot, g = gdelta + delta/r*gr (0 for r == 0 and
// padding), scattered to both ends with atomics (the reference's index_add_ pair).
namespace tmd {
namespace nl {
template <typename T>
__global__ void k_nl_backward_edges(int n, const int32_t* __restrict__ nb, int cap, const T* __restrict__ gd,
                                    const T* __restrict__ gr, const T* __restrict__ dl,
                                    const T* __restrict__ r, T* __restrict__ gpos) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cap) return;
  const int s = nb[e], t = nb[cap + e];
  if (s < 0 || t < 0 || s >= n || t >= n) return;
  const V3<T> g = edge_grad(e, gd, gr, (const T*)nullptr, dl, r);
  if (g.x == T(0) && g.y == T(0) && g.z == T(0)) return;
  atomicAdd(gpos + 3 * s + 0, g.x);
  atomicAdd(gpos + 3 * s + 1, g.y);
  atomicAdd(gpos + 3 * s + 2, g.z);
  atomicAdd(gpos + 3 * t + 0, -g.x);
  atomicAdd(gpos + 3 * t + 1, -g.y);
  atomicAdd(gpos + 3 * t + 2, -g.z);
}
}  // namespace nl
}  // namespace tmd

extern "C" int tmdnet_nl_backward_edges(int dtype, int n_atoms, const int32_t* neighbors, int max_pairs,
                                        const void* grad_deltas, const void* grad_distances,
                                        const void* deltas, const void* distances, void* grad_pos,
                                        void* stream) {
  if (n_atoms <= 0 || max_pairs < 0 || !neighbors || !grad_pos) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  const size_t es = dtype == TMDNET_F64 ? 8 : 4;
  TMD_CHECK(hipMemsetAsync(grad_pos, 0, es * 3 * (size_t)n_atoms, st));
  if (max_pairs == 0) return kOk;
  const int tb = 256;
  dim3 g((unsigned)((max_pairs + tb - 1) / tb));
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(nl::k_nl_backward_edges<float>, g, dim3(tb), 0, st, n_atoms, neighbors, max_pairs,
                       (const float*)grad_deltas, (const float*)grad_distances, (const float*)deltas,
                       (const float*)distances, (float*)grad_pos);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(nl::k_nl_backward_edges<double>, g, dim3(tb), 0, st, n_atoms, neighbors, max_pairs,
                       (const double*)grad_deltas, (const double*)grad_distances, (const double*)deltas,
                       (const double*)distances, (double*)grad_pos);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
