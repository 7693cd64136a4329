// Pair numbering of a symmetric destination-grouped CSR edge list (tmdnet_pair_index).
//
// The ET dk/dv projections (reference torchmd_et.py:282-291) and the RBF features they read are
// functions of |r| only, so an edge and its reverse have bit-identical projections.  Numbering the
// pairs lets the projection GEMM run over (E + N) / 2 rows instead of E; the edge kernels read row
// pair_row[e].  Canonical edge of a pair: the direction with src >= dst (self loops are their own
// pair), numbered row by row in CSR order -- deterministic, no atomics.
//   pass 1  (wave per row)   canonical count per row (ballot popcount)
//   pass 2  (one workgroup)  exclusive scan over rows
//   pass 3  (wave per row)   canonical edges: pair_row[e] = base + ballot rank, pair_edge[p] = e;
//                            the other direction: pair_row[e] = -1 (resolved in pass 4)
//   pass 4  (thread per slot) pair_row[e] = pair_row[T(e)] for the other direction; inert slots 0
// Rows sorted by source (the brute / shared neighbour lists): the canonical edges of a row are its
// suffix, so three thread-parallel passes suffice -- per-row suffix length (binary search), the
// scan, and per-edge numbers in closed form (an edge's reverse T(e) sits at a known offset in its
// own row).  Unsorted rows (cell lists) take the four wave-per-row passes above.
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace pairs {

struct P {
  int n, cap;
  const int32_t* row_ptr;
  const int32_t* src;
  const int32_t* dst;
  const int32_t* tr;
  const int32_t* npairs;
  int32_t* prow;
  int32_t* pedge;
  int slots;
  int* cnt;  // [n + 1]: canonical count per row, then (in place) its exclusive scan; cnt[n] = total
};

__device__ __forceinline__ int valid_edges(const P& p) {
  const int np = p.npairs ? p.npairs[0] : p.row_ptr[p.n];
  return min(np, p.cap);
}

__device__ __forceinline__ void row_count(const P& p, int t) {
  const int lane = lane_id();
  const int b = min(p.row_ptr[t], p.cap), e = min(p.row_ptr[t + 1], p.cap);
  int c = 0;
  for (int k0 = b; k0 < e; k0 += TMD_WAVE) {
    const int k = k0 + lane;
    const bool canon = k < e && p.src[k] >= t;
    c += __popcll(__ballot(canon));
  }
  if (lane == 0) p.cnt[t] = c;
}

__device__ __forceinline__ void row_assign(const P& p, int t) {
  const int lane = lane_id();
  const int b = min(p.row_ptr[t], p.cap), e = min(p.row_ptr[t + 1], p.cap);
  int base = p.cnt[t];
  for (int k0 = b; k0 < e; k0 += TMD_WAVE) {
    const int k = k0 + lane;
    const bool live = k < e;
    const bool canon = live && p.src[k] >= t;
    const unsigned long long m = __ballot(canon);
    if (canon) {
      const int pid = base + lane_prefix(m);
      p.prow[k] = pid < p.slots ? pid : 0;  // (truncated lists: see k_fill_sorted)
      if (pid < p.slots) p.pedge[pid] = k;
    } else if (live) {
      p.prow[k] = -1;
    }
    base += __popcll(m);
  }
}

__device__ __forceinline__ void slot_fill(const P& p, int i, int ve, int total) {
  if (i < p.cap) {
    if (i >= ve) p.prow[i] = 0;
    else if (p.prow[i] < 0) p.prow[i] = p.tr[i] >= 0 ? p.prow[p.tr[i]] : 0;  // unpaired: inert row
  }
  if (i < p.slots && i >= total) p.pedge[i] = 0;
}

__global__ __launch_bounds__(256) void k_count(P p) {
  const int t = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (t < p.n) row_count(p, t);
}

// exclusive scan of cnt[0..n) in place, total in cnt[n] (one workgroup, chunk per thread)
__device__ __forceinline__ void block_scan(const P& p, long long* part) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int chunk = (p.n + nt - 1) / nt;
  const int b = tid * chunk, e = min(p.n, b + chunk);
  long long s = 0;
  for (int i = b; i < e; ++i) s += p.cnt[i];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < nt; o <<= 1) {
    const long long v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  long long run = part[tid] - s;
  for (int i = b; i < e; ++i) {
    const int c = p.cnt[i];
    p.cnt[i] = (int)run;
    run += c;
  }
  if (tid == nt - 1) p.cnt[p.n] = (int)part[nt - 1];
}

__global__ __launch_bounds__(1024) void k_scan(P p) {
  __shared__ long long part[1024];
  block_scan(p, part);
}

__global__ __launch_bounds__(256) void k_assign(P p) {
  const int t = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (t < p.n) row_assign(p, t);
}

__global__ __launch_bounds__(256) void k_fill(P p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < max(p.cap, p.slots)) slot_fill(p, i, valid_edges(p), p.cnt[p.n]);
}

// sorted rows, pass 1: canonical suffix length of row t (first in-row edge with src >= t)
__global__ __launch_bounds__(256) void k_count_sorted(P p) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n) return;
  const int b = min(p.row_ptr[t], p.cap), e = min(p.row_ptr[t + 1], p.cap);
  int lo = b, hi = e;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (p.src[m] < t) lo = m + 1; else hi = m;
  }
  p.cnt[t] = e - lo;
}

// sorted rows, pass 3: pid of edge i, closed form; pass 4's slot fill folded in
__global__ __launch_bounds__(256) void k_fill_sorted(P p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int ve = valid_edges(p), total = p.cnt[p.n];
  if (i < p.cap) {
    int pid = 0;
    if (i < ve) {
      const int s = p.src[i], t = p.dst[i];
      // canonical: own row t; otherwise the reverse edge, canonical in row s
      const int r = s >= t ? t : s;
      const int k = s >= t ? i : p.tr[i];
      if (k >= 0) {
        const int suffix0 = min(p.row_ptr[r + 1], p.cap) - (p.cnt[r + 1] - p.cnt[r]);
        pid = p.cnt[r] + (k - suffix0);
        if (s >= t && pid < p.slots) p.pedge[pid] = i;
      }
    }
    // a capacity-truncated list can hold more canonical edges than slots (its kept rows are a
    // prefix, canonical-heavy): such rows read slot 0, never past the buffer (the overflow is
    // reported by the capacity check)
    p.prow[i] = pid < p.slots ? pid : 0;
  }
  if (i < p.slots && i >= total) p.pedge[i] = 0;
}


}  // namespace pairs
}  // namespace tmd

using namespace tmd;

extern "C" size_t tmdnet_pair_index_workspace_bytes(int n_nodes) {
  return sizeof(int) * ((size_t)(n_nodes > 0 ? n_nodes : 0) + 1);
}

extern "C" int tmdnet_pair_index(int n_nodes, const int32_t* row_ptr, const int32_t* src, const int32_t* dst,
                                 const int32_t* transpose, int max_pairs, const int32_t* num_pairs,
                                 int sorted_rows, int32_t* pair_row, int32_t* pair_edge, int n_pair_slots,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  if (n_nodes <= 0 || max_pairs < 0 || n_pair_slots < 0 || !row_ptr || !src || !transpose || !pair_row ||
      !pair_edge || (sorted_rows && !dst))
    return kBadArgument;
  if (workspace_bytes < tmdnet_pair_index_workspace_bytes(n_nodes) || !workspace) return kWorkspaceTooSmall;
  hipStream_t st = (hipStream_t)stream;
  pairs::P p{n_nodes, max_pairs, row_ptr, src, dst, transpose, num_pairs, pair_row, pair_edge, n_pair_slots,
             (int*)workspace};
  const int m = max(max_pairs, n_pair_slots);
  if (sorted_rows) {
    hipLaunchKernelGGL(pairs::k_count_sorted, dim3((n_nodes + 255) / 256), dim3(256), 0, st, p);
    hipLaunchKernelGGL(pairs::k_scan, dim3(1), dim3(1024), 0, st, p);
    if (m > 0) hipLaunchKernelGGL(pairs::k_fill_sorted, dim3((m + 255) / 256), dim3(256), 0, st, p);
  } else {
    const int wpb = 256 / TMD_WAVE;
    const dim3 gr((n_nodes + wpb - 1) / wpb);
    hipLaunchKernelGGL(pairs::k_count, gr, dim3(256), 0, st, p);
    hipLaunchKernelGGL(pairs::k_scan, dim3(1), dim3(1024), 0, st, p);
    hipLaunchKernelGGL(pairs::k_assign, gr, dim3(256), 0, st, p);
    if (m > 0) hipLaunchKernelGGL(pairs::k_fill, dim3((m + 255) / 256), dim3(256), 0, st, p);
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
