// Per-molecule energy reduction of TorchMD_Net.forward (reference models/model.py:263-283 with
// output_modules.py:27-43): y[b] = mean + std * sum_{n: batch[n] = b} x[n], the `x * std`, the
// torch_scatter sum and the `+ mean` in ONE launch (the reference path is a multiply, a zero fill, an
// out-of-place index_add and an add); its backward g_x[n] = std * g_y[batch[n]] in one more.
// One workgroup accumulates every atom into LDS bins (the caller keeps n_mol <= kMaxBins; the
// reference's CUDA scatter is atomic too, so the summation order is unspecified in both).
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace red {

constexpr int kMaxBins = 8192;

template <typename T>
__global__ __launch_bounds__(1024) void k_atom_sum(int n, int n_mol, const T* __restrict__ x,
                                                   const int64_t* __restrict__ batch,
                                                   const T* __restrict__ std_, const T* __restrict__ mean,
                                                   T* __restrict__ y) {
  __shared__ T bins[kMaxBins];
  for (int b = threadIdx.x; b < n_mol; b += blockDim.x) bins[b] = T(0);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t b = batch[i];
    if (b >= 0 && b < n_mol) atomicAdd(&bins[b], x[i]);
  }
  __syncthreads();
  const T s = std_ ? *std_ : T(1), m = mean ? *mean : T(0);
  for (int b = threadIdx.x; b < n_mol; b += blockDim.x) y[b] = m + s * bins[b];
}

template <typename T>
__global__ void k_atom_sum_bwd(int n, int n_mol, const T* __restrict__ gy, const int64_t* __restrict__ batch,
                               const T* __restrict__ std_, T* __restrict__ gx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t b = batch[i];
  const T s = std_ ? *std_ : T(1);
  gx[i] = (b >= 0 && b < n_mol) ? s * gy[b] : T(0);
}

// Scalar head tail + reduction (reference output_modules.py:83-105 Scalar: Linear(H/2 -> 1) after the
// SiLU, then TorchMD_Net's `x * std`, per-molecule sum and `+ mean`): y[b] = mean + std * sum_n (h[n].w + b0).
// One wave per atom row (K values, lane-strided), the molecule sums in LDS bins.
template <typename T>
__global__ __launch_bounds__(1024) void k_dot_sum(int n, int K, const T* __restrict__ h, int ldh,
                                                  const T* __restrict__ w, const T* __restrict__ b0,
                                                  int n_mol, const int64_t* __restrict__ batch,
                                                  const T* __restrict__ std_, const T* __restrict__ mean,
                                                  T* __restrict__ y) {
  __shared__ T bins[kMaxBins];
  for (int b = threadIdx.x; b < n_mol; b += blockDim.x) bins[b] = T(0);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const T bias = b0 ? *b0 : T(0);
  for (int i = wid; i < n; i += nw) {
    const T* hr = h + (size_t)i * ldh;
    T s = T(0);
    for (int k = lane; k < K; k += 64) s += hr[k] * w[k];
    s = wave_sum(s);
    const int64_t b = batch[i];
    if (lane == 0 && b >= 0 && b < n_mol) atomicAdd(&bins[b], s + bias);
  }
  __syncthreads();
  const T sc = std_ ? *std_ : T(1), m = mean ? *mean : T(0);
  for (int b = threadIdx.x; b < n_mol; b += blockDim.x) y[b] = m + sc * bins[b];
}

// Large systems (one 50k-atom box: the single-workgroup k_dot_sum walked 50k rows in 16 waves, 2.2 ms): the
// row products over the whole grid, 16 lanes per row -> atom[n] = h[n].w + b0, then k_atom_runs sums them.
template <typename T>
__global__ __launch_bounds__(256) void k_row_dot(int n, int K, const T* __restrict__ h, int ldh,
                                                 const T* __restrict__ w, const T* __restrict__ b0,
                                                 T* __restrict__ atom) {
  const int g = threadIdx.x & 15;
  const long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const bool on = row < n;
  const T* hr = h + (size_t)(on ? row : 0) * ldh;
  T s = T(0);
  for (int k = g; k < K; k += 16) s += hr[k] * w[k];
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 16);
  if (on && g == 0) atom[row] = s + (b0 ? *b0 : T(0));
}

// y[b] = mean + std * sum_{batch[n] = b} x[n] for many atoms: thread t sums a contiguous chunk, flushing its
// running sum to the molecule's LDS bin only when the molecule changes (batches are molecule-contiguous in
// practice: ~1 LDS atomic per thread instead of one per atom on one bin).
template <typename T>
__global__ __launch_bounds__(1024) void k_atom_runs(int n, int n_mol, const T* __restrict__ x,
                                                    const int64_t* __restrict__ batch, const T* __restrict__ std_,
                                                    const T* __restrict__ mean, T* __restrict__ y) {
  __shared__ T bins[kMaxBins];
  for (int b = threadIdx.x; b < n_mol; b += blockDim.x) bins[b] = T(0);
  __syncthreads();
  const int c = (n + (int)blockDim.x - 1) / (int)blockDim.x;
  const int i0 = threadIdx.x * c, i1 = min(n, i0 + c);
  int64_t cur = -1;
  T acc = T(0);
  for (int i = i0; i < i1; ++i) {
    const int64_t b = batch[i];
    if (b != cur) {
      if (cur >= 0 && cur < n_mol) atomicAdd(&bins[cur], acc);
      cur = b;
      acc = T(0);
    }
    acc += x[i];
  }
  if (cur >= 0 && cur < n_mol) atomicAdd(&bins[cur], acc);
  __syncthreads();
  const T sc = std_ ? *std_ : T(1), m = mean ? *mean : T(0);
  for (int b = threadIdx.x; b < n_mol; b += blockDim.x) y[b] = m + sc * bins[b];
}

// its input gradient: gh[n][k] = std * gy[batch[n]] * w[k]
template <typename T>
__global__ void k_dot_sum_bwd(int n, int K, const T* __restrict__ gy, const int64_t* __restrict__ batch, int n_mol,
                              const T* __restrict__ std_, const T* __restrict__ w, T* __restrict__ gh) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n * K) return;
  const int a = (int)(i / K), k = (int)(i % K);
  const int64_t b = batch[a];
  const T sc = std_ ? *std_ : T(1);
  gh[i] = (b >= 0 && b < n_mol) ? sc * gy[b] * w[k] : T(0);
}

}  // namespace red
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_atom_sum_fwd(int dtype, int n_atoms, int n_mol, const void* x, const int64_t* batch,
                                   const void* std_, const void* mean, void* y, void* stream) {
  if (n_atoms < 0 || n_mol <= 0 || n_mol > red::kMaxBins || !x || !batch || !y) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  // large systems: contiguous chunks per thread with run-length flushes (one LDS atomic per molecule change,
  // not one per atom on the same bin)
  const bool runs = n_atoms > 4096;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(runs ? red::k_atom_runs<float> : red::k_atom_sum<float>, dim3(1), dim3(1024), 0, st, n_atoms,
                       n_mol, (const float*)x, batch, (const float*)std_, (const float*)mean, (float*)y);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(runs ? red::k_atom_runs<double> : red::k_atom_sum<double>, dim3(1), dim3(1024), 0, st,
                       n_atoms, n_mol, (const double*)x, batch, (const double*)std_, (const double*)mean, (double*)y);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_atom_sum_bwd(int dtype, int n_atoms, int n_mol, const void* grad_y, const int64_t* batch,
                                   const void* std_, void* grad_x, void* stream) {
  if (n_atoms < 0 || n_mol <= 0 || !grad_y || !batch || !grad_x) return kBadArgument;
  if (n_atoms == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)((n_atoms + 255) / 256));
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(red::k_atom_sum_bwd<float>, g, dim3(256), 0, st, n_atoms, n_mol, (const float*)grad_y,
                       batch, (const float*)std_, (float*)grad_x);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(red::k_atom_sum_bwd<double>, g, dim3(256), 0, st, n_atoms, n_mol, (const double*)grad_y,
                       batch, (const double*)std_, (double*)grad_x);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_dot_sum_fwd(int dtype, int n_atoms, int K, const void* h, int ld_h, const void* w,
                                  const void* b0, int n_mol, const int64_t* batch, const void* std_,
                                  const void* mean, void* y, void* stream) {
  if (n_atoms < 0 || K <= 0 || ld_h < K || n_mol <= 0 || n_mol > red::kMaxBins || !h || !w || !batch || !y)
    return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(red::k_dot_sum<float>, dim3(1), dim3(1024), 0, st, n_atoms, K, (const float*)h, ld_h,
                       (const float*)w, (const float*)b0, n_mol, batch, (const float*)std_, (const float*)mean,
                       (float*)y);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(red::k_dot_sum<double>, dim3(1), dim3(1024), 0, st, n_atoms, K, (const double*)h, ld_h,
                       (const double*)w, (const double*)b0, n_mol, batch, (const double*)std_,
                       (const double*)mean, (double*)y);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_dot_sum_bwd(int dtype, int n_atoms, int K, const void* grad_y, const int64_t* batch, int n_mol,
                                  const void* std_, const void* w, void* grad_h, void* stream) {
  if (n_atoms < 0 || K <= 0 || n_mol <= 0 || !grad_y || !batch || !w || !grad_h) return kBadArgument;
  if (n_atoms == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const long long tot = (long long)n_atoms * K;
  const dim3 g((unsigned)((tot + 255) / 256));
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(red::k_dot_sum_bwd<float>, g, dim3(256), 0, st, n_atoms, K, (const float*)grad_y, batch, n_mol,
                       (const float*)std_, (const float*)w, (float*)grad_h);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(red::k_dot_sum_bwd<double>, g, dim3(256), 0, st, n_atoms, K, (const double*)grad_y, batch,
                       n_mol, (const double*)std_, (const double*)w, (double*)grad_h);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// tmdnet_dot_sum_fwd for large systems: the row products over the whole grid into atom_buf [n_atoms] (the
// per-atom energies before std / mean), then the per-molecule sums.  atom_buf NULL: tmdnet_dot_sum_fwd.
extern "C" int tmdnet_dot_sum_fwd_atoms(int dtype, int n_atoms, int K, const void* h, int ld_h, const void* w,
                                        const void* b0, int n_mol, const int64_t* batch, const void* std_,
                                        const void* mean, void* atom_buf, void* y, void* stream) {
  if (!atom_buf) return tmdnet_dot_sum_fwd(dtype, n_atoms, K, h, ld_h, w, b0, n_mol, batch, std_, mean, y, stream);
  if (n_atoms < 0 || K <= 0 || ld_h < K || n_mol <= 0 || n_mol > red::kMaxBins || !h || !w || !batch || !y)
    return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)(((long long)n_atoms * 16 + 255) / 256));
#define TMD_DOTS(T)                                                                                            \
  if (n_atoms > 0)                                                                                             \
    hipLaunchKernelGGL(red::k_row_dot<T>, g, dim3(256), 0, st, n_atoms, K, (const T*)h, ld_h, (const T*)w,     \
                       (const T*)b0, (T*)atom_buf);                                                            \
  hipLaunchKernelGGL(red::k_atom_runs<T>, dim3(1), dim3(1024), 0, st, n_atoms, n_mol, (const T*)atom_buf, batch, \
                     (const T*)std_, (const T*)mean, (T*)y);
  if (dtype == TMDNET_F32) {
    TMD_DOTS(float)
  } else if (dtype == TMDNET_F64) {
    TMD_DOTS(double)
  } else {
    return kUnsupported;
  }
#undef TMD_DOTS
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
