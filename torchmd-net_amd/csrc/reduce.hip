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

}  // namespace red
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_atom_sum_fwd(int dtype, int n_atoms, int n_mol, const void* x, const int64_t* batch,
                                   const void* std_, const void* mean, void* y, void* stream) {
  if (n_atoms < 0 || n_mol <= 0 || n_mol > red::kMaxBins || !x || !batch || !y) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(red::k_atom_sum<float>, dim3(1), dim3(1024), 0, st, n_atoms, n_mol, (const float*)x,
                       batch, (const float*)std_, (const float*)mean, (float*)y);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(red::k_atom_sum<double>, dim3(1), dim3(1024), 0, st, n_atoms, n_mol, (const double*)x,
                       batch, (const double*)std_, (const double*)mean, (double*)y);
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
