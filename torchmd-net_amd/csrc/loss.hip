// Energy + force MSE training loss (reference LNNP.step, module.py:130-179: y_weight * mse(y) +
// neg_dy_weight * mse(neg_dy), both with mean reduction) as one forward and one backward launch.
// In the captured training step the composite (mse_loss x2, the weights, the sum and their backward:
// ~14 ATen launches of 4-5 us) sits on the critical path between the forward and the double backward.
//   forward:  out = w1 * mean((a1 - b1)^2) + w2 * mean((a2 - b2)^2)   (one workgroup, fixed-order sum)
//   backward: d1 = g * w1 * 2 (a1 - b1) / n1,  d2 = g * w2 * 2 (a2 - b2) / n2   (g read on the device)
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace loss {

template <typename T>
__global__ __launch_bounds__(1024) void k_mse2_fwd(int n1, const T* __restrict__ a1, const T* __restrict__ b1, T w1,
                                                   int n2, const T* __restrict__ a2, const T* __restrict__ b2, T w2,
                                                   T* __restrict__ out) {
  __shared__ T red[2][1024 / TMD_WAVE];
  T s1 = T(0), s2 = T(0);
  for (int i = threadIdx.x; i < n1; i += blockDim.x) {
    const T d = a1[i] - b1[i];
    s1 += d * d;
  }
  for (int i = threadIdx.x; i < n2; i += blockDim.x) {
    const T d = a2[i] - b2[i];
    s2 += d * d;
  }
  for (int o = TMD_WAVE / 2; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int w = threadIdx.x / TMD_WAVE, nw = blockDim.x / TMD_WAVE;
  if (lane_id() == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    T t1 = T(0), t2 = T(0);
    for (int i = 0; i < nw; ++i) {
      t1 += red[0][i];
      t2 += red[1][i];
    }
    out[0] = (n1 > 0 ? w1 * t1 / T(n1) : T(0)) + (n2 > 0 ? w2 * t2 / T(n2) : T(0));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_mse2_bwd(int n1, const T* __restrict__ a1, const T* __restrict__ b1, T w1,
                                                  int n2, const T* __restrict__ a2, const T* __restrict__ b2, T w2,
                                                  const T* __restrict__ gout, T* __restrict__ d1, T* __restrict__ d2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const T g = gout[0];
  if (i < n1 && d1) d1[i] = g * w1 * T(2) * (a1[i] - b1[i]) / T(n1);
  if (i < n2 && d2) d2[i] = g * w2 * T(2) * (a2[i] - b2[i]) / T(n2);
}

template <typename T>
static int fwd(int n1, const void* a1, const void* b1, double w1, int n2, const void* a2, const void* b2, double w2,
               void* out, hipStream_t st) {
  hipLaunchKernelGGL(k_mse2_fwd<T>, dim3(1), dim3(1024), 0, st, n1, (const T*)a1, (const T*)b1, (T)w1, n2,
                     (const T*)a2, (const T*)b2, (T)w2, (T*)out);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static int bwd(int n1, const void* a1, const void* b1, double w1, int n2, const void* a2, const void* b2, double w2,
               const void* gout, void* d1, void* d2, hipStream_t st) {
  const int n = max(n1, n2);
  if (n == 0) return kOk;
  hipLaunchKernelGGL(k_mse2_bwd<T>, dim3((n + 255) / 256), dim3(256), 0, st, n1, (const T*)a1, (const T*)b1, (T)w1,
                     n2, (const T*)a2, (const T*)b2, (T)w2, (const T*)gout, (T*)d1, (T*)d2);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

}  // namespace loss
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_mse2_fwd(int dtype, int n1, const void* a1, const void* b1, double w1, int n2, const void* a2,
                               const void* b2, double w2, void* out, void* stream) {
  if (n1 < 0 || n2 < 0 || !out || (n1 && (!a1 || !b1)) || (n2 && (!a2 || !b2))) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) return loss::fwd<float>(n1, a1, b1, w1, n2, a2, b2, w2, out, st);
  if (dtype == TMDNET_F64) return loss::fwd<double>(n1, a1, b1, w1, n2, a2, b2, w2, out, st);
  return kUnsupported;
}

extern "C" int tmdnet_mse2_bwd(int dtype, int n1, const void* a1, const void* b1, double w1, int n2, const void* a2,
                               const void* b2, double w2, const void* grad_out, void* d1, void* d2, void* stream) {
  if (n1 < 0 || n2 < 0 || !grad_out || (n1 && (!a1 || !b1)) || (n2 && (!a2 || !b2))) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) return loss::bwd<float>(n1, a1, b1, w1, n2, a2, b2, w2, grad_out, d1, d2, st);
  if (dtype == TMDNET_F64) return loss::bwd<double>(n1, a1, b1, w1, n2, a2, b2, w2, grad_out, d1, d2, st);
  return kUnsupported;
}
