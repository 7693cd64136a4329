// ET layer epilogue: the node-level elementwise tail of EquivariantMultiHeadAttention.forward
// (reference models/torchmd_et.py:278-280 and 309-311) plus the residual updates of
// TorchMD_ET.forward (torchmd_et.py:181-184), fused into one pass:
//   vec_dot = sum_a vec1[a] * vec2[a]                       (vecp = vec_proj(vec) = [vec1|vec2|vec3])
//   x_out   = x   + vec_dot * o2 + o3                         (o = o_proj(x_agg) = [o1|o2|o3])
//   vec_out = vec + vec3 * o1 + vec_agg
// and its backward.  One thread per (node, channel); every load/store is a coalesced row segment.
// These replace ~8 elementwise launches per layer forward and ~10 in the backward.
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace epi {

template <typename T>
__global__ void k_fwd(int n, int H, const T* __restrict__ x, const T* __restrict__ vec,
                      const T* __restrict__ vecp, const T* __restrict__ o,
                      const T* __restrict__ veca, T* __restrict__ xo, T* __restrict__ veco) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n * H) return;
  const int t = (int)(i / H), c = (int)(i % H);
  const T* vp = vecp + (size_t)t * 9 * H;  // [3][3H] (unused when null)
  const T* ot = o + (size_t)t * 3 * H;
  const T o1 = ot[c], o2 = ot[H + c], o3 = ot[2 * H + c];
  if (vecp == nullptr) {  // vec == 0 (first layer): vec_dot = 0, vec3 = 0
    xo[(size_t)t * H + c] = x[(size_t)t * H + c] + o3;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const size_t iv = ((size_t)t * 3 + a) * H + c;
      veco[iv] = veca[iv];
    }
    return;
  }
  T dot = T(0);
#pragma unroll
  for (int a = 0; a < 3; ++a) dot += vp[a * 3 * H + c] * vp[a * 3 * H + H + c];
  xo[(size_t)t * H + c] = x[(size_t)t * H + c] + dot * o2 + o3;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const size_t iv = ((size_t)t * 3 + a) * H + c;
    veco[iv] = vec[iv] + vp[a * 3 * H + 2 * H + c] * o1 + veca[iv];
  }
}

// gx, gvec: gradients of x_out, vec_out.  Writes g_vecp [N][3][3H], g_o [N][3H].
// (the gradients of x, vec and vec_agg are gx, gvec themselves: identity, no pass needed)
template <typename T>
__global__ void k_bwd(int n, int H, const T* __restrict__ gx, const T* __restrict__ gvec,
                      const T* __restrict__ vecp, const T* __restrict__ o, T* __restrict__ gvecp,
                      T* __restrict__ go) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n * H) return;
  const int t = (int)(i / H), c = (int)(i % H);
  const T* vp = vecp + (size_t)t * 9 * H;
  T* gvp = gvecp + (size_t)t * 9 * H;
  const T* ot = o + (size_t)t * 3 * H;
  const T o1 = ot[c], o2 = ot[H + c];
  const T g = gx[(size_t)t * H + c];
  T* gt = go + (size_t)t * 3 * H;
  if (vecp == nullptr) {
    gt[c] = T(0);
    gt[H + c] = T(0);
    gt[2 * H + c] = g;
    return;
  }
  T dot = T(0), go1 = T(0);
  const T gd = g * o2;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const T v1 = vp[a * 3 * H + c], v2 = vp[a * 3 * H + H + c], v3 = vp[a * 3 * H + 2 * H + c];
    const T gv = gvec[((size_t)t * 3 + a) * H + c];
    dot += v1 * v2;
    go1 += gv * v3;
    gvp[a * 3 * H + c] = gd * v2;
    gvp[a * 3 * H + H + c] = gd * v1;
    gvp[a * 3 * H + 2 * H + c] = gv * o1;
  }
  gt[c] = go1;
  gt[H + c] = g * dot;
  gt[2 * H + c] = g;
}

}  // namespace epi
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_et_epilogue_fwd(int dtype, int n_nodes, int hidden, const void* x,
                                      const void* vec, const void* vecp, const void* o,
                                      const void* vec_agg, void* x_out, void* vec_out, void* stream) {
  const long long work = (long long)n_nodes * hidden;
  if (work <= 0) return kOk;
  const int tb = 256;
  dim3 g((unsigned)((work + tb - 1) / tb));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(epi::k_fwd<float>, g, dim3(tb), 0, st, n_nodes, hidden, (const float*)x,
                       (const float*)vec, (const float*)vecp, (const float*)o, (const float*)vec_agg,
                       (float*)x_out, (float*)vec_out);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(epi::k_fwd<double>, g, dim3(tb), 0, st, n_nodes, hidden, (const double*)x,
                       (const double*)vec, (const double*)vecp, (const double*)o, (const double*)vec_agg,
                       (double*)x_out, (double*)vec_out);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_et_epilogue_bwd(int dtype, int n_nodes, int hidden, const void* grad_x,
                                      const void* grad_vec, const void* vecp, const void* o,
                                      void* grad_vecp, void* grad_o, void* stream) {
  const long long work = (long long)n_nodes * hidden;
  if (work <= 0) return kOk;
  const int tb = 256;
  dim3 g((unsigned)((work + tb - 1) / tb));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(epi::k_bwd<float>, g, dim3(tb), 0, st, n_nodes, hidden, (const float*)grad_x,
                       (const float*)grad_vec, (const float*)vecp, (const float*)o, (float*)grad_vecp,
                       (float*)grad_o);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(epi::k_bwd<double>, g, dim3(tb), 0, st, n_nodes, hidden, (const double*)grad_x,
                       (const double*)grad_vec, (const double*)vecp, (const double*)o,
                       (double*)grad_vecp, (double*)grad_o);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
