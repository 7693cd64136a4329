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

// ------------------------------------------------------------------------------------------------
// Epilogue of layer l fused with the LayerNorm of layer l+1 (reference torchmd_et.py:262 LN at the
// start of EquivariantMultiHeadAttention.forward), and in the backward the LayerNorm backward of
// layer l + its residual with the epilogue backward of layer l-1.  One wave per node, channels
// c = lane + 64 i; two-pass statistics (mean, then centred variance), biased variance and
// rstd = 1/sqrt(var + eps) as torch.native_layer_norm.
namespace tmd {
namespace epi {

template <typename T>
__device__ __forceinline__ T wsum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// flags: bit0 = epilogue present (o != NULL), bit1 = LayerNorm present (ln_w != NULL)
template <typename T, int CPL>
__global__ __launch_bounds__(256) void k_epi_ln_fwd(int n, int H, const T* __restrict__ x,
                                                    const T* __restrict__ vec, const T* __restrict__ vecp,
                                                    const T* __restrict__ o, const T* __restrict__ veca,
                                                    const T* __restrict__ lw, const T* __restrict__ lb,
                                                    T eps, T* __restrict__ xo, T* __restrict__ veco,
                                                    T* __restrict__ xn, T* __restrict__ mean,
                                                    T* __restrict__ rstd) {
  const int t = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  T xv[CPL];
  T s = T(0);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    xv[i] = T(0);
    if (c >= H) continue;
    T xc = x[(size_t)t * H + c];
    if (o) {
      const T* ot = o + (size_t)t * 3 * H;
      const T o1 = ot[c], o2 = ot[H + c], o3 = ot[2 * H + c];
      if (vecp) {
        const T* vp = vecp + (size_t)t * 9 * H;
        T dot = T(0);
#pragma unroll
        for (int a = 0; a < 3; ++a) dot += vp[a * 3 * H + c] * vp[a * 3 * H + H + c];
        xc += dot * o2 + o3;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const size_t iv = ((size_t)t * 3 + a) * H + c;
          veco[iv] = vec[iv] + vp[a * 3 * H + 2 * H + c] * o1 + veca[iv];
        }
      } else {
        xc += o3;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const size_t iv = ((size_t)t * 3 + a) * H + c;
          veco[iv] = veca[iv];
        }
      }
      xo[(size_t)t * H + c] = xc;
    }
    xv[i] = xc;
    s += xc;
  }
  if (!lw) return;
  const T mu = wsum(s) / T(H);
  T q = T(0);
#pragma unroll
  for (int i = 0; i < CPL; ++i)
    if (lane + 64 * i < H) q += (xv[i] - mu) * (xv[i] - mu);
  const T rs = T(1) / sqrt(wsum(q) / T(H) + eps);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < H) xn[(size_t)t * H + c] = (xv[i] - mu) * rs * lw[c] + lb[c];
  }
  if (lane == 0) {
    mean[t] = mu;
    rstd[t] = rs;
  }
}

// g_x = g_res + LN_bwd(g_xn) (no weight gradients; g_res NULL: none); then, when o != NULL, the epilogue backward of
// the previous layer with (g_x, gvec): g_vecp [N][3][3H] (vecp NULL: first layer), g_o [N][3H].
template <typename T, int CPL>
__global__ __launch_bounds__(256) void k_ln_bwd_epi(int n, int H, const T* __restrict__ gxn,
                                                    const T* __restrict__ x, const T* __restrict__ mean,
                                                    const T* __restrict__ rstd, const T* __restrict__ lw,
                                                    const T* __restrict__ gres, T* __restrict__ gx,
                                                    const T* __restrict__ gvec, const T* __restrict__ vecp,
                                                    const T* __restrict__ o, T* __restrict__ gvecp,
                                                    T* __restrict__ go) {
  const int t = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  const T mu = mean[t], rs = rstd[t];
  T gh[CPL], xh[CPL];
  T s1 = T(0), s2 = T(0);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    gh[i] = xh[i] = T(0);
    if (c >= H) continue;
    xh[i] = (x[(size_t)t * H + c] - mu) * rs;
    gh[i] = gxn[(size_t)t * H + c] * lw[c];
    s1 += gh[i];
    s2 += gh[i] * xh[i];
  }
  const T m1 = wsum(s1) / T(H), m2 = wsum(s2) / T(H);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c >= H) continue;
    const T g = (gres ? gres[(size_t)t * H + c] : T(0)) + rs * (gh[i] - m1 - xh[i] * m2);
    gx[(size_t)t * H + c] = g;
    if (!o) continue;
    const T* ot = o + (size_t)t * 3 * H;
    T* gt = go + (size_t)t * 3 * H;
    if (!vecp) {
      gt[c] = T(0);
      gt[H + c] = T(0);
      gt[2 * H + c] = g;
      continue;
    }
    const T* vp = vecp + (size_t)t * 9 * H;
    T* gvp = gvecp + (size_t)t * 9 * H;
    const T o1 = ot[c], o2 = ot[H + c];
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
}

}  // namespace epi
}  // namespace tmd

template <typename T, template <typename, int> class K, typename... A>
static int launch_cpl(int n, int H, hipStream_t st, A... args) {
  const int cpl = (H + 63) / 64;
  dim3 g((n + 3) / 4), b(256);
  if (cpl == 1) hipLaunchKernelGGL((K<T, 1>::fn), g, b, 0, st, n, H, args...);
  else if (cpl == 2) hipLaunchKernelGGL((K<T, 2>::fn), g, b, 0, st, n, H, args...);
  else if (cpl <= 4) hipLaunchKernelGGL((K<T, 4>::fn), g, b, 0, st, n, H, args...);
  else if (cpl <= 8) hipLaunchKernelGGL((K<T, 8>::fn), g, b, 0, st, n, H, args...);
  else return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T, int C> struct KEpiLn { static constexpr auto fn = epi::k_epi_ln_fwd<T, C>; };
template <typename T, int C> struct KLnBwd { static constexpr auto fn = epi::k_ln_bwd_epi<T, C>; };

extern "C" int tmdnet_et_epilogue_ln_fwd(int dtype, int n_nodes, int hidden, const void* x, const void* vec,
                                         const void* vecp, const void* o, const void* vec_agg,
                                         const void* ln_w, const void* ln_b, double eps, void* x_out,
                                         void* vec_out, void* xn, void* mean, void* rstd, void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !x) return kBadArgument;
  if (!o && !ln_w) return kBadArgument;
  if (o && (!vec_agg || !x_out || !vec_out || (vecp && !vec))) return kBadArgument;
  if (ln_w && (!ln_b || !xn || !mean || !rstd)) return kBadArgument;
  if (n_nodes == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return launch_cpl<float, KEpiLn>(n_nodes, hidden, st, (const float*)x, (const float*)vec,
                                     (const float*)vecp, (const float*)o, (const float*)vec_agg,
                                     (const float*)ln_w, (const float*)ln_b, (float)eps, (float*)x_out,
                                     (float*)vec_out, (float*)xn, (float*)mean, (float*)rstd);
  if (dtype == TMDNET_F64)
    return launch_cpl<double, KEpiLn>(n_nodes, hidden, st, (const double*)x, (const double*)vec,
                                      (const double*)vecp, (const double*)o, (const double*)vec_agg,
                                      (const double*)ln_w, (const double*)ln_b, eps, (double*)x_out,
                                      (double*)vec_out, (double*)xn, (double*)mean, (double*)rstd);
  return kUnsupported;
}

extern "C" int tmdnet_ln_bwd_epilogue(int dtype, int n_nodes, int hidden, const void* grad_xn, const void* x,
                                      const void* mean, const void* rstd, const void* ln_w,
                                      const void* grad_res, void* grad_x, const void* grad_vec,
                                      const void* vecp, const void* o, void* grad_vecp, void* grad_o,
                                      void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !grad_xn || !x || !mean || !rstd || !ln_w || !grad_x) return kBadArgument;
  if (o && (!grad_o || (vecp && (!grad_vec || !grad_vecp)))) return kBadArgument;
  if (n_nodes == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return launch_cpl<float, KLnBwd>(n_nodes, hidden, st, (const float*)grad_xn, (const float*)x,
                                     (const float*)mean, (const float*)rstd, (const float*)ln_w,
                                     (const float*)grad_res, (float*)grad_x, (const float*)grad_vec,
                                     (const float*)vecp, (const float*)o, (float*)grad_vecp, (float*)grad_o);
  if (dtype == TMDNET_F64)
    return launch_cpl<double, KLnBwd>(n_nodes, hidden, st, (const double*)grad_xn, (const double*)x,
                                      (const double*)mean, (const double*)rstd, (const double*)ln_w,
                                      (const double*)grad_res, (double*)grad_x, (const double*)grad_vec,
                                      (const double*)vecp, (const double*)o, (double*)grad_vecp,
                                      (double*)grad_o);
  return kUnsupported;
}
