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
// put: store, or (acc: the output buffer holds cotangents injected by the second order) add
template <typename T>
__device__ __forceinline__ void put(T* p, T v, bool acc) { *p = acc ? *p + v : v; }

template <typename T>
__global__ void k_bwd(int n, int H, const T* __restrict__ gx, const T* __restrict__ gvec,
                      const T* __restrict__ vecp, const T* __restrict__ o, T* __restrict__ gvecp,
                      T* __restrict__ go, int acc) {
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
    put(gt + c, T(0), acc);
    put(gt + H + c, T(0), acc);
    put(gt + 2 * H + c, g, acc);
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
    put(gvp + a * 3 * H + c, gd * v2, acc);
    put(gvp + a * 3 * H + H + c, gd * v1, acc);
    put(gvp + a * 3 * H + 2 * H + c, gv * o1, acc);
  }
  put(gt + c, go1, acc);
  put(gt + H + c, g * dot, acc);
  put(gt + 2 * H + c, g, acc);
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

extern "C" int tmdnet_et_epilogue_bwd_acc(int dtype, int n_nodes, int hidden, const void* grad_x,
                                          const void* grad_vec, const void* vecp, const void* o,
                                          void* grad_vecp, void* grad_o, int accumulate, void* stream);

extern "C" int tmdnet_et_epilogue_bwd(int dtype, int n_nodes, int hidden, const void* grad_x,
                                      const void* grad_vec, const void* vecp, const void* o,
                                      void* grad_vecp, void* grad_o, void* stream) {
  return tmdnet_et_epilogue_bwd_acc(dtype, n_nodes, hidden, grad_x, grad_vec, vecp, o, grad_vecp, grad_o, 0,
                                    stream);
}

extern "C" int tmdnet_et_epilogue_bwd_acc(int dtype, int n_nodes, int hidden, const void* grad_x,
                                          const void* grad_vec, const void* vecp, const void* o,
                                          void* grad_vecp, void* grad_o, int accumulate, void* stream) {
  const long long work = (long long)n_nodes * hidden;
  if (work <= 0) return kOk;
  const int tb = 256;
  dim3 g((unsigned)((work + tb - 1) / tb));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(epi::k_bwd<float>, g, dim3(tb), 0, st, n_nodes, hidden, (const float*)grad_x,
                       (const float*)grad_vec, (const float*)vecp, (const float*)o, (float*)grad_vecp,
                       (float*)grad_o, accumulate);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(epi::k_bwd<double>, g, dim3(tb), 0, st, n_nodes, hidden, (const double*)grad_x,
                       (const double*)grad_vec, (const double*)vecp, (const double*)o,
                       (double*)grad_vecp, (double*)grad_o, accumulate);
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
                                                    T* __restrict__ go, T* __restrict__ wrows,
                                                    const T* __restrict__ gres2, int acc) {
  const int t = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  const T mu = mean[t], rs = rstd[t];
  T gh[CPL], xh[CPL];
  // the epilogue-backward operands are loaded with the LayerNorm's, before the two row sums: one
  // memory round trip per node instead of two (C2: 9 -> see DESIGN 3b)
  T gr[CPL], o1[CPL], o2[CPL], vq[CPL][9], gq[CPL][3];
  // accumulate mode: the outputs' current values, loaded here too (a read-modify-write after the row sums
  // was a second dependent memory round trip: 13-17 us per launch in the training step vs 5-6 us)
  T pv[CPL][9], po[CPL][3];
  const bool ev = o != nullptr && vecp != nullptr;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    gr[i] = o1[i] = o2[i] = T(0);
#pragma unroll
    for (int a = 0; a < 9; ++a) vq[i][a] = pv[i][a] = T(0);
#pragma unroll
    for (int a = 0; a < 3; ++a) gq[i][a] = po[i][a] = T(0);
    if (c >= H) continue;
    if (acc && o) {
      const T* gt = go + (size_t)t * 3 * H;
#pragma unroll
      for (int a = 0; a < 3; ++a) po[i][a] = gt[a * H + c];
      if (vecp) {
        const T* gvp = gvecp + (size_t)t * 9 * H;
#pragma unroll
        for (int a = 0; a < 9; ++a) pv[i][a] = gvp[a * H + c];
      }
    }
    if (gres) gr[i] += gres[(size_t)t * H + c];
    if (gres2) gr[i] += gres2[(size_t)t * H + c];
    if (ev) {
      const T* ot = o + (size_t)t * 3 * H;
      const T* vp = vecp + (size_t)t * 9 * H;
      o1[i] = ot[c];
      o2[i] = ot[H + c];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        vq[i][3 * a] = vp[a * 3 * H + c];
        vq[i][3 * a + 1] = vp[a * 3 * H + H + c];
        vq[i][3 * a + 2] = vp[a * 3 * H + 2 * H + c];
        gq[i][a] = gvec[((size_t)t * 3 + a) * H + c];
      }
    }
  }
  T s1 = T(0), s2 = T(0);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    gh[i] = xh[i] = T(0);
    if (c >= H) continue;
    xh[i] = (x[(size_t)t * H + c] - mu) * rs;
    const T gn = gxn[(size_t)t * H + c];
    if (wrows) wrows[(size_t)t * H + c] = gn * xh[i];  // the LayerNorm weight gradient's row term
    gh[i] = gn * lw[c];
    s1 += gh[i];
    s2 += gh[i] * xh[i];
  }
  const T m1 = wsum(s1) / T(H), m2 = wsum(s2) / T(H);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c >= H) continue;
    const T g = gr[i] + rs * (gh[i] - m1 - xh[i] * m2);
    gx[(size_t)t * H + c] = g;
    if (!o) continue;
    T* gt = go + (size_t)t * 3 * H;
    if (!vecp) {
      gt[c] = po[i][0];
      gt[H + c] = po[i][1];
      gt[2 * H + c] = po[i][2] + g;
      continue;
    }
    T* gvp = gvecp + (size_t)t * 9 * H;
    T dot = T(0), go1 = T(0);
    const T gd = g * o2[i];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const T v1 = vq[i][3 * a], v2 = vq[i][3 * a + 1], v3 = vq[i][3 * a + 2];
      const T gv = gq[i][a];
      dot += v1 * v2;
      go1 += gv * v3;
      gvp[a * 3 * H + c] = pv[i][3 * a] + gd * v2;
      gvp[a * 3 * H + H + c] = pv[i][3 * a + 1] + gd * v1;
      gvp[a * 3 * H + 2 * H + c] = pv[i][3 * a + 2] + gv * o1[i];
    }
    gt[c] = po[i][0] + go1;
    gt[H + c] = po[i][1] + g * dot;
    gt[2 * H + c] = po[i][2] + g;
  }
}

// ---------------------------------------------------------------------------------------------
// Second order (force-matching training): the adjoint of the backward's node tail, fused per node
// (one wave per node, CPL channels per lane).  Layer l's epilogue-backward VJP and layer l+1's
// LayerNorm-backward VJP are adjacent in the adjoint pass (et_stack._second_order), so one kernel:
//   epilogue part (o != NULL), for cotangents gb_o [N][3H], gb_vecp [N][3][3H] of (g_o, g_vecp) =
//   EPI_BWD(gX, gV; vecp, o):
//     gbar_x_out  = gbar_x_in + gb_o2 dot + gb_o3 + o2 sum_a(c1 v2 + c2 v1)
//     gbar_vec_out = gbar_vec_in + gb_o1 v3 + c3 o1
//     vecp_bar = [gb_o2 gX v2 + c2 gX o2 | gb_o2 gX v1 + c1 gX o2 | gb_o1 gV],
//     o_bar = [sum_a c3 gV | gX sum_a(c1 v2 + c2 v1) | 0]        (c = gb_vecp; vecp NULL: only gb_o3)
//   LayerNorm part (ln_w != NULL), for the cotangent g = gbar_x_out (o NULL: gbar_x_in) of
//   g_x = LNB(g_y, x) = rstd (a - mean a - xh mean(a xh)), a = g_y w:
//     gbar_gy = w J0 g,  J0 v = rstd (v - mean v - xh mean(v xh))
//     x_bar   = -S rstd^2 xh / H - rstd/H ((a.xh) J0 g + (g.xh) J0 a),
//               S = g.a - (sum g)(sum a)/H - (g.xh)(a.xh)/H
//     w_rows  = g_y J0 g   (per row; the weight cotangent is its column sum)
template <typename T, int CPL>
__global__ __launch_bounds__(256) void k_adj_epi_ln(
    int n, int H, const T* __restrict__ gbo, const T* __restrict__ gbvp, const T* __restrict__ gX,
    const T* __restrict__ gV, const T* __restrict__ vecp, const T* __restrict__ o, const T* __restrict__ gbx_in,
    const T* __restrict__ gbv_in, const T* __restrict__ gbv_in2, T* __restrict__ gbx_out, T* __restrict__ gbv_out,
    T* __restrict__ vpbar, T* __restrict__ obar, const T* __restrict__ x, const T* __restrict__ mean,
    const T* __restrict__ rstd, const T* __restrict__ lw, const T* __restrict__ gy, T* __restrict__ gbgy,
    T* __restrict__ xbar, T* __restrict__ wrows) {
  const int t = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  T g[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    g[i] = T(0);
    if (c >= H) continue;
    const size_t ix = (size_t)t * H + c;
    T gb = gbx_in[ix];
    if (o) {
      const T* ot = o + (size_t)t * 3 * H;
      const T* bo = gbo + (size_t)t * 3 * H;
      const T o1 = ot[c], o2 = ot[H + c];
      const T b1 = bo[c], b2 = bo[H + c], b3 = bo[2 * H + c];
      T* ob = obar + (size_t)t * 3 * H;
      if (!vecp) {
        gb += b3;
        ob[c] = T(0);
        ob[H + c] = T(0);
        ob[2 * H + c] = T(0);
        if (gbv_out) {
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            const size_t iv = ((size_t)t * 3 + a) * H + c;
            gbv_out[iv] = (gbv_in ? gbv_in[iv] : T(0)) + (gbv_in2 ? gbv_in2[iv] : T(0));
          }
        }
      } else {
        const T* vp = vecp + (size_t)t * 9 * H;
        const T* cb = gbvp + (size_t)t * 9 * H;
        T* vb = vpbar + (size_t)t * 9 * H;
        const T gx = gX[ix];
        T dot = T(0), cross = T(0), o1b = T(0);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const T v1 = vp[a * 3 * H + c], v2 = vp[a * 3 * H + H + c], v3 = vp[a * 3 * H + 2 * H + c];
          const T c1 = cb[a * 3 * H + c], c2 = cb[a * 3 * H + H + c], c3 = cb[a * 3 * H + 2 * H + c];
          const size_t iv = ((size_t)t * 3 + a) * H + c;
          const T gv = gV[iv];
          dot += v1 * v2;
          cross += c1 * v2 + c2 * v1;
          o1b += c3 * gv;
          gbv_out[iv] = (gbv_in ? gbv_in[iv] : T(0)) + (gbv_in2 ? gbv_in2[iv] : T(0)) + b1 * v3 + c3 * o1;
          vb[a * 3 * H + c] = b2 * gx * v2 + c2 * gx * o2;
          vb[a * 3 * H + H + c] = b2 * gx * v1 + c1 * gx * o2;
          vb[a * 3 * H + 2 * H + c] = b1 * gv;
        }
        gb += b2 * dot + b3 + o2 * cross;
        ob[c] = o1b;
        ob[H + c] = gx * cross;
        ob[2 * H + c] = T(0);
      }
      gbx_out[ix] = gb;
    }
    g[i] = gb;
  }
  if (!lw) return;
  const T mu = mean[t], rs = rstd[t];
  T xh[CPL], av[CPL];
  T sg = T(0), sa = T(0), sgx = T(0), sax = T(0), sga = T(0);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    xh[i] = av[i] = T(0);
    if (c >= H) continue;
    const size_t ix = (size_t)t * H + c;
    xh[i] = (x[ix] - mu) * rs;
    av[i] = gy[ix] * lw[c];
    sg += g[i];
    sa += av[i];
    sgx += g[i] * xh[i];
    sax += av[i] * xh[i];
    sga += g[i] * av[i];
  }
  sg = wsum(sg);
  sa = wsum(sa);
  sgx = wsum(sgx);
  sax = wsum(sax);
  sga = wsum(sga);
  const T iH = T(1) / T(H);
  const T S = sga - sg * sa * iH - sgx * sax * iH;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c >= H) continue;
    const size_t ix = (size_t)t * H + c;
    const T jg = rs * (g[i] - sg * iH - xh[i] * sgx * iH);
    const T ja = rs * (av[i] - sa * iH - xh[i] * sax * iH);
    gbgy[ix] = lw[c] * jg;
    xbar[ix] = -S * rs * rs * xh[i] * iH - rs * iH * (sax * jg + sgx * ja);
    wrows[ix] = gy[ix] * jg;
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
template <typename T, int C> struct KAdj { static constexpr auto fn = epi::k_adj_epi_ln<T, C>; };

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

extern "C" int tmdnet_ln_bwd_epilogue_w(int dtype, int n_nodes, int hidden, const void* grad_xn, const void* x,
                                        const void* mean, const void* rstd, const void* ln_w,
                                        const void* grad_res, const void* grad_res2, void* grad_x,
                                        const void* grad_vec, const void* vecp, const void* o, void* grad_vecp,
                                        void* grad_o, void* w_rows, int accumulate, void* stream);

extern "C" int tmdnet_ln_bwd_epilogue(int dtype, int n_nodes, int hidden, const void* grad_xn, const void* x,
                                      const void* mean, const void* rstd, const void* ln_w,
                                      const void* grad_res, void* grad_x, const void* grad_vec,
                                      const void* vecp, const void* o, void* grad_vecp, void* grad_o,
                                      void* stream) {
  return tmdnet_ln_bwd_epilogue_w(dtype, n_nodes, hidden, grad_xn, x, mean, rstd, ln_w, grad_res, nullptr,
                                  grad_x, grad_vec, vecp, o, grad_vecp, grad_o, nullptr, 0, stream);
}

extern "C" int tmdnet_ln_bwd_epilogue_w(int dtype, int n_nodes, int hidden, const void* grad_xn, const void* x,
                                        const void* mean, const void* rstd, const void* ln_w,
                                        const void* grad_res, const void* grad_res2, void* grad_x,
                                        const void* grad_vec, const void* vecp, const void* o, void* grad_vecp,
                                        void* grad_o, void* w_rows, int accumulate, void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !grad_xn || !x || !mean || !rstd || !ln_w || !grad_x) return kBadArgument;
  if (o && (!grad_o || (vecp && (!grad_vec || !grad_vecp)))) return kBadArgument;
  if (n_nodes == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return launch_cpl<float, KLnBwd>(n_nodes, hidden, st, (const float*)grad_xn, (const float*)x,
                                     (const float*)mean, (const float*)rstd, (const float*)ln_w,
                                     (const float*)grad_res, (float*)grad_x, (const float*)grad_vec,
                                     (const float*)vecp, (const float*)o, (float*)grad_vecp, (float*)grad_o,
                                     (float*)w_rows, (const float*)grad_res2, accumulate);
  if (dtype == TMDNET_F64)
    return launch_cpl<double, KLnBwd>(n_nodes, hidden, st, (const double*)grad_xn, (const double*)x,
                                      (const double*)mean, (const double*)rstd, (const double*)ln_w,
                                      (const double*)grad_res, (double*)grad_x, (const double*)grad_vec,
                                      (const double*)vecp, (const double*)o, (double*)grad_vecp,
                                      (double*)grad_o, (double*)w_rows, (const double*)grad_res2, accumulate);
  return kUnsupported;
}

extern "C" int tmdnet_et_adjoint_epi_ln2(int dtype, int n_nodes, int hidden, const void* gb_o, const void* gb_vecp,
                                         const void* grad_x, const void* grad_vec, const void* vecp, const void* o,
                                         const void* gbar_x_in, const void* gbar_vec_in, const void* gbar_vec_in2,
                                         void* gbar_x_out, void* gbar_vec_out, void* vecp_bar, void* o_bar,
                                         const void* x, const void* mean, const void* rstd, const void* ln_w,
                                         const void* grad_xn, void* gbar_grad_xn, void* x_bar, void* w_bar_rows,
                                         void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !gbar_x_in) return kBadArgument;
  if (o && (!gb_o || !gbar_x_out || !o_bar || (vecp && (!gb_vecp || !grad_x || !grad_vec || !gbar_vec_out ||
                                                        !vecp_bar))))
    return kBadArgument;
  if (ln_w && (!x || !mean || !rstd || !grad_xn || !gbar_grad_xn || !x_bar || !w_bar_rows)) return kBadArgument;
  if (!o && !ln_w) return kBadArgument;
  if (n_nodes == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
#define TMD_ADJ(T)                                                                                            \
  return launch_cpl<T, KAdj>(n_nodes, hidden, st, (const T*)gb_o, (const T*)gb_vecp, (const T*)grad_x,       \
                             (const T*)grad_vec, (const T*)vecp, (const T*)o, (const T*)gbar_x_in,            \
                             (const T*)gbar_vec_in, (const T*)gbar_vec_in2, (T*)gbar_x_out, (T*)gbar_vec_out,    \
                             (T*)vecp_bar, (T*)o_bar,                                                          \
                             (const T*)x, (const T*)mean, (const T*)rstd, (const T*)ln_w, (const T*)grad_xn,  \
                             (T*)gbar_grad_xn, (T*)x_bar, (T*)w_bar_rows)
  if (dtype == TMDNET_F32) TMD_ADJ(float);
  if (dtype == TMDNET_F64) TMD_ADJ(double);
#undef TMD_ADJ
  return kUnsupported;
}

extern "C" int tmdnet_et_adjoint_epi_ln(int dtype, int n_nodes, int hidden, const void* gb_o, const void* gb_vecp,
                                        const void* grad_x, const void* grad_vec, const void* vecp, const void* o,
                                        const void* gbar_x_in, const void* gbar_vec_in, void* gbar_x_out,
                                        void* gbar_vec_out, void* vecp_bar, void* o_bar, const void* x,
                                        const void* mean, const void* rstd, const void* ln_w, const void* grad_xn,
                                        void* gbar_grad_xn, void* x_bar, void* w_bar_rows, void* stream) {
  return tmdnet_et_adjoint_epi_ln2(dtype, n_nodes, hidden, gb_o, gb_vecp, grad_x, grad_vec, vecp, o, gbar_x_in,
                                   gbar_vec_in, nullptr, gbar_x_out, gbar_vec_out, vecp_bar, o_bar, x, mean, rstd,
                                   ln_w, grad_xn, gbar_grad_xn, x_bar, w_bar_rows, stream);
}
