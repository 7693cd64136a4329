// LayerNorm over the last dimension (reference nn.LayerNorm, eps 1e-5): TensorNet's init_norm
// (models/tensornet.py:322, C = H) and out_norm (:232, C = 3H), the rows being atoms.
//
// Forward: one wave per row, the row in registers (CPL = C / 64 values per lane), mean and variance by
// two wave reductions (the exact two-pass form), y = (x - mean) * rstd * w + b; mean / rstd saved.
// Backward (input): gx = rstd * (g w - mean(g w) - xhat * mean(g w xhat)), one wave per row.
// Weight / bias gradients (training only): column sums of g * xhat and g over the rows, in two
// deterministic passes (row-chunk partials in chunk order, then their sum).
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace ln {

template <int CPL>
__global__ __launch_bounds__(256) void k_fwd(int rows, int C, const float* __restrict__ x, int ldx,
                                             const float* __restrict__ w, const float* __restrict__ b, float eps,
                                             float* __restrict__ y, int ldy, float* __restrict__ mean,
                                             float* __restrict__ rstd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (row >= rows) return;
  const float* xr = x + (size_t)row * ldx;
  float v[CPL];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? xr[c] : 0.f;
    s += v[j];
  }
  const float mu = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    const float d = c < C ? v[j] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / (float)C + eps);
  float* yr = y + (size_t)row * ldy;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    if (c < C) yr[c] = (v[j] - mu) * rs * w[c] + b[c];
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

template <int CPL>
__global__ __launch_bounds__(256) void k_bwd(int rows, int C, const float* __restrict__ x, int ldx,
                                             const float* __restrict__ w, const float* __restrict__ mean,
                                             const float* __restrict__ rstd, const float* __restrict__ gy,
                                             int ldg, float* __restrict__ gx, int acc) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (row >= rows) return;
  const float mu = mean[row], rs = rstd[row];
  const float* xr = x + (size_t)row * ldx;
  const float* gr = gy + (size_t)row * ldg;
  float h[CPL], gw[CPL];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    h[j] = c < C ? (xr[c] - mu) * rs : 0.f;
    gw[j] = c < C ? gr[c] * w[c] : 0.f;
    s1 += gw[j];
    s2 += gw[j] * h[j];
  }
  const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
  float* o = gx + (size_t)row * C;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    if (c < C) {
      const float v = rs * (gw[j] - m1 - h[j] * m2);
      o[c] = acc ? o[c] + v : v;
    }
  }
}

// Second order (force-matching training through TensorNet's init_norm / out_norm): the VJP of the first
// backward (gx = r (G - mean G - h mean(G h)), G = gy w, h = (x - mean) r; gw = colsum gy h; gb = colsum gy) for
// cotangents (X, Wb, Bb) of (gx, gw, gb), per row (one wave):
//   T     = r (X - mean X - h mean(X h))                      (dw = colsum gy T, formed by the caller)
//   d_gy  = w T + Wb h + Bb
//   u     = -r (G mean(X h) + mean(G h) X) + Wb gy            (the adjoint of h)
//   v     = sum X (G - mean G - h mean(G h))                  (the adjoint of r, times r)
//   d_x   = r (u - mean u - h mean(u h)) - v r^2 h / C
template <int CPL>
__global__ __launch_bounds__(256) void k_bwd2(int rows, int C, const float* __restrict__ x, int ldx,
                                              const float* __restrict__ w, const float* __restrict__ mean,
                                              const float* __restrict__ rstd, const float* __restrict__ gy, int ldg,
                                              const float* __restrict__ X, const float* __restrict__ Wb,
                                              const float* __restrict__ Bb, float* __restrict__ dgy,
                                              float* __restrict__ dx, float* __restrict__ T) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (row >= rows) return;
  const float mu = mean[row], rs = rstd[row];
  const float* xr = x + (size_t)row * ldx;
  const float* gr = gy + (size_t)row * ldg;
  float h[CPL], G[CPL], Xv[CPL], g[CPL];
  float sx = 0.f, sxh = 0.f, sg = 0.f, sgh = 0.f, sxg = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    const bool on = c < C;
    h[j] = on ? (xr[c] - mu) * rs : 0.f;
    g[j] = on ? gr[c] : 0.f;
    G[j] = on ? g[j] * w[c] : 0.f;
    Xv[j] = (on && X) ? X[(size_t)row * C + c] : 0.f;
    sx += Xv[j];
    sxh += Xv[j] * h[j];
    sg += G[j];
    sgh += G[j] * h[j];
    sxg += Xv[j] * G[j];
  }
  const float invC = 1.f / (float)C;
  const float mX = wave_sum(sx) * invC, mXh = wave_sum(sxh) * invC, mG = wave_sum(sg) * invC,
              mGh = wave_sum(sgh) * invC, SXG = wave_sum(sxg);
  const float v = SXG - (float)C * (mG * mX + mGh * mXh);
  float u[CPL];
  float su = 0.f, suh = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    const bool on = c < C;
    const float wb = (on && Wb) ? Wb[c] : 0.f;
    const float t = rs * (Xv[j] - mX - h[j] * mXh);
    if (on) {
      if (T) T[(size_t)row * C + c] = t;
      if (dgy) dgy[(size_t)row * C + c] = w[c] * t + wb * h[j] + ((Bb) ? Bb[c] : 0.f);
    }
    u[j] = on ? -rs * (G[j] * mXh + mGh * Xv[j]) + wb * g[j] : 0.f;
    su += u[j];
    suh += u[j] * h[j];
  }
  if (!dx) return;
  const float mu_ = wave_sum(su) * invC, muh = wave_sum(suh) * invC;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane + 64 * j;
    if (c < C) dx[(size_t)row * C + c] = rs * (u[j] - mu_ - h[j] * muh) - v * rs * rs * h[j] * invC;
  }
}

// weight / bias gradient partials: block k sums rows [k * chunk, (k + 1) * chunk) for every column.  The
// chunk is short (>= 16 rows, at most ~256 chunks): a C2 out_norm (678 x 128) at 128-row chunks was 6
// blocks walking 128 dependent rows each, 34 us.
static inline int wgrad_chunk(int rows) { return max(16, (rows + 255) / 256); }
__global__ __launch_bounds__(256) void k_wgrad_part(int rows, int C, int chunk, const float* __restrict__ x, int ldx,
                                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                                    const float* __restrict__ gy, int ldg, float* __restrict__ part) {
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
    float sw = 0.f, sb = 0.f;
#pragma unroll 4
    for (int r = r0; r < r1; ++r) {
      const float g = gy[(size_t)r * ldg + c];
      sw += g * (x[(size_t)r * ldx + c] - mean[r]) * rstd[r];
      sb += g;
    }
    part[((size_t)blockIdx.y * 2) * C + c] = sw;
    part[((size_t)blockIdx.y * 2 + 1) * C + c] = sb;
  }
}

__global__ __launch_bounds__(256) void k_wgrad_sum(int C, int chunks, const float* __restrict__ part,
                                                   float* __restrict__ gw, float* __restrict__ gb) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float sw = 0.f, sb = 0.f;
  for (int k = 0; k < chunks; ++k) {
    sw += part[((size_t)k * 2) * C + c];
    sb += part[((size_t)k * 2 + 1) * C + c];
  }
  if (gw) gw[c] = sw;
  if (gb) gb[c] = sb;
}

}  // namespace ln
}  // namespace tmd

using namespace tmd;

#define TMD_LN_CPL(C_, F)                                 \
  do {                                                    \
    if ((C_) <= 128) F(2);                                \
    else if ((C_) <= 256) F(4);                           \
    else if ((C_) <= 384) F(6);                           \
    else if ((C_) <= 512) F(8);                           \
    else F(16);                                           \
  } while (0)

extern "C" int tmdnet_layernorm_fwd_f32(int rows, int C, const void* x, int ldx, const void* w, const void* b,
                                        double eps, void* y, int ldy, void* mean, void* rstd, void* stream) {
  if (rows < 0 || C <= 0 || C > 1024 || ldx < C || ldy < C || !x || !w || !b || !y || !mean || !rstd)
    return kBadArgument;
  if (rows == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((rows + 3) / 4), t(256);
#define TMD_F(K) hipLaunchKernelGGL(ln::k_fwd<K>, g, t, 0, st, rows, C, (const float*)x, ldx, (const float*)w, \
                                    (const float*)b, (float)eps, (float*)y, ldy, (float*)mean, (float*)rstd)
  TMD_LN_CPL(C, TMD_F);
#undef TMD_F
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_layernorm_bwd_f32(int rows, int C, const void* x, int ldx, const void* w, const void* mean,
                                        const void* rstd, const void* grad_y, int ldg, void* grad_x, int accumulate,
                                        void* stream) {
  if (rows < 0 || C <= 0 || C > 1024 || ldx < C || ldg < C || !x || !w || !mean || !rstd || !grad_y || !grad_x)
    return kBadArgument;
  if (rows == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((rows + 3) / 4), t(256);
#define TMD_F(K)                                                                                                \
  hipLaunchKernelGGL(ln::k_bwd<K>, g, t, 0, st, rows, C, (const float*)x, ldx, (const float*)w, (const float*)mean, \
                     (const float*)rstd, (const float*)grad_y, ldg, (float*)grad_x, accumulate)
  TMD_LN_CPL(C, TMD_F);
#undef TMD_F
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" size_t tmdnet_layernorm_wgrad_workspace_bytes(int rows, int C) {
  if (rows <= 0 || C <= 0) return 0;
  const int ch = ln::wgrad_chunk(rows);
  return (size_t)((rows + ch - 1) / ch) * 2 * C * sizeof(float);
}

extern "C" int tmdnet_layernorm_wgrad_f32(int rows, int C, const void* x, int ldx, const void* mean, const void* rstd,
                                          const void* grad_y, int ldg, void* grad_w, void* grad_b, void* workspace,
                                          size_t workspace_bytes, void* stream) {
  if (rows < 0 || C <= 0 || ldx < C || ldg < C || !x || !mean || !rstd || !grad_y || (!grad_w && !grad_b))
    return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (rows == 0) {  // empty sums: zeros
    hipLaunchKernelGGL(ln::k_wgrad_sum, dim3((C + 255) / 256), dim3(256), 0, st, C, 0, (const float*)nullptr,
                       (float*)grad_w, (float*)grad_b);
    return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
  }
  if (!workspace || workspace_bytes < tmdnet_layernorm_wgrad_workspace_bytes(rows, C)) return kWorkspaceTooSmall;
  const int ch = ln::wgrad_chunk(rows), chunks = (rows + ch - 1) / ch;
  hipLaunchKernelGGL(ln::k_wgrad_part, dim3((C + 255) / 256, chunks), dim3(256), 0, st, rows, C, ch, (const float*)x,
                     ldx,
                     (const float*)mean, (const float*)rstd, (const float*)grad_y, ldg, (float*)workspace);
  hipLaunchKernelGGL(ln::k_wgrad_sum, dim3((C + 255) / 256), dim3(256), 0, st, C, chunks, (const float*)workspace,
                     (float*)grad_w, (float*)grad_b);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_layernorm_bwd2_f32(int rows, int C, const void* x, int ldx, const void* w, const void* mean,
                                         const void* rstd, const void* grad_y, int ldg, const void* t_gx,
                                         const void* t_gw, const void* t_gb, void* d_grad_y, void* d_x, void* t_row,
                                         void* stream) {
  if (rows < 0 || C <= 0 || C > 1024 || ldx < C || ldg < C || !x || !w || !mean || !rstd || !grad_y)
    return kBadArgument;
  if (rows == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((rows + 3) / 4), t(256);
#define TMD_F(K)                                                                                                  \
  hipLaunchKernelGGL(ln::k_bwd2<K>, g, t, 0, st, rows, C, (const float*)x, ldx, (const float*)w, (const float*)mean, \
                     (const float*)rstd, (const float*)grad_y, ldg, (const float*)t_gx, (const float*)t_gw,          \
                     (const float*)t_gb, (float*)d_grad_y, (float*)d_x, (float*)t_row)
  TMD_LN_CPL(C, TMD_F);
#undef TMD_F
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
