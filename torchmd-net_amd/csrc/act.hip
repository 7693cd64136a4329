// Fused SiLU (with an optional per-row scale) and its backward, for the scalar MLPs around the
// hot path: TensorNet's edge MLP `act(linear(.)) * C` (reference models/tensornet.py:385-389), its
// embedding / output MLPs (:322-323, :233) and the Scalar head (output_modules.py:70-79).
// Autograd's own SiLU backward under create_graph=True (the force pass) is a chain of seven
// elementwise kernels (sigmoid, fill, add, mul, add_, mul, mul); here it is one pass.
//   forward:  out[r][c] = silu(x[r][c]) * (scale ? scale[r] : 1)
//   backward: gx[r][c] = g[r][c] * scale[r] * silu'(x[r][c]);
//             gscale[r] = sum_c g[r][c] * silu(x[r][c])   (one wave per row, no atomics)
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace act {

template <typename T> struct ActArgs {
  int rows, cols, ldx, ldg;
  const T* x; const T* scale; T* out;
  const T* g; T* gx; T* gscale;
};

template <typename T>
__global__ __launch_bounds__(256) void k_silu_fwd(ActArgs<T> A) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)A.rows * A.cols) return;
  const int r = (int)(t / A.cols), c = (int)(t % A.cols);
  const T v = A.x[(size_t)r * A.ldx + c];
  Silu<T> s(v);
  A.out[t] = A.scale ? s.s * A.scale[r] : s.s;
}

// one wave per row: gx for every column, the row's gscale as a wave sum
template <typename T>
__global__ __launch_bounds__(256) void k_silu_bwd(ActArgs<T> A) {
  const int r = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (r >= A.rows) return;
  const T sc = A.scale ? A.scale[r] : T(1);
  T acc = T(0);
  for (int c = lane_id(); c < A.cols; c += TMD_WAVE) {
    const T v = A.x[(size_t)r * A.ldx + c];
    const T g = A.g[(size_t)r * A.ldg + c];
    Silu<T> s(v);
    A.gx[(size_t)r * A.cols + c] = g * sc * s.d(v);
    acc += g * s.s;
  }
  if (A.gscale) {
    acc = wave_sum(acc);
    if (lane_id() == 0) A.gscale[r] = acc;
  }
}

// ---- second order of the Linear + SiLU stacks (kernels._MLPActBwd: TensorNet's edge / embedding / output MLPs
// under force-matching training).  The first backward maps gy to g_i = a_i * silu'(p_i) layer by layer (a_i the
// upstream gradient of layer i's activation, a_{L-1} = gy * s); its reverse-mode VJP needs, per layer, the
// adjoint ghat of g_i turned into the adjoint of a_i and the extra adjoint of p_i:
//   up:   ahat = ghat * silu'(p),  dp = ghat * a * silu''(p)
//         last layer (a = gy * s, and the row sums gs = sum_c gy * silu(p) with adjoint sbar):
//         dp += sbar * gy * silu'(p),  dgy = ahat * s + sbar * silu(p),  ds = sum_c ahat * gy
//   down: c = dp + dh * silu'(p)   (the adjoint of p_{i-1} once layer i's input adjoint dh is known)
// silu = p sig, silu' = sig (1 + p (1 - sig)), silu'' = sig (1 - sig) (2 + p (1 - 2 sig)).
template <typename T> struct Mlp2Args {
  int rows, cols, ldp, lda;
  const T *p, *ghat, *a, *gy, *scale, *sbar;
  T *ahat, *dp, *dgy, *dscale;
  const T* dh;
  T* c;
};

template <typename T> __device__ __forceinline__ T sigm(T x) { return T(1) / (T(1) + exp(-x)); }

template <typename T>
__global__ __launch_bounds__(256) void k_mlp2_up(Mlp2Args<T> A) {
  const int r = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
  if (r >= A.rows) return;
  const T sc = A.scale ? A.scale[r] : T(1);
  const T sb = A.sbar ? A.sbar[r] : T(0);
  T acc = T(0);
  for (int c = lane_id(); c < A.cols; c += TMD_WAVE) {
    const size_t o = (size_t)r * A.cols + c;
    const T x = A.p[(size_t)r * A.ldp + c];
    const T sg = sigm(x);
    const T d1 = sg * (T(1) + x * (T(1) - sg));
    const T d2 = sg * (T(1) - sg) * (T(2) + x * (T(1) - T(2) * sg));
    const T gh = A.ghat[o];
    const T ah = gh * d1;
    A.ahat[o] = ah;
    if (A.gy) {
      const T g = A.gy[o];
      A.dp[o] = gh * g * sc * d2 + sb * g * d1;
      if (A.dgy) A.dgy[o] = ah * sc + sb * x * sg;
      acc += ah * g;
    } else {
      A.dp[o] = gh * A.a[(size_t)r * A.lda + c] * d2;
    }
  }
  if (A.dscale) {
    acc = wave_sum(acc);
    if (lane_id() == 0) A.dscale[r] = acc;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_mlp2_down(Mlp2Args<T> A) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)A.rows * A.cols) return;
  const int r = (int)(t / A.cols), c = (int)(t % A.cols);
  const T x = A.p[(size_t)r * A.ldp + c];
  const T sg = sigm(x);
  A.c[t] = A.dp[t] + A.dh[t] * sg * (T(1) + x * (T(1) - sg));
}

}  // namespace act
}  // namespace tmd

using namespace tmd;

template <typename T>
static int silu_fwd(int rows, int cols, const void* x, int ldx, const void* scale, void* out,
                    hipStream_t st) {
  act::ActArgs<T> A{rows, cols, ldx, 0, (const T*)x, (const T*)scale, (T*)out, nullptr, nullptr, nullptr};
  const size_t n = (size_t)rows * cols;
  if (n == 0) return kOk;
  hipLaunchKernelGGL(act::k_silu_fwd<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static int silu_bwd(int rows, int cols, const void* x, int ldx, const void* scale, const void* g,
                    int ldg, void* gx, void* gscale, hipStream_t st) {
  act::ActArgs<T> A{rows, cols, ldx, ldg, (const T*)x, (const T*)scale, nullptr, (const T*)g, (T*)gx,
                    (T*)gscale};
  if (rows == 0 || cols == 0) return kOk;
  hipLaunchKernelGGL(act::k_silu_bwd<T>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_silu_fwd(int dtype, int rows, int cols, const void* x, int ld_x,
                               const void* row_scale, void* out, void* stream) {
  if (rows < 0 || cols < 0 || ld_x < cols || !x || !out) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) return silu_fwd<float>(rows, cols, x, ld_x, row_scale, out, st);
  if (dtype == TMDNET_F64) return silu_fwd<double>(rows, cols, x, ld_x, row_scale, out, st);
  return kUnsupported;
}

extern "C" int tmdnet_silu_bwd(int dtype, int rows, int cols, const void* x, int ld_x,
                               const void* row_scale, const void* grad_out, int ld_g, void* grad_x,
                               void* grad_scale, void* stream) {
  if (rows < 0 || cols < 0 || ld_x < cols || ld_g < cols || !x || !grad_out || !grad_x)
    return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return silu_bwd<float>(rows, cols, x, ld_x, row_scale, grad_out, ld_g, grad_x, grad_scale, st);
  if (dtype == TMDNET_F64)
    return silu_bwd<double>(rows, cols, x, ld_x, row_scale, grad_out, ld_g, grad_x, grad_scale, st);
  return kUnsupported;
}

template <typename T>
static int mlp2_up(int rows, int cols, const void* pre, int ld_pre, const void* ghat, const void* a, int ld_a,
                   const void* gy, const void* scale, const void* sbar, void* ahat, void* dpre, void* dgy, void* dscale,
                   hipStream_t st) {
  act::Mlp2Args<T> A{rows, cols, ld_pre, ld_a, (const T*)pre, (const T*)ghat, (const T*)a, (const T*)gy,
                     (const T*)scale, (const T*)sbar, (T*)ahat, (T*)dpre, (T*)dgy, (T*)dscale, nullptr, nullptr};
  if (rows == 0 || cols == 0) return kOk;
  hipLaunchKernelGGL(act::k_mlp2_up<T>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static int mlp2_down(int rows, int cols, const void* pre, int ld_pre, const void* dh, const void* dp, void* c,
                     hipStream_t st) {
  act::Mlp2Args<T> A{rows, cols, ld_pre, 0, (const T*)pre, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                     nullptr, nullptr, nullptr, (const T*)dh, (T*)c};
  A.dp = (T*)dp;
  const size_t n = (size_t)rows * cols;
  if (n == 0) return kOk;
  hipLaunchKernelGGL(act::k_mlp2_down<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_mlp2_up(int dtype, int rows, int cols, const void* pre, int ld_pre, const void* ghat,
                              const void* a, int ld_a, const void* gy, const void* scale, const void* sbar, void* ahat,
                              void* dpre, void* dgy, void* dscale, void* stream) {
  if (rows < 0 || cols < 0 || ld_pre < cols || !pre || !ghat || !ahat || !dpre || (!gy && (!a || ld_a < cols)))
    return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return mlp2_up<float>(rows, cols, pre, ld_pre, ghat, a, ld_a, gy, scale, sbar, ahat, dpre, dgy, dscale, st);
  if (dtype == TMDNET_F64)
    return mlp2_up<double>(rows, cols, pre, ld_pre, ghat, a, ld_a, gy, scale, sbar, ahat, dpre, dgy, dscale, st);
  return kUnsupported;
}

extern "C" int tmdnet_mlp2_down(int dtype, int rows, int cols, const void* pre, int ld_pre, const void* dh,
                                const void* dp, void* c, void* stream) {
  if (rows < 0 || cols < 0 || ld_pre < cols || !pre || !dh || !dp || !c) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) return mlp2_down<float>(rows, cols, pre, ld_pre, dh, dp, c, st);
  if (dtype == TMDNET_F64) return mlp2_down<double>(rows, cols, pre, ld_pre, dh, dp, c, st);
  return kUnsupported;
}
