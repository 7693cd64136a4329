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
