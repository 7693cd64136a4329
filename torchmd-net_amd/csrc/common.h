// Shared device helpers for the torchmd-net_amd HIP library (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TMD_WAVE 64

// Index-range checks of the CSR kernels, compiled only into the debug library (`make debug`:
// -DTMDNET_DEBUG_INDEX, lib/libtmdnet_hip_debug.so).  A failing check aborts the kernel (device
// assert), naming the file and line.  The product library compiles them out.
#ifdef TMDNET_DEBUG_INDEX
#include <assert.h>
#define TMD_DCHECK(c) assert(c)
#else
#define TMD_DCHECK(c) ((void)0)
#endif

namespace tmd {

// ---- status codes returned across the C ABI (never throw across it) ----
enum Status : int {
  kOk = 0,
  kBadArgument = 1,
  kUnsupported = 2,
  kLaunchFailed = 3,
  kWorkspaceTooSmall = 4,
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & (TMD_WAVE - 1); }

// XCD-contiguous block remap (bijective, cdna_hip_programming.md §5 "XCD swizzle"): hardware deals
// workgroups round-robin over the 8 XCDs; the remap gives each XCD one contiguous range of logical
// blocks, so data shared by neighbouring logical blocks stays in that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  if (nwg < 16) return b;
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Number of set bits of `mask` strictly below this lane (exclusive lane prefix of a ballot).
__device__ __forceinline__ int lane_prefix(unsigned long long mask) {
  unsigned lo = __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u);
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), lo);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Sum over aligned groups of `width` lanes (width a power of two <= 64).
template <typename T>
__device__ __forceinline__ T group_sum(T v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename T> __device__ __forceinline__ T sigmoid(T x) { return T(1) / (T(1) + exp(-x)); }
// fp32: hardware exp2 and reciprocal (v_exp_f32, v_rcp_f32; <= 1 ulp each) instead of the ~10-instruction
// IEEE division sequence -- the edge kernels evaluate 16 of these per lane per edge.  exp(-x) -> inf gives
// rcp(inf) = 0, the correct limit.
template <> __device__ __forceinline__ float sigmoid<float>(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

// silu and its derivative, sharing the sigmoid
template <typename T> struct Silu {
  T s, sig;
  __device__ __forceinline__ explicit Silu(T x) {
    sig = sigmoid<T>(x);
    s = x * sig;
  }
  __device__ __forceinline__ T d(T x) const { return sig * (T(1) + x * (T(1) - sig)); }
  // second derivative: s(1-s)(2 + x(1-2s))
  __device__ __forceinline__ T dd(T x) const { return sig * (T(1) - sig) * (T(2) + x * (T(1) - T(2) * sig)); }
};

// The reference's act_class_mapping (models/utils.py:579-584) as a wave-uniform runtime code of the
// ET message kernels (TMDNET_ET_ACT flags bits): value, first and second derivative.  Code 0 is SiLU,
// evaluated exactly as Silu above (the default path adds one scalar branch per evaluation).
enum ActCode : int { kActSilu = 0, kActSsp = 1, kActTanh = 2, kActSigmoid = 3 };

template <typename T> __device__ __forceinline__ T softplus_(T x) {  // F.softplus (beta 1, threshold 20)
  return x > T(20) ? x : log1p(exp(x));
}

template <typename T> struct ActF {
  T s, sg;  // value; the sigmoid (SiLU, shifted softplus, sigmoid) the derivatives reuse
  int c;
  __device__ __forceinline__ ActF(T x, int code) : c(code) {
    if (code == kActSilu) {
      sg = sigmoid<T>(x);
      s = x * sg;
    } else if (code == kActSsp) {  // ShiftedSoftplus: softplus(x) - log 2 (rounded to fp32 as the
      sg = sigmoid<T>(x);          // reference's shift, models/utils.py:354-359)
      s = softplus_<T>(x) - T(0.693147182464599609375);
    } else if (code == kActTanh) {
      s = tanh(x);
      sg = T(0);
    } else {
      sg = sigmoid<T>(x);
      s = sg;
    }
  }
  __device__ __forceinline__ T d(T x) const {
    if (c == kActSilu) return sg * (T(1) + x * (T(1) - sg));
    if (c == kActSsp) return sg;
    if (c == kActTanh) return T(1) - s * s;
    return sg * (T(1) - sg);
  }
  __device__ __forceinline__ T dd(T x) const {
    if (c == kActSilu) return sg * (T(1) - sg) * (T(2) + x * (T(1) - T(2) * sg));
    if (c == kActSsp) return sg * (T(1) - sg);
    if (c == kActTanh) return T(-2) * s * (T(1) - s * s);
    return sg * (T(1) - sg) * (T(1) - T(2) * sg);
  }
};

}  // namespace tmd
