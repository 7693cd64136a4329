// TensorNet node-level tensor algebra, fused per channel (reference models/tensornet.py:16-67,
// 200-234, 287-326, 335-410).  The reference evaluates each of these steps as 10-40 elementwise
// PyTorch kernels over [N][H][3][3] tensors; here each step is ONE pass with a thread per
// (atom, channel) holding its 3x3 tensor in registers.  Interior tensors use the compact
// component-major layout of tn_node.h ([9][N][H]); the layer input / output X keeps the
// reference's [N][H][3][3].
//
//   TMDNET_TN_PRE      X -> c = decomp(X / (|X|^2 + 1))                      (tensornet.py:391-392)
//   TMDNET_TN_POST_O3  (Y, M) -> decomp(Z) / (|Z|^2 + 1), Z = M Y + Y M      (tensornet.py:398-406)
//   TMDNET_TN_POST_SO3 (Y, M) -> same with Z = 2 Y M
//   TMDNET_TN_RESID    (X, D) -> X / (|X|^2 + 1) + D + D D                    (tensornet.py:391, 410)
//   TMDNET_TN_NORMS    X -> [|I|^2 | |A|^2 | |S|^2]  as [N][3H]              (tensornet.py:230-231)
//   TMDNET_TN_ENORM    c -> |full(c)|^2  as [N][H]                            (tensornet.py:317)
//   TMDNET_TN_EOUT     (c, f[N][H][3]) -> f_I I + f_A A + f_S S as [N][H][3][3] (tensornet.py:321-326)
// Backward passes are the exact VJPs (derived in the comments of each case).
#include "common.h"
#include "tmdnet.h"
#include "tn_node.h"

namespace tmd {
namespace node {

// CP / OP: the input / output "pointer" types -- const T* / T* for the first-order passes, DIn / DOut
// (value and tangent arrays) for the second order's dual-number evaluation below
template <typename T, typename CP = const T*, typename OP = T*> struct NodeArgs {
  int n, H;
  size_t nh;
  CP a; CP b; OP out;           // forward
  CP gout; OP ga; OP gb; CP gadd;  // backward
};

// (Dual / DIn / DOut: tn_node.h, shared with the TensorNet edge kernels' second order)
template <typename T, typename P> __device__ __forceinline__ void ldc(T (&o)[9], P p, size_t nh) {
#pragma unroll
  for (int k = 0; k < 9; ++k) o[k] = p[k * nh];
}
template <typename T, typename P> __device__ __forceinline__ void stc(P p, size_t nh, const T (&o)[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) p[k * nh] = o[k];
}
template <typename T, typename P> __device__ __forceinline__ void ld9(T (&o)[9], P p) {
#pragma unroll
  for (int k = 0; k < 9; ++k) o[k] = p[k];
}
template <typename T, typename P> __device__ __forceinline__ void st9(P p, const T (&o)[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) p[k] = o[k];
}

template <typename T, int OP, typename AR = NodeArgs<T>>
__global__ __launch_bounds__(256) void k_node_fwd(AR A) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A.nh) return;
  const int n = (int)(t / A.H), h = (int)(t % A.H);
  if constexpr (OP == TMDNET_TN_PRE) {
    T X[9], c[9];
    ld9(X, A.a + 9 * t);
    const T inv = T(1) / (sq9(X) + T(1));
#pragma unroll
    for (int k = 0; k < 9; ++k) X[k] *= inv;
    decomp(c, X);
    stc(A.out + t, A.nh, c);
  } else if constexpr (OP == TMDNET_TN_POST_O3 || OP == TMDNET_TN_POST_SO3) {
    T yc[9], mc[9], Y[9], M[9], Z[9], c[9];
    ldc(yc, A.a + t, A.nh);
    ldc(mc, A.b + t, A.nh);
    full(Y, yc);
    full(M, mc);
    if constexpr (OP == TMDNET_TN_POST_O3) {
      T P[9];
      mm(Z, M, Y);
      mm(P, Y, M);
#pragma unroll
      for (int k = 0; k < 9; ++k) Z[k] += P[k];
    } else {
      mm(Z, Y, M);
#pragma unroll
      for (int k = 0; k < 9; ++k) Z[k] *= T(2);
    }
    decomp(c, Z);
    const T inv = T(1) / (sq9(Z) + T(1));
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] *= inv;
    stc(A.out + t, A.nh, c);
  } else if constexpr (OP == TMDNET_TN_RESID) {
    // the reference's residual is the NORMALISED input: X is reassigned by X / (|X|^2 + 1) (:391)
    T X[9], dc[9], D[9], DD[9];
    ld9(X, A.a + 9 * t);
    ldc(dc, A.b + t, A.nh);
    const T inv = T(1) / (sq9(X) + T(1));
    full(D, dc);
    mm(DD, D, D);
#pragma unroll
    for (int k = 0; k < 9; ++k) X[k] = X[k] * inv + D[k] + DD[k];
    st9(A.out + 9 * t, X);
  } else if constexpr (OP == TMDNET_TN_NORMS) {
    T X[9], c[9];
    ld9(X, A.a + 9 * t);
    decomp(c, X);
    const T ss = c[4] + c[5];
    auto o = A.out + (size_t)n * 3 * A.H + h;
    o[0] = T(3) * c[0] * c[0];
    o[A.H] = T(2) * (c[1] * c[1] + c[2] * c[2] + c[3] * c[3]);
    o[2 * A.H] = c[4] * c[4] + c[5] * c[5] + ss * ss + T(2) * (c[6] * c[6] + c[7] * c[7] + c[8] * c[8]);
  } else if constexpr (OP == TMDNET_TN_ENORM) {
    T c[9], F[9];
    ldc(c, A.a + t, A.nh);
    full(F, c);
    A.out[t] = sq9(F);
  } else if constexpr (OP == TMDNET_TN_EOUT) {
    T c[9], F[9];
    ldc(c, A.a + t, A.nh);
    auto f = A.b + 3 * t;  // norm.reshape(N, H, 3)
    const T fI = f[0], fA = f[1], fS = f[2];
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] *= ctype_scale(k, fI, fA, fS);
    full(F, c);
    st9(A.out + 9 * t, F);
  }
}

template <typename T, int OP, typename AR = NodeArgs<T>>
__global__ __launch_bounds__(256) void k_node_bwd(AR A) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A.nh) return;
  const int n = (int)(t / A.H), h = (int)(t % A.H);
  if constexpr (OP == TMDNET_TN_PRE) {
    // out = decomp(X / s), s = |X|^2 + 1:  gX = G / s - 2 X <G, X> / s^2,  G = decomp^T(g)
    T X[9], gc[9], G[9];
    ld9(X, A.a + 9 * t);
    ldc(gc, A.gout + t, A.nh);
    decompT(G, gc);
    const T inv = T(1) / (sq9(X) + T(1));
    T d = T(0);
#pragma unroll
    for (int k = 0; k < 9; ++k) d += G[k] * X[k];
    const T w = T(2) * d * inv * inv;
    T gX[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) gX[k] = G[k] * inv - w * X[k];
    if (A.gadd) {
#pragma unroll
      for (int k = 0; k < 9; ++k) gX[k] += A.gadd[9 * t + k];
    }
    st9(A.ga + 9 * t, gX);
  } else if constexpr (OP == TMDNET_TN_POST_O3 || OP == TMDNET_TN_POST_SO3) {
    // out = decomp(Z) / s, s = |Z|^2 + 1:  gZ = decomp^T(g) / s - 2 Z <g, decomp(Z)> / s^2
    // O(3):  Z = M Y + Y M:  gM = gZ Y^T + Y^T gZ,  gY = M^T gZ + gZ M^T
    // SO(3): Z = 2 Y M:      gY = 2 gZ M^T,          gM = 2 Y^T gZ
    T yc[9], mc[9], Y[9], M[9], Z[9], c[9], g[9], gZ[9];
    ldc(yc, A.a + t, A.nh);
    ldc(mc, A.b + t, A.nh);
    ldc(g, A.gout + t, A.nh);
    full(Y, yc);
    full(M, mc);
    if constexpr (OP == TMDNET_TN_POST_O3) {
      T P[9];
      mm(Z, M, Y);
      mm(P, Y, M);
#pragma unroll
      for (int k = 0; k < 9; ++k) Z[k] += P[k];
    } else {
      mm(Z, Y, M);
#pragma unroll
      for (int k = 0; k < 9; ++k) Z[k] *= T(2);
    }
    decomp(c, Z);
    const T inv = T(1) / (sq9(Z) + T(1));
    T d = T(0);
#pragma unroll
    for (int k = 0; k < 9; ++k) d += g[k] * c[k];
    decompT(gZ, g);
    const T w = T(2) * d * inv * inv;
#pragma unroll
    for (int k = 0; k < 9; ++k) gZ[k] = gZ[k] * inv - w * Z[k];
    T gY[9], gM[9];
    if constexpr (OP == TMDNET_TN_POST_O3) {
      T P[9];
      mmNT(gM, gZ, Y);
      mmTN(P, Y, gZ);
#pragma unroll
      for (int k = 0; k < 9; ++k) gM[k] += P[k];
      mmTN(gY, M, gZ);
      mmNT(P, gZ, M);
#pragma unroll
      for (int k = 0; k < 9; ++k) gY[k] += P[k];
    } else {
      mmNT(gY, gZ, M);
      mmTN(gM, Y, gZ);
#pragma unroll
      for (int k = 0; k < 9; ++k) { gY[k] *= T(2); gM[k] *= T(2); }
    }
    T gyc[9], gmc[9];
    fullT(gyc, gY);
    fullT(gmc, gM);
    stc(A.ga + t, A.nh, gyc);
    stc(A.gb + t, A.nh, gmc);
  } else if constexpr (OP == TMDNET_TN_RESID) {
    // out = X / s + D + D D, s = |X|^2 + 1:  gX = g / s - 2 X <g, X> / s^2,  gD = g + g D^T + D^T g
    T X[9], dc[9], D[9], g[9], P[9], Q[9], gdc[9];
    ld9(X, A.a + 9 * t);
    ldc(dc, A.b + t, A.nh);
    ld9(g, A.gout + 9 * t);
    full(D, dc);
    mmNT(P, g, D);
    mmTN(Q, D, g);
#pragma unroll
    for (int k = 0; k < 9; ++k) P[k] += g[k] + Q[k];
    fullT(gdc, P);
    stc(A.gb + t, A.nh, gdc);
    const T inv = T(1) / (sq9(X) + T(1));
    T d = T(0);
#pragma unroll
    for (int k = 0; k < 9; ++k) d += g[k] * X[k];
    const T w = T(2) * d * inv * inv;
#pragma unroll
    for (int k = 0; k < 9; ++k) g[k] = g[k] * inv - w * X[k];
    if (A.gadd) {
#pragma unroll
      for (int k = 0; k < 9; ++k) g[k] += A.gadd[9 * t + k];
    }
    st9(A.ga + 9 * t, g);
  } else if constexpr (OP == TMDNET_TN_NORMS) {
    // |I|^2 = 3 i^2, |A|^2 = 2 sum a^2, |S|^2 = s00^2 + s11^2 + (s00+s11)^2 + 2 sum s_off^2
    T X[9], c[9], gc[9], gX[9];
    ld9(X, A.a + 9 * t);
    decomp(c, X);
    auto go = A.gout + (size_t)n * 3 * A.H + h;
    const T g0 = go[0], g1 = go[A.H], g2 = go[2 * A.H];
    const T ss = c[4] + c[5];
    gc[0] = T(6) * g0 * c[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) gc[k] = T(4) * g1 * c[k];
    gc[4] = T(2) * g2 * (c[4] + ss);
    gc[5] = T(2) * g2 * (c[5] + ss);
#pragma unroll
    for (int k = 6; k < 9; ++k) gc[k] = T(4) * g2 * c[k];
    decompT(gX, gc);
    if (A.gadd) {
#pragma unroll
      for (int k = 0; k < 9; ++k) gX[k] += A.gadd[9 * t + k];
    }
    st9(A.ga + 9 * t, gX);
  } else if constexpr (OP == TMDNET_TN_ENORM) {
    // out = |full(c)|^2:  gc = full^T(2 g F)
    T c[9], F[9], gc[9];
    ldc(c, A.a + t, A.nh);
    full(F, c);
    const T g2 = T(2) * A.gout[t];
#pragma unroll
    for (int k = 0; k < 9; ++k) F[k] *= g2;
    fullT(gc, F);
    if (A.gadd) {
#pragma unroll
      for (int k = 0; k < 9; ++k) gc[k] += A.gadd[k * A.nh + t];
    }
    stc(A.ga + t, A.nh, gc);
  } else if constexpr (OP == TMDNET_TN_EOUT) {
    // out = full(c * f_type):  gc_k = f_type(k) (full^T g)_k,  gf_t = sum_{k of type t} (full^T g)_k c_k
    T c[9], g[9], gc[9];
    ldc(c, A.a + t, A.nh);
    ld9(g, A.gout + 9 * t);
    fullT(gc, g);
    auto f = A.b + 3 * t;
    const T fI = f[0], fA = f[1], fS = f[2];
    T gI = gc[0] * c[0];
    T gA = gc[1] * c[1] + gc[2] * c[2] + gc[3] * c[3];
    T gS = gc[4] * c[4] + gc[5] * c[5] + gc[6] * c[6] + gc[7] * c[7] + gc[8] * c[8];
#pragma unroll
    for (int k = 0; k < 9; ++k) gc[k] *= ctype_scale(k, fI, fA, fS);
    stc(A.ga + t, A.nh, gc);
    auto gf = A.gb + 3 * t;
    gf[0] = gI;
    gf[1] = gA;
    gf[2] = gS;
  }
}

template <typename T, int OP>
static int launch_op(bool bwd, const NodeArgs<T>& A, hipStream_t st) {
  const int tb = 256;
  const unsigned grid = (unsigned)((A.nh + tb - 1) / tb);
  if (bwd) hipLaunchKernelGGL((k_node_bwd<T, OP>), dim3(grid), dim3(tb), 0, st, A);
  else hipLaunchKernelGGL((k_node_fwd<T, OP>), dim3(grid), dim3(tb), 0, st, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static int run(int op, bool bwd, const NodeArgs<T>& A, hipStream_t st) {
  if (A.nh == 0) return kOk;
  switch (op) {
    case TMDNET_TN_PRE: return launch_op<T, TMDNET_TN_PRE>(bwd, A, st);
    case TMDNET_TN_POST_O3: return launch_op<T, TMDNET_TN_POST_O3>(bwd, A, st);
    case TMDNET_TN_POST_SO3: return launch_op<T, TMDNET_TN_POST_SO3>(bwd, A, st);
    case TMDNET_TN_RESID: return launch_op<T, TMDNET_TN_RESID>(bwd, A, st);
    case TMDNET_TN_NORMS: return launch_op<T, TMDNET_TN_NORMS>(bwd, A, st);
    case TMDNET_TN_ENORM: return launch_op<T, TMDNET_TN_ENORM>(bwd, A, st);
    case TMDNET_TN_EOUT: return launch_op<T, TMDNET_TN_EOUT>(bwd, A, st);
    default: return kBadArgument;
  }
}

// second order (see Dual above): d_g = J_f (t_a, t_b) by the forward on duals (tangent output only) and
// (d_a, d_b) = H (t_a, t_b) by the first backward on duals (g with a zero tangent; tangent outputs only)
template <typename T, int OP>
static int launch_op2(const NodeArgs<T>& A, const T* ta, const T* tb, T* d_g, T* d_a, T* d_b, hipStream_t st) {
  using DA = NodeArgs<Dual<T>, DIn<T>, DOut<T>>;
  const int tb_ = 256;
  const unsigned grid = (unsigned)((A.nh + tb_ - 1) / tb_);
  const DIn<T> a{A.a, ta}, b{A.b, tb};
  if (d_g) {
    DA F{A.n, A.H, A.nh, a, b, DOut<T>{nullptr, d_g}, DIn<T>{nullptr, nullptr}, DOut<T>{nullptr, nullptr},
         DOut<T>{nullptr, nullptr}, DIn<T>{nullptr, nullptr}};
    hipLaunchKernelGGL((k_node_fwd<Dual<T>, OP, DA>), dim3(grid), dim3(tb_), 0, st, F);
  }
  if (d_a || d_b) {
    DA B{A.n, A.H, A.nh, a, b, DOut<T>{nullptr, nullptr}, DIn<T>{A.gout, nullptr}, DOut<T>{nullptr, d_a},
         DOut<T>{nullptr, d_b}, DIn<T>{nullptr, nullptr}};
    hipLaunchKernelGGL((k_node_bwd<Dual<T>, OP, DA>), dim3(grid), dim3(tb_), 0, st, B);
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

template <typename T>
static int run2(int op, const NodeArgs<T>& A, const T* ta, const T* tb, T* d_g, T* d_a, T* d_b, hipStream_t st) {
  if (A.nh == 0) return kOk;
  switch (op) {
    case TMDNET_TN_PRE: return launch_op2<T, TMDNET_TN_PRE>(A, ta, tb, d_g, d_a, d_b, st);
    case TMDNET_TN_POST_O3: return launch_op2<T, TMDNET_TN_POST_O3>(A, ta, tb, d_g, d_a, d_b, st);
    case TMDNET_TN_POST_SO3: return launch_op2<T, TMDNET_TN_POST_SO3>(A, ta, tb, d_g, d_a, d_b, st);
    case TMDNET_TN_RESID: return launch_op2<T, TMDNET_TN_RESID>(A, ta, tb, d_g, d_a, d_b, st);
    case TMDNET_TN_NORMS: return launch_op2<T, TMDNET_TN_NORMS>(A, ta, tb, d_g, d_a, d_b, st);
    case TMDNET_TN_ENORM: return launch_op2<T, TMDNET_TN_ENORM>(A, ta, tb, d_g, d_a, d_b, st);
    case TMDNET_TN_EOUT: return launch_op2<T, TMDNET_TN_EOUT>(A, ta, tb, d_g, d_a, d_b, st);
    default: return kBadArgument;
  }
}

}  // namespace node
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_tn_node_bwd2(int dtype, int op, int n_nodes, int hidden, const void* a, const void* b,
                                   const void* grad_out, const void* t_a, const void* t_b, void* d_grad_out,
                                   void* d_a, void* d_b, void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !a || !grad_out) return kBadArgument;
  const bool two = op == TMDNET_TN_POST_O3 || op == TMDNET_TN_POST_SO3 || op == TMDNET_TN_RESID || op == TMDNET_TN_EOUT;
  if (two && !b) return kBadArgument;
  if (!two && (t_b || d_b)) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) {
    node::NodeArgs<float> A{n_nodes, hidden, (size_t)n_nodes * hidden, (const float*)a, (const float*)b, nullptr,
                            (const float*)grad_out, nullptr, nullptr, nullptr};
    return node::run2<float>(op, A, (const float*)t_a, (const float*)t_b, (float*)d_grad_out, (float*)d_a,
                             (float*)d_b, st);
  } else if (dtype == TMDNET_F64) {
    node::NodeArgs<double> A{n_nodes, hidden, (size_t)n_nodes * hidden, (const double*)a, (const double*)b, nullptr,
                             (const double*)grad_out, nullptr, nullptr, nullptr};
    return node::run2<double>(op, A, (const double*)t_a, (const double*)t_b, (double*)d_grad_out, (double*)d_a,
                              (double*)d_b, st);
  }
  return kUnsupported;
}

extern "C" int tmdnet_tn_node_fwd(int dtype, int op, int n_nodes, int hidden, const void* a,
                                  const void* b, void* out, void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !a || !out) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) {
    node::NodeArgs<float> A{n_nodes, hidden, (size_t)n_nodes * hidden, (const float*)a,
                            (const float*)b, (float*)out, nullptr, nullptr, nullptr, nullptr};
    return node::run<float>(op, false, A, st);
  } else if (dtype == TMDNET_F64) {
    node::NodeArgs<double> A{n_nodes, hidden, (size_t)n_nodes * hidden, (const double*)a,
                             (const double*)b, (double*)out, nullptr, nullptr, nullptr, nullptr};
    return node::run<double>(op, false, A, st);
  }
  return kUnsupported;
}

extern "C" int tmdnet_tn_node_bwd(int dtype, int op, int n_nodes, int hidden, const void* a,
                                  const void* b, const void* grad_out, const void* grad_add,
                                  void* ga, void* gb, void* stream) {
  if (n_nodes < 0 || hidden <= 0 || !grad_out) return kBadArgument;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32) {
    node::NodeArgs<float> A{n_nodes, hidden, (size_t)n_nodes * hidden, (const float*)a,
                            (const float*)b, nullptr, (const float*)grad_out, (float*)ga,
                            (float*)gb, (const float*)grad_add};
    return node::run<float>(op, true, A, st);
  } else if (dtype == TMDNET_F64) {
    node::NodeArgs<double> A{n_nodes, hidden, (size_t)n_nodes * hidden, (const double*)a,
                             (const double*)b, nullptr, (const double*)grad_out, (double*)ga,
                             (double*)gb, (const double*)grad_add};
    return node::run<double>(op, true, A, st);
  }
  return kUnsupported;
}
