// TensorNet per-channel 3x3 algebra on the compact basis (shared by tn_message.hip / tn_node.hip).
//
// A channel's tensor X = I + A + S (reference decompose_tensor, models/tensornet.py:47-52) is held
// as 9 coefficients c = [i, a01, a02, a12, s00, s11, s01, s02, s12]:
//   I = i Id,  A = [[0,a01,a02],[-a01,0,a12],[-a02,-a12,0]],
//   S = [[s00,s01,s02],[s01,s11,s12],[s02,s12,-s00-s11]].
// full(c) is the row-major 3x3 matrix, decomp(F) its reference decomposition (decomp(full(c)) = c);
// fullT / decompT are their transposes (gradient maps).
#pragma once

namespace tmd {
namespace node {

// component type of compact row k: 0 = I (k = 0), 1 = A (k = 1..3), 2 = S (k = 4..8)
template <typename T>
__device__ __forceinline__ T ctype_scale(int k, T fI, T fA, T fS) {
  return k == 0 ? fI : (k < 4 ? fA : fS);
}

template <typename T> __device__ __forceinline__ void full(T (&F)[9], const T (&c)[9]) {
  F[0] = c[0] + c[4];  F[1] = c[1] + c[6];  F[2] = c[2] + c[7];
  F[3] = c[6] - c[1];  F[4] = c[0] + c[5];  F[5] = c[3] + c[8];
  F[6] = c[7] - c[2];  F[7] = c[8] - c[3];  F[8] = c[0] - c[4] - c[5];
}

template <typename T> __device__ __forceinline__ void decomp(T (&c)[9], const T (&F)[9]) {
  const T i = (F[0] + F[4] + F[8]) / T(3);
  c[0] = i;
  c[1] = T(0.5) * (F[1] - F[3]);
  c[2] = T(0.5) * (F[2] - F[6]);
  c[3] = T(0.5) * (F[5] - F[7]);
  c[4] = F[0] - i;
  c[5] = F[4] - i;
  c[6] = T(0.5) * (F[1] + F[3]);
  c[7] = T(0.5) * (F[2] + F[6]);
  c[8] = T(0.5) * (F[5] + F[7]);
}

// gc = full^T gF
template <typename T> __device__ __forceinline__ void fullT(T (&gc)[9], const T (&g)[9]) {
  gc[0] = g[0] + g[4] + g[8];
  gc[1] = g[1] - g[3];
  gc[2] = g[2] - g[6];
  gc[3] = g[5] - g[7];
  gc[4] = g[0] - g[8];
  gc[5] = g[4] - g[8];
  gc[6] = g[1] + g[3];
  gc[7] = g[2] + g[6];
  gc[8] = g[5] + g[7];
}

// gF = decomp^T gc
template <typename T> __device__ __forceinline__ void decompT(T (&g)[9], const T (&gc)[9]) {
  const T t = (gc[0] - gc[4] - gc[5]) / T(3);
  g[0] = t + gc[4];
  g[4] = t + gc[5];
  g[8] = t;
  g[1] = T(0.5) * (gc[6] + gc[1]);
  g[3] = T(0.5) * (gc[6] - gc[1]);
  g[2] = T(0.5) * (gc[7] + gc[2]);
  g[6] = T(0.5) * (gc[7] - gc[2]);
  g[5] = T(0.5) * (gc[8] + gc[3]);
  g[7] = T(0.5) * (gc[8] - gc[3]);
}

// C = A B (row-major 3x3)
template <typename T> __device__ __forceinline__ void mm(T (&C)[9], const T (&A)[9], const T (&B)[9]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
// C = A^T B
template <typename T> __device__ __forceinline__ void mmTN(T (&C)[9], const T (&A)[9], const T (&B)[9]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[r] * B[c] + A[3 + r] * B[3 + c] + A[6 + r] * B[6 + c];
}
// C = A B^T
template <typename T> __device__ __forceinline__ void mmNT(T (&C)[9], const T (&A)[9], const T (&B)[9]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[3 * r] * B[3 * c] + A[3 * r + 1] * B[3 * c + 1] + A[3 * r + 2] * B[3 * c + 2];
}

template <typename T> __device__ __forceinline__ T sq9(const T (&a)[9]) {
  T s = T(0);
#pragma unroll
  for (int i = 0; i < 9; ++i) s += a[i] * a[i];
  return s;
}

// ---- second order by forward-over-reverse on dual numbers (value, tangent).  The first backward maps
// (a, b, g) to (ga, gb) = J_f(a, b)^T g; its VJP for cotangents (t_a, t_b) of (ga, gb) is
//   d_g      = J_f (t_a, t_b)                         -- the forward pass with tangents (t_a, t_b)
//   (d_a, d_b) = H_<g, f> (t_a, t_b)                   -- the first backward with tangents (t_a, t_b), g fixed
// (the Hessian of <g, f(a, b)> is symmetric).  Every pass above only adds, subtracts, multiplies and
// divides, so the SAME code evaluated on Dual<T> gives both (the derivative of a quotient included).
template <typename T> struct Dual {
  T v, d;
  __host__ __device__ __forceinline__ Dual() : v(0), d(0) {}
  __host__ __device__ __forceinline__ Dual(double x) : v(T(x)), d(0) {}  // constants
  __host__ __device__ __forceinline__ Dual(T v_, T d_) : v(v_), d(d_) {}
};
template <typename T> __device__ __forceinline__ Dual<T> operator+(Dual<T> x, Dual<T> y) { return {x.v + y.v, x.d + y.d}; }
template <typename T> __device__ __forceinline__ Dual<T> operator-(Dual<T> x, Dual<T> y) { return {x.v - y.v, x.d - y.d}; }
template <typename T> __device__ __forceinline__ Dual<T> operator-(Dual<T> x) { return {-x.v, -x.d}; }
template <typename T> __device__ __forceinline__ Dual<T> operator*(Dual<T> x, Dual<T> y) {
  return {x.v * y.v, x.d * y.v + x.v * y.d};
}
template <typename T> __device__ __forceinline__ Dual<T> operator/(Dual<T> x, Dual<T> y) {
  const T q = x.v / y.v;
  return {q, (x.d - q * y.d) / y.v};
}
template <typename T> __device__ __forceinline__ Dual<T>& operator+=(Dual<T>& x, Dual<T> y) { return x = x + y; }
template <typename T> __device__ __forceinline__ Dual<T>& operator-=(Dual<T>& x, Dual<T> y) { return x = x - y; }
template <typename T> __device__ __forceinline__ Dual<T>& operator*=(Dual<T>& x, Dual<T> y) { return x = x * y; }
// input: value and tangent arrays (tangent NULL: 0)
template <typename T> struct DIn {
  const T* v; const T* d;
  __device__ __forceinline__ DIn operator+(size_t o) const { return {v + o, d ? d + o : nullptr}; }
  __device__ __forceinline__ Dual<T> operator[](size_t i) const { return {v[i], d ? d[i] : T(0)}; }
  __device__ __forceinline__ explicit operator bool() const { return v != nullptr; }
};
// output: value and tangent arrays (either NULL: not stored)
template <typename T> struct DRef {
  T* v; T* d;
  __device__ __forceinline__ void operator=(Dual<T> x) const {
    if (v) *v = x.v;
    if (d) *d = x.d;
  }
};
template <typename T> struct DOut {
  T* v; T* d;
  __device__ __forceinline__ DOut operator+(size_t o) const { return {v ? v + o : nullptr, d ? d + o : nullptr}; }
  __device__ __forceinline__ DRef<T> operator[](size_t i) const { return {v ? v + i : nullptr, d ? d + i : nullptr}; }
  __device__ __forceinline__ explicit operator bool() const { return v != nullptr || d != nullptr; }
};

// wave sums of both parts (the edge kernels' per-edge channel sums)
template <typename T> __device__ __forceinline__ Dual<T> wave_sum(Dual<T> x) {
  return {tmd::wave_sum(x.v), tmd::wave_sum(x.d)};
}

}  // namespace node
}  // namespace tmd
