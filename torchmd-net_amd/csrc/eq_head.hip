// EquivariantScalar output head, fused: the two GatedEquivariantBlocks of reference
// models/output_modules.py:80-115 (blocks: models/utils.py:456-522) for a tile of atoms per
// workgroup, plus -- in the same pass -- the per-atom Jacobian of the atom's output y_n with respect
// to its inputs (x_n, vec_n).  The head is purely per-atom and ends in ONE scalar per atom, so the
// backward of the energy (forces) is y's cotangent times that Jacobian: the ~60 small GEMM /
// elementwise launches of the head's forward and backward become one launch here and one scale
// kernel in the backward.
//
// Block(Hi -> O, intermediate I = Hi), per atom (a = 0..2 the Cartesian axis):
//   vb[a] = W1 vec[a]           (Hi x Hi)      v2[a] = W2 vec[a]      (O x Hi)
//   vec1  = |vb| over a          (0 gradient where |vb| = 0, as torch.norm's backward)
//   u = U1 [x | vec1] + b1       (Hi x 2Hi)    s = SiLU(u)
//   o = U2 s + b2                (2O x Hi)     xo = o[:O], vo = o[O:]
//   x' = scalar_act ? SiLU(xo) : xo,           vec'[a] = vo * v2[a]
// EquivariantScalar = Block(H -> H/2, scalar_act) then Block(H/2 -> 1); y = x'' (+ 0 * sum vec'').
//
// Mapping: 256 threads, NT atoms per workgroup, every intermediate in LDS.  Row products
// (out[j] = sum_k W[j][k] in[k]) give one output row per thread with the input broadcast from LDS;
// transposed products of the backward (out[k] = sum_i W[i][k] g[i]) give one column per thread, so
// consecutive threads read consecutive weights.  Weights (~0.4 MB at H = 128) stay L2-resident
// across workgroups.
#include <cstdlib>

#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace head {

template <typename T>
struct Weights {
  const T *w1, *w2, *u1w, *u1b, *u2w, *u2b;  // block 1 (H -> H/2)
  const T *v1, *v2, *p1w, *p1b, *p2w, *p2b;  // block 2 (H/2 -> 1)
};

// Per-atom factors of the weight gradients (weights mode; NULL = not written).  Each weight gradient
// is then one GEMM over atoms, e.g. dU1|db1 = gu^T [x | vec1 | 1].
template <typename T>
struct Saves {
  T* a1;     // [N][3][H+O]   [g_vb | g_v2]         -> [dW1; dW2] = a1^T vec
  T* gu;     // [N][H]                              -> [dU1 | db1] = gu^T hext
  T* hext;   // [N][2H+1]     [x | vec1 | 1]
  T* go;     // [N][2O]                             -> [dU2 | db2] = go^T sext
  T* sext;   // [N][H+1]      [s | 1]
  T* a2;     // [N][3][Q+1]   [g_vb2 | 0]           -> [dV1; dV2] = a2^T v1
  T* v1;     // [N][3][O]
  T* gu2;    // [N][Q]                              -> [dP1 | db1'] = gu2^T h2ext
  T* h2ext;  // [N][2Q+1]     [x1 | vec1' | 1]
  T* go2;    // [N][2]        [g_y | 0]             -> [dP2 | db2'] = go2^T s2ext
  T* s2ext;  // [N][Q+1]      [s2 | 1]
};

template <typename T>
__device__ __forceinline__ T sig(T x) { return T(1) / (T(1) + exp(-x)); }
template <>
__device__ __forceinline__ float sig<float>(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// out[t][r][j] = bias[j] + sum_k W[j][k] in[t][r][k] for j < J (rows of A) then rows of B (J2 rows,
// written to out2), r < R vectors per atom; atom stride P, vector stride ld.  Each group of KS
// adjacent lanes owns JT rows and splits K between its lanes (interleaved 4-wide chunks, then an
// xor-shuffle sum): the narrow products (64-128 rows) still occupy the whole workgroup and each
// lane's dependent chain is K/KS long.  VEC: K, ldi, P multiples of 4 -> one 16-byte weight load
// per row and one broadcast ds_read_b128 per (atom, vector) feed 4*JT FMAs.
template <typename T, int NT, int R, int JT, bool VEC, int KS = 1>
__device__ __forceinline__ void rows2(const T* __restrict__ A, const T* __restrict__ ab, int J,
                                      const T* __restrict__ B, const T* __restrict__ bb, int J2, int K,
                                      const T* in, int ldi, T* out, int ldo, T* out2, int ldo2, int P) {
  using V4 = T __attribute__((ext_vector_type(4)));
  const int JJ = J + J2;
  const int ks = threadIdx.x % KS;
  for (int j0 = (threadIdx.x / KS) * JT; j0 < JJ; j0 += (blockDim.x / KS) * JT) {
    const T* w[JT];
    T acc[JT][NT][R];
#pragma unroll
    for (int q = 0; q < JT; ++q) {
      const int j = j0 + q;
      const bool ok = j < JJ, first = j < J;
      const int jj = first ? j : j - J;
      w[q] = !ok ? A : first ? A + (size_t)jj * K : B + (size_t)jj * K;  // dead rows read row 0
      const T* bp = first ? ab : bb;
      const T b0 = (ok && bp && ks == 0) ? bp[jj] : T(0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[q][t][r] = b0;
    }
    if (VEC) {
#pragma unroll 4
      for (int k = 4 * ks; k < K; k += 4 * KS) {
        V4 wv[JT];
#pragma unroll
        for (int q = 0; q < JT; ++q) wv[q] = *reinterpret_cast<const V4*>(w[q] + k);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const V4 iv = *reinterpret_cast<const V4*>(in + t * P + r * ldi + k);
#pragma unroll
            for (int q = 0; q < JT; ++q)
              acc[q][t][r] += wv[q].x * iv.x + wv[q].y * iv.y + wv[q].z * iv.z + wv[q].w * iv.w;
          }
      }
    } else {
#pragma unroll 8
      for (int k = ks; k < K; k += KS) {
        T wv[JT];
#pragma unroll
        for (int q = 0; q < JT; ++q) wv[q] = w[q][k];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T iv = in[t * P + r * ldi + k];
#pragma unroll
            for (int q = 0; q < JT; ++q) acc[q][t][r] += wv[q] * iv;
          }
      }
    }
    if constexpr (KS > 1) {
#pragma unroll
      for (int q = 0; q < JT; ++q)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int o = 1; o < KS; o <<= 1) acc[q][t][r] += __shfl_xor(acc[q][t][r], o);
      if (ks) continue;
    }
#pragma unroll
    for (int q = 0; q < JT; ++q) {
      const int j = j0 + q;
      if (j >= JJ) continue;
      const bool first = j < J;
      T* o = first ? out + j : out2 + (j - J);
      const int ld = first ? ldo : ldo2;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) o[t * P + r * ld] = acc[q][t][r];
    }
  }
}

// out[t][r][k] = sum_i A[i][k] g[t][r][i] (+ sum_i B[i][k] g2[t][r][i]) for k < K (K even); A, B row
// strides lda, ldb (even).  Each thread owns 2 adjacent columns (one 8-byte weight load per i);
// VEC: I, ldg, P multiples of 4 -> broadcast ds_read_b128 of g.  Destination: LDS (atom stride P) or
// global (atom stride gstride, atoms t < nt).
template <typename T, int NT, int R, bool VEC>
__device__ __forceinline__ void cols_part(T (&acc)[2][NT][R], const T* __restrict__ A, int lda, int I,
                                          const T* g, int ldg, int k0, int P) {
  using V2 = T __attribute__((ext_vector_type(2)));
  using V4 = T __attribute__((ext_vector_type(4)));
  if (VEC && (I & 3) == 0) {
#pragma unroll 2
    for (int i = 0; i < I; i += 4) {
      V2 wv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) wv[q] = *reinterpret_cast<const V2*>(A + (size_t)(i + q) * lda + k0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const V4 gv = *reinterpret_cast<const V4*>(g + t * P + r * ldg + i);
          acc[0][t][r] += wv[0].x * gv.x + wv[1].x * gv.y + wv[2].x * gv.z + wv[3].x * gv.w;
          acc[1][t][r] += wv[0].y * gv.x + wv[1].y * gv.y + wv[2].y * gv.z + wv[3].y * gv.w;
        }
    }
  } else {
#pragma unroll 8
    for (int i = 0; i < I; ++i) {
      const V2 wv = *reinterpret_cast<const V2*>(A + (size_t)i * lda + k0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const T gv = g[t * P + r * ldg + i];
          acc[0][t][r] += wv.x * gv;
          acc[1][t][r] += wv.y * gv;
        }
    }
  }
}

template <typename T, int NT, int R, bool VEC>
__device__ __forceinline__ void cols2(const T* __restrict__ A, int lda, int I, const T* g, int ldg,
                                      const T* __restrict__ B, int ldb, int I2, const T* g2, int ldg2,
                                      int K, T* out, int ldo, int P, int nt, size_t gstride, bool global) {
  for (int k0 = threadIdx.x * 2; k0 < K; k0 += blockDim.x * 2) {
    T acc[2][NT][R];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[q][t][r] = T(0);
    cols_part<T, NT, R, VEC>(acc, A, lda, I, g, ldg, k0, P);
    if (I2 > 0) cols_part<T, NT, R, VEC>(acc, B, ldb, I2, g2, ldg2, k0, P);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (global && t >= nt) continue;
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (global)
            out[t * gstride + r * ldo + k0 + q] = acc[q][t][r];
          else
            out[t * P + r * ldo + k0 + q] = acc[q][t][r];
        }
    }
  }
}

// cols2 with the I rows split over thread slices: at K = 64-128 output columns cols2 keeps only K/2
// threads of the workgroup busy, each walking all I (+ I2) weight rows as a dependent chain of L2
// round trips.  Here IS = blockDim / (K/2) slices each sum their share of the rows, the partial
// sums meet in LDS (`red`: IS x NT x R x K values) and are added in slice order (deterministic).
// Every thread of the workgroup must call it (one internal barrier).
template <typename T, int NT, int R, bool VEC>
__device__ __forceinline__ void cols_range(T (&acc)[2][NT][R], const T* __restrict__ A, int lda, int i0, int i1,
                                           const T* g, int ldg, int k0, int P) {
  using V2 = T __attribute__((ext_vector_type(2)));
  using V4 = T __attribute__((ext_vector_type(4)));
  if (VEC) {  // i0, i1 multiples of 4
#pragma unroll 4
    for (int i = i0; i < i1; i += 4) {
      V2 wv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) wv[q] = *reinterpret_cast<const V2*>(A + (size_t)(i + q) * lda + k0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const V4 gv = *reinterpret_cast<const V4*>(g + t * P + r * ldg + i);
          acc[0][t][r] += wv[0].x * gv.x + wv[1].x * gv.y + wv[2].x * gv.z + wv[3].x * gv.w;
          acc[1][t][r] += wv[0].y * gv.x + wv[1].y * gv.y + wv[2].y * gv.z + wv[3].y * gv.w;
        }
    }
  } else {
#pragma unroll 8
    for (int i = i0; i < i1; ++i) {
      const V2 wv = *reinterpret_cast<const V2*>(A + (size_t)i * lda + k0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const T gv = g[t * P + r * ldg + i];
          acc[0][t][r] += wv.x * gv;
          acc[1][t][r] += wv.y * gv;
        }
    }
  }
}

template <typename T, int NT, int R, bool VEC>
__device__ __forceinline__ void cols2s(const T* __restrict__ A, int lda, int I, const T* g, int ldg,
                                       const T* __restrict__ B, int ldb, int I2, const T* g2, int ldg2,
                                       int K, T* out, int ldo, int P, int nt, size_t gstride, bool global,
                                       T* red) {
  const int CP = K / 2;
  if (CP > (int)blockDim.x) {  // wider than the workgroup: the unsplit form
    cols2<T, NT, R, VEC>(A, lda, I, g, ldg, B, ldb, I2, g2, ldg2, K, out, ldo, P, nt, gstride, global);
    return;
  }
  int IS = 1;
  while (2 * IS * CP <= (int)blockDim.x && 2 * IS <= 8) IS *= 2;
  const int s = threadIdx.x / CP, k0 = (threadIdx.x % CP) * 2;
  if (s < IS) {
    T acc[2][NT][R];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[q][t][r] = T(0);
    const int gran = VEC ? 4 : 1;
    const int pa = ((I + IS * gran - 1) / (IS * gran)) * gran;
    cols_range<T, NT, R, VEC>(acc, A, lda, min(I, s * pa), min(I, (s + 1) * pa), g, ldg, k0, P);
    if (I2 > 0) {
      const int pb = ((I2 + IS * gran - 1) / (IS * gran)) * gran;
      cols_range<T, NT, R, VEC>(acc, B, ldb, min(I2, s * pb), min(I2, (s + 1) * pb), g2, ldg2, k0, P);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 2; ++q) red[((s * NT + t) * R + r) * K + k0 + q] = acc[q][t][r];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NT * R * K; e += blockDim.x) {
    const int t = e / (R * K), r = (e / K) % R, k = e % K;
    T v = T(0);
    for (int s2 = 0; s2 < IS; ++s2) v += red[((s2 * NT + t) * R + r) * K + k];
    if (global) {
      if (t < nt) out[t * gstride + r * ldo + k] = v;
    } else {
      out[t * P + r * ldo + k] = v;
    }
  }
  __syncthreads();  // `red` is reused by the next call
}

// LDS scratch of cols2s per atom: IS x R x K <= (2 x 256 threads / K) x 3 x K values
constexpr int kColsRed = 2 * 256 * 3;

// the split form when the launch could give the workgroup its `red` scratch (LDS budget), else cols2
template <bool SPLIT, typename T, int NT, int R, bool VEC>
__device__ __forceinline__ void colsx(const T* __restrict__ A, int lda, int I, const T* g, int ldg,
                                      const T* __restrict__ B, int ldb, int I2, const T* g2, int ldg2, int K,
                                      T* out, int ldo, int P, int nt, size_t gstride, bool global, T* red) {
  if constexpr (SPLIT)
    cols2s<T, NT, R, VEC>(A, lda, I, g, ldg, B, ldb, I2, g2, ldg2, K, out, ldo, P, nt, gstride, global, red);
  else
    cols2<T, NT, R, VEC>(A, lda, I, g, ldg, B, ldb, I2, g2, ldg2, K, out, ldo, P, nt, gstride, global);
}

// LDS layout of one atom (units of T); H = hidden, O = H/2 (block-1 output = block-2 input), Q = O.
struct Layout {
  int v, h, vb, v2, u, s, o, v1, h2, vb2, v22, u2, s2, o2;      // forward
  int gu2, gh2, gvb2, gv1, go, gu, gvec1, gvb, gv2;             // backward
  int P;
  __host__ __device__ Layout(int H) {
    const int O = H / 2, Q = O;
    int p = 0;
    v = p;    p += 3 * H;
    h = p;    p += 2 * H;   // [x | vec1]
    vb = p;   p += 3 * H;
    v2 = p;   p += 3 * O;
    u = p;    p += H;
    s = p;    p += H;
    o = p;    p += 2 * O;   // [xo | vo]
    v1 = p;   p += 3 * O;
    h2 = p;   p += 2 * Q;   // [x1 | vec1']
    vb2 = p;  p += 3 * Q;
    v22 = p;  p += 4;
    u2 = p;   p += Q;
    s2 = p;   p += Q;
    o2 = p;   p += 4;
    gu2 = p;  p += Q;
    gh2 = p;  p += 2 * Q;
    gvb2 = p; p += 3 * Q;
    gv1 = p;  p += 3 * O;
    go = p;   p += 2 * O;
    gu = p;   p += H;
    gvec1 = p; p += H;
    gvb = p;  p += 3 * H;
    gv2 = p;  p += 3 * O;
    P = (p + 3) & ~3;  // 16-byte aligned atoms (broadcast reads: no bank conflicts to avoid)
  }
};

// y may be NULL; jx / jv receive d(seed * y)/d(x, vec) with seed = gy[n] (gy NULL: 1, i.e. the
// Jacobian).  S: weight-gradient factors (weights mode), all NULL otherwise.
template <typename T, int NT, bool VEC, bool SPLIT>
__global__ __launch_bounds__(256) void k_eq_head(int n, int H, const T* __restrict__ x,
                                                 const T* __restrict__ vec, Weights<T> W,
                                                 T* __restrict__ y, T* __restrict__ jx,
                                                 T* __restrict__ jv, const T* __restrict__ gy,
                                                 Saves<T> S) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const Layout L(H);
  const int P = L.P, O = H / 2, Q = O;
  const int n0 = blockIdx.x * NT;
  const int nt = min(NT, n - n0);
  const int tid = threadIdx.x, bs = blockDim.x;
  T* red = sm + NT * P;  // cols2s scratch (launch adds NT x kColsRed values)

  // stage x -> h[0:H], vec -> v (rows of absent atoms are zero)
  for (int i = tid; i < NT * 4 * H; i += bs) {
    const int t = i / (4 * H), c = i - t * 4 * H;
    const bool live = t < nt;
    if (c < H)
      sm[t * P + L.h + c] = live ? x[(size_t)(n0 + t) * H + c] : T(0);
    else
      sm[t * P + L.v + c - H] = live ? vec[(size_t)(n0 + t) * 3 * H + c - H] : T(0);
  }
  __syncthreads();

  // ---------------- block 1 forward
  rows2<T, NT, 3, 2, VEC, 2>(W.w1, nullptr, H, W.w2, nullptr, O, H, sm + L.v, H, sm + L.vb, H, sm + L.v2, O, P);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    const T* vb = sm + t * P + L.vb;
    const T a0 = vb[c], a1 = vb[H + c], a2 = vb[2 * H + c];
    sm[t * P + L.h + H + c] = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 4>(W.u1w, W.u1b, H, nullptr, nullptr, 0, 2 * H, sm + L.h, 0, sm + L.u, 0, nullptr, 0, P);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    const T u = sm[t * P + L.u + c];
    sm[t * P + L.s + c] = u * sig(u);
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 4>(W.u2w, W.u2b, 2 * O, nullptr, nullptr, 0, H, sm + L.s, 0, sm + L.o, 0, nullptr, 0, P);
  __syncthreads();
  for (int i = tid; i < NT * O; i += bs) {
    const int t = i / O, c = i - t * O;
    T* a = sm + t * P;
    const T xo = a[L.o + c], vo = a[L.o + O + c];
    a[L.h2 + c] = xo * sig(xo);  // scalar activation of block 1
#pragma unroll
    for (int r = 0; r < 3; ++r) a[L.v1 + r * O + c] = vo * a[L.v2 + r * O + c];
  }
  __syncthreads();

  // ---------------- block 2 forward (Q = O inputs, 1 output)
  rows2<T, NT, 3, 2, VEC, 4>(W.v1, nullptr, Q, W.v2, nullptr, 1, O, sm + L.v1, O, sm + L.vb2, Q, sm + L.v22, 1, P);
  __syncthreads();
  for (int i = tid; i < NT * Q; i += bs) {
    const int t = i / Q, c = i - t * Q;
    const T* vb = sm + t * P + L.vb2;
    const T a0 = vb[c], a1 = vb[Q + c], a2 = vb[2 * Q + c];
    sm[t * P + L.h2 + Q + c] = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 8>(W.p1w, W.p1b, Q, nullptr, nullptr, 0, 2 * Q, sm + L.h2, 0, sm + L.u2, 0, nullptr, 0, P);
  __syncthreads();
  for (int i = tid; i < NT * Q; i += bs) {
    const int t = i / Q, c = i - t * Q;
    const T u = sm[t * P + L.u2 + c];
    const T sg = sig(u);
    sm[t * P + L.s2 + c] = u * sg;
    // backward seed: dy/do2 = (seed, 0) -> g_s2 = seed p2w[0][:]; g_u2 = g_s2 * SiLU'(u2)
    const T seed = gy ? (t < nt ? gy[n0 + t] : T(0)) : T(1);
    sm[t * P + L.gu2 + c] = seed * W.p2w[c] * sg * (T(1) + u * (T(1) - sg));
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 16>(W.p2w, W.p2b, 1, nullptr, nullptr, 0, Q, sm + L.s2, 0, sm + L.o2, 0, nullptr, 0, P);
  __syncthreads();
  if (y && tid < nt) y[n0 + tid] = sm[tid * P + L.o2];
  if (jx == nullptr) return;

  // ---------------- reverse pass for J = d y / d (x, vec), seed dy = 1 (vec'' enters y as 0 * sum)
  // block 2: g_h2 = P1^T g_u2
  colsx<SPLIT, T, NT, 1, VEC>(W.p1w, 2 * Q, Q, sm + L.gu2, 0, nullptr, 0, 0, nullptr, 0, 2 * Q, sm + L.gh2, 0, P, nt, 0,
                  false, red);
  __syncthreads();
  for (int i = tid; i < NT * Q; i += bs) {
    const int t = i / Q, c = i - t * Q;
    T* a = sm + t * P;
    const T nrm = a[L.h2 + Q + c];
    const T sc = nrm > T(0) ? a[L.gh2 + Q + c] / nrm : T(0);
#pragma unroll
    for (int r = 0; r < 3; ++r) a[L.gvb2 + r * Q + c] = sc * a[L.vb2 + r * Q + c];
  }
  __syncthreads();
  // g_v1 = V1^T g_vb2 (the vec'' gate contributes nothing: its cotangent is 0)
  colsx<SPLIT, T, NT, 3, VEC>(W.v1, O, Q, sm + L.gvb2, Q, nullptr, 0, 0, nullptr, 0, O, sm + L.gv1, O, P, nt, 0, false, red);
  __syncthreads();
  // block 1 gate: g_xo = g_x1 SiLU'(xo), g_vo = sum_a g_v1 v2, g_v2 = g_v1 vo
  for (int i = tid; i < NT * O; i += bs) {
    const int t = i / O, c = i - t * O;
    T* a = sm + t * P;
    const T xo = a[L.o + c], vo = a[L.o + O + c];
    const T sg = sig(xo);
    a[L.go + c] = a[L.gh2 + c] * sg * (T(1) + xo * (T(1) - sg));
    T gvo = T(0);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const T g = a[L.gv1 + r * O + c];
      gvo += g * a[L.v2 + r * O + c];
      a[L.gv2 + r * O + c] = g * vo;
    }
    a[L.go + O + c] = gvo;
  }
  __syncthreads();
  // g_s = U2^T g_o, g_u = g_s SiLU'(u)
  colsx<SPLIT, T, NT, 1, VEC>(W.u2w, H, 2 * O, sm + L.go, 0, nullptr, 0, 0, nullptr, 0, H, sm + L.gu, 0, P, nt, 0, false, red);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    T* a = sm + t * P;
    const T u = a[L.u + c];
    const T sg = sig(u);
    a[L.gu + c] *= sg * (T(1) + u * (T(1) - sg));
  }
  __syncthreads();
  // g_h = U1^T g_u (U1 is [H][2H]): the x half is J_x (global), the vec1 half stays in LDS
  colsx<SPLIT, T, NT, 1, VEC>(W.u1w, 2 * H, H, sm + L.gu, 0, nullptr, 0, 0, nullptr, 0, H, jx + (size_t)n0 * H, 0, P, nt,
                  (size_t)H, true, red);
  colsx<SPLIT, T, NT, 1, VEC>(W.u1w + H, 2 * H, H, sm + L.gu, 0, nullptr, 0, 0, nullptr, 0, H, sm + L.gvec1, 0, P, nt, 0,
                  false, red);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    T* a = sm + t * P;
    const T nrm = a[L.h + H + c];
    const T sc = nrm > T(0) ? a[L.gvec1 + c] / nrm : T(0);
#pragma unroll
    for (int r = 0; r < 3; ++r) a[L.gvb + r * H + c] = sc * a[L.vb + r * H + c];
  }
  __syncthreads();
  // J_vec[a] = W1^T g_vb[a] + W2^T g_v2[a]
  colsx<SPLIT, T, NT, 3, VEC>(W.w1, H, H, sm + L.gvb, H, W.w2, H, O, sm + L.gv2, O, H, jv + (size_t)n0 * 3 * H, H, P,
                  nt, (size_t)3 * H, true, red);
  if (S.a1 == nullptr) return;
  // weights mode: every LDS buffer is still intact (no aliasing); dump the per-atom factors
  const int wa1 = H + O, wa2 = Q + 1;
  for (int i = tid; i < nt * 3 * wa1; i += bs) {
    const int t = i / (3 * wa1), r = (i / wa1) % 3, c = i % wa1;
    const T* a = sm + t * P;
    S.a1[(size_t)(n0 + t) * 3 * wa1 + r * wa1 + c] = c < H ? a[L.gvb + r * H + c] : a[L.gv2 + r * O + c - H];
  }
  for (int i = tid; i < nt * 3 * wa2; i += bs) {
    const int t = i / (3 * wa2), r = (i / wa2) % 3, c = i % wa2;
    S.a2[(size_t)(n0 + t) * 3 * wa2 + r * wa2 + c] = c < Q ? sm[t * P + L.gvb2 + r * Q + c] : T(0);
  }
  for (int i = tid; i < nt * 3 * O; i += bs) {
    const int t = i / (3 * O), c = i % (3 * O);
    S.v1[(size_t)(n0 + t) * 3 * O + c] = sm[t * P + L.v1 + c];
  }
  for (int i = tid; i < nt * (2 * H + 1); i += bs) {
    const int t = i / (2 * H + 1), c = i % (2 * H + 1);
    S.hext[(size_t)(n0 + t) * (2 * H + 1) + c] = c < 2 * H ? sm[t * P + L.h + c] : T(1);
  }
  for (int i = tid; i < nt * (H + 1); i += bs) {
    const int t = i / (H + 1), c = i % (H + 1);
    S.sext[(size_t)(n0 + t) * (H + 1) + c] = c < H ? sm[t * P + L.s + c] : T(1);
    if (c < H) S.gu[(size_t)(n0 + t) * H + c] = sm[t * P + L.gu + c];
  }
  for (int i = tid; i < nt * 2 * O; i += bs) {
    const int t = i / (2 * O), c = i % (2 * O);
    S.go[(size_t)(n0 + t) * 2 * O + c] = sm[t * P + L.go + c];
  }
  for (int i = tid; i < nt * (2 * Q + 1); i += bs) {
    const int t = i / (2 * Q + 1), c = i % (2 * Q + 1);
    S.h2ext[(size_t)(n0 + t) * (2 * Q + 1) + c] = c < 2 * Q ? sm[t * P + L.h2 + c] : T(1);
  }
  for (int i = tid; i < nt * (Q + 1); i += bs) {
    const int t = i / (Q + 1), c = i % (Q + 1);
    S.s2ext[(size_t)(n0 + t) * (Q + 1) + c] = c < Q ? sm[t * P + L.s2 + c] : T(1);
    if (c < Q) S.gu2[(size_t)(n0 + t) * Q + c] = sm[t * P + L.gu2 + c];
  }
  if (tid < nt) {
    S.go2[(size_t)(n0 + tid) * 2] = gy ? gy[n0 + tid] : T(1);
    S.go2[(size_t)(n0 + tid) * 2 + 1] = T(0);
  }
}

// ---------------------------------------------------------------------------------------------------
// Second order (force-matching training).  The first-order backward maps (g_y, x, vec) to
// (g_x, g_vec) = g_y * J(x, vec); its VJP for cotangents (t_x, t_vec) of (g_x, g_vec) is, because the
// Hessian is symmetric, the DIRECTIONAL derivative of that gradient along (t_x, t_vec):
// forward-over-reverse.  Per atom: the forward, the tangent forward (dotted quantities), the reverse
// seeded with g_y and its tangent, all in LDS:
//   d_x, d_vec = g_y * d/dt [J](x + t t_x, vec + t t_vec)        (the HVP)
//   d_g_y      = <t_x, J_x> + <t_vec, J_vec> = ydot                (the tangent of y)
//   d W       = d/dt of the weight gradient of g_y * y, each a GEMM over [tangent rows ; plain rows]:
//               e.g. d U1 = sum_n gdot_u (x) [h | 1] + g_u (x) [hdot | 0].
// SiLU'(u) = s (1 + u (1 - s)), SiLU''(u) = s (1 - s) (2 + u (1 - 2 s)), s = sigmoid(u).  The norm's
// tangent and its gradient's tangent are 0 where the norm is 0 (the reference masks those rows).
template <typename T>
__device__ __forceinline__ T dsilu(T u) {
  const T s = sig(u);
  return s * (T(1) + u * (T(1) - s));
}
template <typename T>
__device__ __forceinline__ T d2silu(T u) {
  const T s = sig(u);
  return s * (T(1) - s) * (T(2) + u * (T(1) - T(2) * s));
}

// Layout plus g_s (U2^T g_o before SiLU') and the tangent buffers (prefix t).
struct Layout2 : Layout {
  int gs, th, tv, tvb, tv2, tu, ts, to, th2, tv1, tvb2, tu2, ts2;          // tangent forward
  int tgu2, tgh2, tgvb2, tgv1, tgo, tgv2, tgs, tgu, tgvec1, tgvb;          // tangent reverse
  int P2;
  __host__ __device__ Layout2(int H) : Layout(H) {
    const int O = H / 2, Q = O;
    int p = P;
    gs = p;     p += H;
    th = p;     p += 2 * H;  // [t_x | vec1dot]
    tv = p;     p += 3 * H;
    tvb = p;    p += 3 * H;
    tv2 = p;    p += 3 * O;
    tu = p;     p += H;
    ts = p;     p += H;
    to = p;     p += 2 * O;
    th2 = p;    p += 2 * Q;
    tv1 = p;    p += 3 * O;
    tvb2 = p;   p += 3 * Q;
    tu2 = p;    p += Q;
    ts2 = p;    p += Q;
    tgu2 = p;   p += Q;
    tgh2 = p;   p += 2 * Q;
    tgvb2 = p;  p += 3 * Q;
    tgv1 = p;   p += 3 * O;
    tgo = p;    p += 2 * O;
    tgv2 = p;   p += 3 * O;
    tgs = p;    p += H;
    tgu = p;    p += H;
    tgvec1 = p; p += H;
    tgvb = p;   p += 3 * H;
    P2 = (p + 3) & ~3;
  }
};

// Per-atom factors of the weight-gradient tangents: every array holds 2N atoms, [tangent half (atoms
// 0..N-1) ; plain half (N..2N-1)], so each weight's tangent is ONE GEMM over 2N (or 6N) rows with the
// layouts of Saves; vv [2][N][3][H] = [vec ; t_vec] is the second operand of [dW1; dW2].
template <typename T>
struct Saves2 {
  Saves<T> s;
  T* vv;
};

template <typename T, int NT, bool VEC, bool SPLIT>
__global__ __launch_bounds__(256) void k_eq_head_hvp(int n, int H, const T* __restrict__ x,
                                                     const T* __restrict__ vec, Weights<T> W,
                                                     const T* __restrict__ gy, const T* __restrict__ tx,
                                                     const T* __restrict__ tvec, T* __restrict__ dx,
                                                     T* __restrict__ dvec, T* __restrict__ dgy, Saves2<T> S2) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const Layout2 L(H);
  const int P = L.P2, O = H / 2, Q = O;
  const int n0 = blockIdx.x * NT;
  const int nt = min(NT, n - n0);
  const int tid = threadIdx.x, bs = blockDim.x;
  T* red = sm + NT * P;  // colsx scratch (SPLIT launches add NT x kColsRed values)

  // stage x -> h[0:H], vec -> v, t_x -> th[0:H], t_vec -> tv (absent atoms / tangents: zero)
  for (int i = tid; i < NT * 8 * H; i += bs) {
    const int t = i / (8 * H), c0 = i - t * 8 * H;
    const bool live = t < nt, tang = c0 >= 4 * H;
    const int c = tang ? c0 - 4 * H : c0;
    const T* src = c < H ? (tang ? tx : x) : (tang ? tvec : vec);
    T val = T(0);
    if (live && src) val = c < H ? src[(size_t)(n0 + t) * H + c] : src[(size_t)(n0 + t) * 3 * H + c - H];
    sm[t * P + (c < H ? (tang ? L.th : L.h) + c : (tang ? L.tv : L.v) + c - H)] = val;
  }
  __syncthreads();

  // ---------------- forward (block 1, block 2 up to s2; the gate vec'' does not reach y)
  rows2<T, NT, 3, 2, VEC, 2>(W.w1, nullptr, H, W.w2, nullptr, O, H, sm + L.v, H, sm + L.vb, H, sm + L.v2, O, P);
  rows2<T, NT, 3, 2, VEC, 2>(W.w1, nullptr, H, W.w2, nullptr, O, H, sm + L.tv, H, sm + L.tvb, H, sm + L.tv2, O, P);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    T* a = sm + t * P;
    const T b0 = a[L.vb + c], b1 = a[L.vb + H + c], b2 = a[L.vb + 2 * H + c];
    const T nrm = sqrt(b0 * b0 + b1 * b1 + b2 * b2);
    a[L.h + H + c] = nrm;
    a[L.th + H + c] = nrm > T(0)
        ? (b0 * a[L.tvb + c] + b1 * a[L.tvb + H + c] + b2 * a[L.tvb + 2 * H + c]) / nrm : T(0);
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 4>(W.u1w, W.u1b, H, W.u1w, nullptr, 0, 2 * H, sm + L.h, 0, sm + L.u, 0, nullptr, 0, P);
  rows2<T, NT, 1, 2, VEC, 4>(W.u1w, nullptr, H, W.u1w, nullptr, 0, 2 * H, sm + L.th, 0, sm + L.tu, 0, nullptr, 0, P);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    T* a = sm + t * P;
    const T u = a[L.u + c];
    a[L.s + c] = u * sig(u);
    a[L.ts + c] = dsilu(u) * a[L.tu + c];
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 4>(W.u2w, W.u2b, 2 * O, W.u2w, nullptr, 0, H, sm + L.s, 0, sm + L.o, 0, nullptr, 0, P);
  rows2<T, NT, 1, 2, VEC, 4>(W.u2w, nullptr, 2 * O, W.u2w, nullptr, 0, H, sm + L.ts, 0, sm + L.to, 0, nullptr, 0, P);
  __syncthreads();
  for (int i = tid; i < NT * O; i += bs) {
    const int t = i / O, c = i - t * O;
    T* a = sm + t * P;
    const T xo = a[L.o + c], vo = a[L.o + O + c], txo = a[L.to + c], tvo = a[L.to + O + c];
    a[L.h2 + c] = xo * sig(xo);
    a[L.th2 + c] = dsilu(xo) * txo;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      a[L.v1 + r * O + c] = vo * a[L.v2 + r * O + c];
      a[L.tv1 + r * O + c] = tvo * a[L.v2 + r * O + c] + vo * a[L.tv2 + r * O + c];
    }
  }
  __syncthreads();
  rows2<T, NT, 3, 2, VEC, 4>(W.v1, nullptr, Q, W.v1, nullptr, 0, O, sm + L.v1, O, sm + L.vb2, Q, sm + L.vb2, Q, P);
  rows2<T, NT, 3, 2, VEC, 4>(W.v1, nullptr, Q, W.v1, nullptr, 0, O, sm + L.tv1, O, sm + L.tvb2, Q, sm + L.tvb2, Q, P);
  __syncthreads();
  for (int i = tid; i < NT * Q; i += bs) {
    const int t = i / Q, c = i - t * Q;
    T* a = sm + t * P;
    const T b0 = a[L.vb2 + c], b1 = a[L.vb2 + Q + c], b2 = a[L.vb2 + 2 * Q + c];
    const T nrm = sqrt(b0 * b0 + b1 * b1 + b2 * b2);
    a[L.h2 + Q + c] = nrm;
    a[L.th2 + Q + c] = nrm > T(0)
        ? (b0 * a[L.tvb2 + c] + b1 * a[L.tvb2 + Q + c] + b2 * a[L.tvb2 + 2 * Q + c]) / nrm : T(0);
  }
  __syncthreads();
  rows2<T, NT, 1, 2, VEC, 8>(W.p1w, W.p1b, Q, W.p1w, nullptr, 0, 2 * Q, sm + L.h2, 0, sm + L.u2, 0, nullptr, 0, P);
  rows2<T, NT, 1, 2, VEC, 8>(W.p1w, nullptr, Q, W.p1w, nullptr, 0, 2 * Q, sm + L.th2, 0, sm + L.tu2, 0, nullptr, 0, P);
  __syncthreads();
  for (int i = tid; i < NT * Q; i += bs) {
    const int t = i / Q, c = i - t * Q;
    T* a = sm + t * P;
    const T u = a[L.u2 + c], tu = a[L.tu2 + c];
    const T seed = t < nt ? gy[n0 + t] : T(0);
    a[L.s2 + c] = u * sig(u);
    a[L.ts2 + c] = dsilu(u) * tu;
    // g_s2 = seed P2[0][:] (constant in x, vec): g_u2 = g_s2 SiLU'(u2), its tangent g_s2 SiLU''(u2) u2dot
    a[L.gu2 + c] = seed * W.p2w[c] * dsilu(u);
    a[L.tgu2 + c] = seed * W.p2w[c] * d2silu(u) * tu;
  }
  __syncthreads();

  // ---------------- reverse and its tangent (the transposed products shared in pairs)
  colsx<SPLIT, T, NT, 1, VEC>(W.p1w, 2 * Q, Q, sm + L.gu2, 0, nullptr, 0, 0, nullptr, 0, 2 * Q, sm + L.gh2, 0, P, nt, 0,
                       false, red);
  colsx<SPLIT, T, NT, 1, VEC>(W.p1w, 2 * Q, Q, sm + L.tgu2, 0, nullptr, 0, 0, nullptr, 0, 2 * Q, sm + L.tgh2, 0, P, nt, 0,
                       false, red);
  __syncthreads();
  for (int i = tid; i < NT * Q; i += bs) {
    const int t = i / Q, c = i - t * Q;
    T* a = sm + t * P;
    const T nrm = a[L.h2 + Q + c];
    const T inv = nrm > T(0) ? T(1) / nrm : T(0);
    const T gn = a[L.gh2 + Q + c] * inv, tgn = a[L.tgh2 + Q + c] * inv, tn = a[L.th2 + Q + c] * inv;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const T b = a[L.vb2 + r * Q + c];
      a[L.gvb2 + r * Q + c] = gn * b;
      a[L.tgvb2 + r * Q + c] = tgn * b + gn * (a[L.tvb2 + r * Q + c] - b * tn);
    }
  }
  __syncthreads();
  colsx<SPLIT, T, NT, 3, VEC>(W.v1, O, Q, sm + L.gvb2, Q, nullptr, 0, 0, nullptr, 0, O, sm + L.gv1, O, P, nt, 0, false, red);
  colsx<SPLIT, T, NT, 3, VEC>(W.v1, O, Q, sm + L.tgvb2, Q, nullptr, 0, 0, nullptr, 0, O, sm + L.tgv1, O, P, nt, 0, false, red);
  __syncthreads();
  for (int i = tid; i < NT * O; i += bs) {
    const int t = i / O, c = i - t * O;
    T* a = sm + t * P;
    const T xo = a[L.o + c], vo = a[L.o + O + c], txo = a[L.to + c], tvo = a[L.to + O + c];
    const T gx1 = a[L.gh2 + c], tgx1 = a[L.tgh2 + c];
    const T d1 = dsilu(xo);
    a[L.go + c] = gx1 * d1;
    a[L.tgo + c] = tgx1 * d1 + gx1 * d2silu(xo) * txo;
    T gvo = T(0), tgvo = T(0);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const T g = a[L.gv1 + r * O + c], tg = a[L.tgv1 + r * O + c];
      const T v2 = a[L.v2 + r * O + c], tv2 = a[L.tv2 + r * O + c];
      gvo += g * v2;
      tgvo += tg * v2 + g * tv2;
      a[L.gv2 + r * O + c] = g * vo;
      a[L.tgv2 + r * O + c] = tg * vo + g * tvo;
    }
    a[L.go + O + c] = gvo;
    a[L.tgo + O + c] = tgvo;
  }
  __syncthreads();
  colsx<SPLIT, T, NT, 1, VEC>(W.u2w, H, 2 * O, sm + L.go, 0, nullptr, 0, 0, nullptr, 0, H, sm + L.gs, 0, P, nt, 0, false, red);
  colsx<SPLIT, T, NT, 1, VEC>(W.u2w, H, 2 * O, sm + L.tgo, 0, nullptr, 0, 0, nullptr, 0, H, sm + L.tgs, 0, P, nt, 0, false, red);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    T* a = sm + t * P;
    const T u = a[L.u + c], gsv = a[L.gs + c];
    const T d1 = dsilu(u);
    a[L.gu + c] = gsv * d1;
    a[L.tgu + c] = a[L.tgs + c] * d1 + gsv * d2silu(u) * a[L.tu + c];
  }
  __syncthreads();
  // U1^T: the x half of the tangent is d_x (global); the vec1 halves stay in LDS
  colsx<SPLIT, T, NT, 1, VEC>(W.u1w, 2 * H, H, sm + L.tgu, 0, nullptr, 0, 0, nullptr, 0, H, dx + (size_t)n0 * H, 0, P, nt,
                       (size_t)H, true, red);
  colsx<SPLIT, T, NT, 1, VEC>(W.u1w + H, 2 * H, H, sm + L.gu, 0, nullptr, 0, 0, nullptr, 0, H, sm + L.gvec1, 0, P, nt, 0,
                       false, red);
  colsx<SPLIT, T, NT, 1, VEC>(W.u1w + H, 2 * H, H, sm + L.tgu, 0, nullptr, 0, 0, nullptr, 0, H, sm + L.tgvec1, 0, P, nt, 0,
                       false, red);
  __syncthreads();
  for (int i = tid; i < NT * H; i += bs) {
    const int t = i / H, c = i - t * H;
    T* a = sm + t * P;
    const T nrm = a[L.h + H + c];
    const T inv = nrm > T(0) ? T(1) / nrm : T(0);
    const T gn = a[L.gvec1 + c] * inv, tgn = a[L.tgvec1 + c] * inv, tn = a[L.th + H + c] * inv;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const T b = a[L.vb + r * H + c];
      a[L.gvb + r * H + c] = gn * b;
      a[L.tgvb + r * H + c] = tgn * b + gn * (a[L.tvb + r * H + c] - b * tn);
    }
  }
  __syncthreads();
  // d_vec[a] = W1^T gdot_vb[a] + W2^T gdot_v2[a]
  colsx<SPLIT, T, NT, 3, VEC>(W.w1, H, H, sm + L.tgvb, H, W.w2, H, O, sm + L.tgv2, O, H, dvec + (size_t)n0 * 3 * H, H, P,
                       nt, (size_t)3 * H, true, red);
  // d_g_y = ydot = P2[0][:] . s2dot
  if (dgy && tid < nt) {
    const T* a = sm + tid * P;
    T acc = T(0);
    for (int c = 0; c < Q; ++c) acc += W.p2w[c] * a[L.ts2 + c];
    dgy[n0 + tid] = acc;
  }
  if (S2.vv == nullptr) return;
  const Saves<T> S = S2.s;
  // tangent half at atom n0 + t, plain half at n + n0 + t
  const int wa1 = H + O, wa2 = Q + 1;
  for (int i = tid; i < nt * 2 * 3 * wa1; i += bs) {
    const int half = i / (nt * 3 * wa1), j = i - half * nt * 3 * wa1;
    const int t = j / (3 * wa1), r = (j / wa1) % 3, c = j % wa1;
    const T* a = sm + t * P;
    const int gvb = half ? L.gvb : L.tgvb, gv2 = half ? L.gv2 : L.tgv2;
    S.a1[((size_t)half * n + n0 + t) * 3 * wa1 + r * wa1 + c] = c < H ? a[gvb + r * H + c] : a[gv2 + r * O + c - H];
  }
  for (int i = tid; i < nt * 2 * 3 * H; i += bs) {
    const int half = i / (nt * 3 * H), j = i - half * nt * 3 * H;
    const int t = j / (3 * H), c = j % (3 * H);
    S2.vv[((size_t)half * n + n0 + t) * 3 * H + c] = sm[t * P + (half ? L.tv : L.v) + c];
  }
  for (int i = tid; i < nt * 2 * 3 * wa2; i += bs) {
    const int half = i / (nt * 3 * wa2), j = i - half * nt * 3 * wa2;
    const int t = j / (3 * wa2), r = (j / wa2) % 3, c = j % wa2;
    S.a2[((size_t)half * n + n0 + t) * 3 * wa2 + r * wa2 + c] =
        c < Q ? sm[t * P + (half ? L.gvb2 : L.tgvb2) + r * Q + c] : T(0);
  }
  for (int i = tid; i < nt * 2 * 3 * O; i += bs) {
    const int half = i / (nt * 3 * O), j = i - half * nt * 3 * O;
    const int t = j / (3 * O), c = j % (3 * O);
    S.v1[((size_t)half * n + n0 + t) * 3 * O + c] = sm[t * P + (half ? L.tv1 : L.v1) + c];
  }
  for (int i = tid; i < nt * 2 * (2 * H + 1); i += bs) {
    const int half = i / (nt * (2 * H + 1)), j = i - half * nt * (2 * H + 1);
    const int t = j / (2 * H + 1), c = j % (2 * H + 1);
    S.hext[((size_t)half * n + n0 + t) * (2 * H + 1) + c] =
        c < 2 * H ? sm[t * P + (half ? L.th : L.h) + c] : T(half ? 0 : 1);
  }
  for (int i = tid; i < nt * 2 * (H + 1); i += bs) {
    const int half = i / (nt * (H + 1)), j = i - half * nt * (H + 1);
    const int t = j / (H + 1), c = j % (H + 1);
    S.sext[((size_t)half * n + n0 + t) * (H + 1) + c] = c < H ? sm[t * P + (half ? L.ts : L.s) + c] : T(half ? 0 : 1);
    if (c < H) S.gu[((size_t)half * n + n0 + t) * H + c] = sm[t * P + (half ? L.gu : L.tgu) + c];
  }
  for (int i = tid; i < nt * 2 * 2 * O; i += bs) {
    const int half = i / (nt * 2 * O), j = i - half * nt * 2 * O;
    const int t = j / (2 * O), c = j % (2 * O);
    S.go[((size_t)half * n + n0 + t) * 2 * O + c] = sm[t * P + (half ? L.go : L.tgo) + c];
  }
  for (int i = tid; i < nt * 2 * (2 * Q + 1); i += bs) {
    const int half = i / (nt * (2 * Q + 1)), j = i - half * nt * (2 * Q + 1);
    const int t = j / (2 * Q + 1), c = j % (2 * Q + 1);
    S.h2ext[((size_t)half * n + n0 + t) * (2 * Q + 1) + c] =
        c < 2 * Q ? sm[t * P + (half ? L.th2 : L.h2) + c] : T(half ? 0 : 1);
  }
  for (int i = tid; i < nt * 2 * (Q + 1); i += bs) {
    const int half = i / (nt * (Q + 1)), j = i - half * nt * (Q + 1);
    const int t = j / (Q + 1), c = j % (Q + 1);
    S.s2ext[((size_t)half * n + n0 + t) * (Q + 1) + c] =
        c < Q ? sm[t * P + (half ? L.ts2 : L.s2) + c] : T(half ? 0 : 1);
    if (c < Q) S.gu2[((size_t)half * n + n0 + t) * Q + c] = sm[t * P + (half ? L.gu2 : L.tgu2) + c];
  }
  if (tid < 2 * nt) {
    const int half = tid / nt, t = tid % nt;
    S.go2[((size_t)half * n + n0 + t) * 2] = half ? gy[n0 + t] : T(0);
    S.go2[((size_t)half * n + n0 + t) * 2 + 1] = T(0);
  }
}

// g_x[n] = g_y[n] J_x[n],  g_vec[n] = g_y[n] J_vec[n]
template <typename T>
__global__ void k_scale(int n, int H, const T* __restrict__ gy, const T* __restrict__ jx,
                        const T* __restrict__ jv, T* __restrict__ gx, T* __restrict__ gv) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n * 4 * H) return;
  const int t = (int)(i / (4 * H)), c = (int)(i - (long long)t * 4 * H);
  const T g = gy[t];
  if (c < H)
    gx[(size_t)t * H + c] = g * jx[(size_t)t * H + c];
  else
    gv[(size_t)t * 3 * H + c - H] = g * jv[(size_t)t * 3 * H + c - H];
}

}  // namespace head
}  // namespace tmd

using namespace tmd;

// Atoms per workgroup: the kernel is latency-bound (~20 dependent product phases), so small systems
// want many workgroups (1 atom each); from ~2k atoms 2 atoms share each weight load (measured on
// MI355X: 56 us at 580 atoms with 1, 41 ns/atom at 50k atoms with 2; 4 is slower at every size).
static int head_tile(int dtype, int H, int n, size_t* smem, bool* split) {
  const size_t es = dtype == TMDNET_F64 ? 8 : 4;
  const size_t per = (size_t)head::Layout(H).P * es;
  int cap = n < 2048 ? 1 : 2;
  static const int env_nt = [] { const char* e = getenv("TMDNET_HEAD_NT"); return e ? atoi(e) : 0; }();  // tuning, read once
  if (env_nt > 0) cap = env_nt >= 4 ? 4 : env_nt >= 2 ? 2 : 1;
  for (int nt = cap; nt >= 1; nt /= 2)
    if (nt * per <= 64 * 1024) {
      // the split transposed products (cols2s) when their scratch fits the same 64 KB
      const size_t with = nt * (per + (size_t)head::kColsRed * es);
      *split = with <= 64 * 1024;
      *smem = *split ? with : nt * per;
      return nt;
    }
  return 0;
}

template <typename T>
static int launch_head(int n, int H, const void* x, const void* vec, const void* const* w, void* y,
                       void* jx, void* jv, const void* gy, void* const* sv, int nt, size_t smem, bool split,
                       hipStream_t st) {
  head::Saves<T> S{};
  if (sv)
    S = head::Saves<T>{(T*)sv[0], (T*)sv[1], (T*)sv[2], (T*)sv[3], (T*)sv[4], (T*)sv[5],
                       (T*)sv[6], (T*)sv[7], (T*)sv[8], (T*)sv[9], (T*)sv[10]};
  head::Weights<T> W{(const T*)w[0], (const T*)w[1], (const T*)w[2], (const T*)w[3],
                     (const T*)w[4], (const T*)w[5], (const T*)w[6], (const T*)w[7],
                     (const T*)w[8], (const T*)w[9], (const T*)w[10], (const T*)w[11]};
  dim3 g((n + nt - 1) / nt), b(256);
  const bool vec4 = H % 8 == 0;  // every LDS offset / row length a multiple of 4
#define TMD_HEAD_LAUNCH(NT_, V_)                                                                          \
  if (split)                                                                                             \
    hipLaunchKernelGGL((head::k_eq_head<T, NT_, V_, true>), g, b, smem, st, n, H, (const T*)x, (const T*)vec, \
                       W, (T*)y, (T*)jx, (T*)jv, (const T*)gy, S);                                         \
  else                                                                                                   \
    hipLaunchKernelGGL((head::k_eq_head<T, NT_, V_, false>), g, b, smem, st, n, H, (const T*)x, (const T*)vec, \
                       W, (T*)y, (T*)jx, (T*)jv, (const T*)gy, S)
  if (vec4) {
    if (nt == 4) TMD_HEAD_LAUNCH(4, true);
    else if (nt == 2) TMD_HEAD_LAUNCH(2, true);
    else TMD_HEAD_LAUNCH(1, true);
  } else {
    if (nt == 4) TMD_HEAD_LAUNCH(4, false);
    else if (nt == 2) TMD_HEAD_LAUNCH(2, false);
    else TMD_HEAD_LAUNCH(1, false);
  }
#undef TMD_HEAD_LAUNCH
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_eq_head_fwd(int dtype, int n_atoms, int hidden, const void* x, const void* vec,
                                  const void* const* weights, void* y, void* jac_x, void* jac_vec,
                                  void* stream) {
  if (n_atoms < 0 || hidden < 4 || hidden % 4 || !x || !vec || !weights || !y) return kBadArgument;
  if ((jac_x == nullptr) != (jac_vec == nullptr)) return kBadArgument;
  for (int i = 0; i < 12; ++i)
    if (!weights[i]) return kBadArgument;
  if (n_atoms == 0) return kOk;
  size_t smem = 0;
  bool split = false;
  const int nt = head_tile(dtype, hidden, n_atoms, &smem, &split);
  if (nt == 0) return kUnsupported;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return launch_head<float>(n_atoms, hidden, x, vec, weights, y, jac_x, jac_vec, nullptr, nullptr, nt, smem, split, st);
  if (dtype == TMDNET_F64)
    return launch_head<double>(n_atoms, hidden, x, vec, weights, y, jac_x, jac_vec, nullptr, nullptr, nt, smem, split, st);
  return kUnsupported;
}

extern "C" int tmdnet_eq_head_bwd_weights(int dtype, int n_atoms, int hidden, const void* x,
                                          const void* vec, const void* const* weights,
                                          const void* grad_y, void* grad_x, void* grad_vec,
                                          void* const* saves, void* stream) {
  if (n_atoms < 0 || hidden < 4 || hidden % 4 || !x || !vec || !weights || !grad_y || !grad_x ||
      !grad_vec || !saves)
    return kBadArgument;
  for (int i = 0; i < 12; ++i)
    if (!weights[i]) return kBadArgument;
  for (int i = 0; i < 11; ++i)
    if (!saves[i]) return kBadArgument;
  if (n_atoms == 0) return kOk;
  size_t smem = 0;
  bool split = false;
  const int nt = head_tile(dtype, hidden, n_atoms, &smem, &split);
  if (nt == 0) return kUnsupported;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return launch_head<float>(n_atoms, hidden, x, vec, weights, nullptr, grad_x, grad_vec, grad_y, saves, nt,
                              smem, split, st);
  if (dtype == TMDNET_F64)
    return launch_head<double>(n_atoms, hidden, x, vec, weights, nullptr, grad_x, grad_vec, grad_y, saves, nt,
                               smem, split, st);
  return kUnsupported;
}

template <typename T>
static int launch_head_hvp(int n, int H, const void* x, const void* vec, const void* const* w, const void* gy,
                           const void* tx, const void* tvec, void* dx, void* dvec, void* dgy, void* const* sv,
                           hipStream_t st) {
  head::Saves2<T> S{};
  if (sv)
    S = head::Saves2<T>{{(T*)sv[0], (T*)sv[1], (T*)sv[2], (T*)sv[3], (T*)sv[4], (T*)sv[5], (T*)sv[6], (T*)sv[7],
                         (T*)sv[8], (T*)sv[9], (T*)sv[10]},
                        (T*)sv[11]};
  head::Weights<T> W{(const T*)w[0], (const T*)w[1], (const T*)w[2], (const T*)w[3],
                     (const T*)w[4], (const T*)w[5], (const T*)w[6], (const T*)w[7],
                     (const T*)w[8], (const T*)w[9], (const T*)w[10], (const T*)w[11]};
  const size_t per = (size_t)head::Layout2(H).P2 * sizeof(T);
  // one atom per workgroup below 2048 atoms (latency-bound chain), two above when they fit 64 KB
  const int nt = (n >= 2048 && 2 * per <= 64 * 1024) ? 2 : 1;
  if (per > 64 * 1024) return kUnsupported;
  const size_t with = nt * (per + (size_t)head::kColsRed * sizeof(T));  // + the split products' scratch
  const bool split = with <= 64 * 1024;
  const size_t smem = split ? with : nt * per;
  dim3 g((n + nt - 1) / nt), b(256);
  const bool vec4 = H % 8 == 0;
#define TMD_HVP_LAUNCH(NT_, V_)                                                                              \
  if (split)                                                                                                \
    hipLaunchKernelGGL((head::k_eq_head_hvp<T, NT_, V_, true>), g, b, smem, st, n, H, (const T*)x, (const T*)vec, \
                       W, (const T*)gy, (const T*)tx, (const T*)tvec, (T*)dx, (T*)dvec, (T*)dgy, S);            \
  else                                                                                                      \
    hipLaunchKernelGGL((head::k_eq_head_hvp<T, NT_, V_, false>), g, b, smem, st, n, H, (const T*)x,           \
                       (const T*)vec, W, (const T*)gy, (const T*)tx, (const T*)tvec, (T*)dx, (T*)dvec, (T*)dgy, S)
  if (vec4) {
    if (nt == 2) TMD_HVP_LAUNCH(2, true);
    else TMD_HVP_LAUNCH(1, true);
  } else {
    if (nt == 2) TMD_HVP_LAUNCH(2, false);
    else TMD_HVP_LAUNCH(1, false);
  }
#undef TMD_HVP_LAUNCH
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_eq_head_hvp(int dtype, int n_atoms, int hidden, const void* x, const void* vec,
                                  const void* const* weights, const void* grad_y, const void* tan_x,
                                  const void* tan_vec, void* d_x, void* d_vec, void* d_grad_y,
                                  void* const* saves, void* stream) {
  if (n_atoms < 0 || hidden < 4 || hidden % 4 || !x || !vec || !weights || !grad_y || !d_x || !d_vec)
    return kBadArgument;
  for (int i = 0; i < 12; ++i)
    if (!weights[i]) return kBadArgument;
  if (saves)
    for (int i = 0; i < 12; ++i)
      if (!saves[i]) return kBadArgument;
  if (n_atoms == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    return launch_head_hvp<float>(n_atoms, hidden, x, vec, weights, grad_y, tan_x, tan_vec, d_x, d_vec, d_grad_y,
                                  saves, st);
  if (dtype == TMDNET_F64)
    return launch_head_hvp<double>(n_atoms, hidden, x, vec, weights, grad_y, tan_x, tan_vec, d_x, d_vec, d_grad_y,
                                   saves, st);
  return kUnsupported;
}

extern "C" int tmdnet_eq_head_bwd(int dtype, int n_atoms, int hidden, const void* grad_y,
                                  const void* jac_x, const void* jac_vec, void* grad_x, void* grad_vec,
                                  void* stream) {
  if (n_atoms < 0 || hidden < 1 || !grad_y || !jac_x || !jac_vec || !grad_x || !grad_vec) return kBadArgument;
  const long long work = (long long)n_atoms * 4 * hidden;
  if (work == 0) return kOk;
  const int tb = 256;
  dim3 g((unsigned)((work + tb - 1) / tb));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMDNET_F32)
    hipLaunchKernelGGL(head::k_scale<float>, g, dim3(tb), 0, st, n_atoms, hidden, (const float*)grad_y,
                       (const float*)jac_x, (const float*)jac_vec, (float*)grad_x, (float*)grad_vec);
  else if (dtype == TMDNET_F64)
    hipLaunchKernelGGL(head::k_scale<double>, g, dim3(tb), 0, st, n_atoms, hidden, (const double*)grad_y,
                       (const double*)jac_x, (const double*)jac_vec, (double*)grad_x, (double*)grad_vec);
  else
    return kUnsupported;
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
