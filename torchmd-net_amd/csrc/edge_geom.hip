// Fused per-edge geometry: RBF expansion (expnorm / gauss) + cosine cutoff + unit vectors.
// Reference: ExpNormalSmearing (models/utils.py:303-344), GaussianSmearing (utils.py:272-300),
// CosineCutoff (utils.py:362-390), d_ij normalisation (torchmd_et.py:173-174, tensornet.py:223-226).
// HBM-bound streaming kernels: forward reads delta/r (16 B/edge) and writes R+4 values per edge;
// backward reads the R+4 incoming gradients and writes 16 B/edge.
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace geom {

template <typename T> struct Cfg {
  int E, R, type;
  const int32_t* src;
  const int32_t* dst;
  const T* dl;
  const T* r;
  const T* mu;
  const T* beta;
  T cl, cu, alpha;
};

template <typename T> __device__ __forceinline__ T pi() { return T(3.14159265358979323846); }

// CosineCutoff(cl, cu) and its derivative w.r.t. r (utils.py:368-390)
template <typename T> __device__ __forceinline__ void cosine_cutoff(T r, T cl, T cu, T& c, T& dc) {
  if (cl > T(0)) {
    const T w = T(2) * pi<T>() / (cu - cl);
    const T arg = pi<T>() * (T(2) * (r - cl) / (cu - cl) + T(1));
    const bool in = (r < cu) && (r > cl);
    c = in ? T(0.5) * (cos(arg) + T(1)) : T(0);
    dc = in ? T(-0.5) * sin(arg) * w : T(0);
  } else {
    const bool in = r < cu;
    const T arg = r * pi<T>() / cu;
    c = in ? T(0.5) * (cos(arg) + T(1)) : T(0);
    dc = in ? T(-0.5) * sin(arg) * pi<T>() / cu : T(0);
  }
}

// CosineCutoff with its first and second derivatives w.r.t. r
template <typename T> __device__ __forceinline__ void cosine_cutoff2(T r, T cl, T cu, T& c, T& dc, T& d2c) {
  const bool in = cl > T(0) ? (r < cu) && (r > cl) : r < cu;
  const T w = cl > T(0) ? T(2) * pi<T>() / (cu - cl) : pi<T>() / cu;
  const T arg = cl > T(0) ? pi<T>() * (T(2) * (r - cl) / (cu - cl) + T(1)) : r * pi<T>() / cu;
  const T cs = cos(arg);
  c = in ? T(0.5) * (cs + T(1)) : T(0);
  dc = in ? T(-0.5) * sin(arg) * w : T(0);
  d2c = in ? T(-0.5) * cs * w * w : T(0);
}

// basis value, d/dr and d2/dr2 (the force-loss second order)
template <typename T>
__device__ __forceinline__ void basis2(const Cfg<T>& P, T r, int k, T& f, T& df, T& d2f) {
  if (P.type == TMDNET_RBF_EXPNORM) {
    T c0, dc0, d2c0;
    cosine_cutoff2<T>(r, T(0), P.cu, c0, dc0, d2c0);
    const T u = exp(P.alpha * (P.cl - r));
    const T du = -P.alpha * u, d2u = P.alpha * P.alpha * u;
    const T b = P.beta[k];
    const T z = u - P.mu[k];
    const T g = exp(-b * z * z);
    const T q = T(-2) * b * z * du;  // dg = g q
    const T dg = g * q;
    const T d2g = g * (q * q - T(2) * b * (du * du + z * d2u));
    f = c0 * g;
    df = dc0 * g + c0 * dg;
    d2f = d2c0 * g + T(2) * dc0 * dg + c0 * d2g;
  } else {
    const T z = r - P.mu[k];
    const T coeff = P.beta[0];
    f = exp(coeff * z * z);
    df = f * T(2) * coeff * z;
    d2f = f * (T(4) * coeff * coeff * z * z + T(2) * coeff);
  }
}

// basis value and d/dr
template <typename T>
__device__ __forceinline__ void basis(const Cfg<T>& P, T r, int k, T& f, T& df) {
  if (P.type == TMDNET_RBF_EXPNORM) {
    T c0, dc0;
    cosine_cutoff<T>(r, T(0), P.cu, c0, dc0);
    const T u = exp(P.alpha * (P.cl - r));
    const T du = -P.alpha * u;
    const T z = u - P.mu[k];
    const T g = exp(-P.beta[k] * z * z);
    const T dg = g * (T(-2) * P.beta[k] * z * du);
    f = c0 * g;
    df = dc0 * g + c0 * dg;
  } else {
    const T z = r - P.mu[k];
    const T coeff = P.beta[0];
    f = exp(coeff * z * z);
    df = f * T(2) * coeff * z;
  }
}

// rows != NULL: also the features of the edges rows[p] into frows [n_rows][R] (the pair rows the ET
// projection GEMM reads; replaces a gather of f), and with drows != NULL their r-derivatives into drows
// (the dr-mode force pass's operand; replaces a tmdnet_rbf_deriv launch after the forward)
template <typename T>
__global__ void k_fwd(Cfg<T> P, T* __restrict__ f, T* __restrict__ C, T* __restrict__ u,
                      const int32_t* __restrict__ rows, int n_rows, T* __restrict__ frows, T* __restrict__ drows) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nf = f ? (long long)P.E * P.R : 0;
  if (i < nf) {
    const int e = (int)(i / P.R), k = (int)(i % P.R);
    T v, dv;
    basis(P, P.r[e], k, v, dv);
    f[i] = v;
  }
  if (rows && i < (long long)n_rows * P.R) {
    const int p = (int)(i / P.R), k = (int)(i % P.R);
    T v, dv;
    basis(P, P.r[rows[p]], k, v, dv);
    frows[i] = v;
    if (drows) drows[i] = dv;
  }
  if (i < P.E) {
    const int e = (int)i;
    if (C) {
      T c, dc;
      cosine_cutoff<T>(P.r[e], P.cl, P.cu, c, dc);
      C[e] = c;
    }
    if (u) {
      const T x = P.dl[3 * e], y = P.dl[3 * e + 1], z = P.dl[3 * e + 2];
      if (P.src[e] == P.dst[e]) {
        u[3 * e] = x; u[3 * e + 1] = y; u[3 * e + 2] = z;
      } else {
        const T n = sqrt(x * x + y * y + z * z);
        u[3 * e] = x / n; u[3 * e + 1] = y / n; u[3 * e + 2] = z / n;
      }
    }
  }
}

// The incoming gradients of the rbf and cutoff outputs: up to 3 each (one per consumer of the output;
// summed here in slot order instead of by separate autograd add launches), NULL slots skipped.
template <typename T> struct GIn {
  const T* f[3];
  const T* c[3];
};

// One wave per edge (grid-stride); lanes over the basis index.
template <typename T>
__global__ __launch_bounds__(256) void k_bwd(Cfg<T> P, GIn<T> G, const T* __restrict__ gu, T* __restrict__ gr,
                                             T* __restrict__ gdl) {
  const int lane = lane_id();
  const int nw = gridDim.x * (blockDim.x / TMD_WAVE);
  const bool anyf = G.f[0] || G.f[1] || G.f[2], anyc = G.c[0] || G.c[1] || G.c[2];
  for (int e = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE; e < P.E; e += nw) {
    const T r = P.r[e];
    T acc = T(0);
    if (anyf) {
      for (int k = lane; k < P.R; k += TMD_WAVE) {
        T v, dv;
        basis(P, r, k, v, dv);
        const long long o = (long long)e * P.R + k;
        T g = G.f[0] ? G.f[0][o] : T(0);
        if (G.f[1]) g += G.f[1][o];
        if (G.f[2]) g += G.f[2][o];
        acc += g * dv;
      }
      acc = wave_sum(acc);
    }
    if (lane == 0) {
      if (anyc) {
        T c, dc;
        cosine_cutoff<T>(r, P.cl, P.cu, c, dc);
        T g = G.c[0] ? G.c[0][e] : T(0);
        if (G.c[1]) g += G.c[1][e];
        if (G.c[2]) g += G.c[2][e];
        acc += g * dc;
      }
      gr[e] = acc;
      T gx = T(0), gy = T(0), gz = T(0);
      if (gu) {
        const T x = P.dl[3 * e], y = P.dl[3 * e + 1], z = P.dl[3 * e + 2];
        const T a = gu[3 * e], b = gu[3 * e + 1], c = gu[3 * e + 2];
        if (P.src[e] == P.dst[e]) {
          gx = a; gy = b; gz = c;
        } else {
          const T n = sqrt(x * x + y * y + z * z);
          const T ux = x / n, uy = y / n, uz = z / n;
          const T dot = ux * a + uy * b + uz * c;
          gx = (a - ux * dot) / n;
          gy = (b - uy * dot) / n;
          gz = (c - uz * dot) / n;
        }
      }
      gdl[3 * e] = gx;
      gdl[3 * e + 1] = gy;
      gdl[3 * e + 2] = gz;
    }
  }
}

// No basis-row gradient at all (every consumer of the rbf rows took the dr route: the fused C5 stack and
// neighbour embedding hand back g_r themselves): one thread per edge -- the cutoff and unit-vector terms
// only, every load and store coalesced (the lane-parallel form below leaves 13 of an edge's 16 lanes
// idle then: C5 0.33 ms).
template <typename T>
__global__ __launch_bounds__(256) void k_bwd_e(Cfg<T> P, GIn<T> G, const T* __restrict__ gu, T* __restrict__ gr,
                                               T* __restrict__ gdl) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= P.E) return;
  const T r = P.r[e];
  T acc = T(0);
  if (G.c[0] || G.c[1] || G.c[2]) {
    T c, dc;
    cosine_cutoff<T>(r, P.cl, P.cu, c, dc);
    T g = G.c[0] ? G.c[0][e] : T(0);
    if (G.c[1]) g += G.c[1][e];
    if (G.c[2]) g += G.c[2][e];
    acc = g * dc;
  }
  gr[e] = acc;
  T gx = T(0), gy = T(0), gz = T(0);
  if (gu) {
    const T x = P.dl[3 * e], y = P.dl[3 * e + 1], z = P.dl[3 * e + 2];
    const T a = gu[3 * e], b = gu[3 * e + 1], c = gu[3 * e + 2];
    if (P.src[e] == P.dst[e]) {
      gx = a; gy = b; gz = c;
    } else {
      const T n = sqrt(x * x + y * y + z * z);
      const T ux = x / n, uy = y / n, uz = z / n;
      const T dot = ux * a + uy * b + uz * c;
      gx = (a - ux * dot) / n;
      gy = (b - uy * dot) / n;
      gz = (c - uz * dot) / n;
    }
  }
  gdl[3 * e] = gx;
  gdl[3 * e + 1] = gy;
  gdl[3 * e + 2] = gz;
}

// Lane-parallel form of k_bwd (the default): LPE = R / KPL lanes per edge, each lane owning KPL = 16 /
// sizeof(T) consecutive basis indices (one 16-byte load per gradient slot), 64 / LPE edges per wave, so
// a wave reads 64 / LPE whole gradient rows as one coalesced stream.  The per-edge terms of the basis
// (exp(alpha (cl - r)), the cosine cutoff and its derivative) are formed once per lane instead of once
// per basis index; the lane group's partial sums meet in an xor butterfly (identical in every lane),
// and the group's lanes 0 / 1..3 write g_r and the three unit-vector Jacobian components.
template <typename T, int LPE>
__global__ __launch_bounds__(256) void k_bwd_v(Cfg<T> P, GIn<T> G, const T* __restrict__ gu, T* __restrict__ gr,
                                               T* __restrict__ gdl) {
  constexpr int KPL = 16 / (int)sizeof(T), EPW = TMD_WAVE / LPE;
  using V = T __attribute__((ext_vector_type(KPL)));
  const int lane = lane_id(), sub = lane % LPE, slot = lane / LPE;
  const long long nw = (long long)gridDim.x * (blockDim.x / TMD_WAVE);
  const bool anyf = G.f[0] || G.f[1] || G.f[2], anyc = G.c[0] || G.c[1] || G.c[2];
  const bool expnorm = P.type == TMDNET_RBF_EXPNORM;
  for (long long w = (long long)blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE;
       w * EPW < P.E; w += nw) {
    const long long e = w * EPW + slot;
    const bool live = e < P.E;
    const T r = live ? P.r[e] : T(0);
    T acc = T(0);
    if (anyf) {
      const long long o = e * P.R + (long long)sub * KPL;
      V g{};
      if (live) {
        if (G.f[0]) g = *reinterpret_cast<const V*>(G.f[0] + o);
        if (G.f[1]) g += *reinterpret_cast<const V*>(G.f[1] + o);
        if (G.f[2]) g += *reinterpret_cast<const V*>(G.f[2] + o);
      }
      if (expnorm) {
        T c0, dc0;
        cosine_cutoff<T>(r, T(0), P.cu, c0, dc0);
        const T u = exp(P.alpha * (P.cl - r));
        const T du = -P.alpha * u;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
          const int k = sub * KPL + i;
          const T b = P.beta[k];
          const T z = u - P.mu[k];
          const T gk = exp(-b * z * z);
          acc += g[i] * gk * (dc0 + c0 * (T(-2) * b * z * du));
        }
      } else {
        const T coeff = P.beta[0];
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
          const T z = r - P.mu[sub * KPL + i];
          acc += g[i] * exp(coeff * z * z) * T(2) * coeff * z;
        }
      }
#pragma unroll
      for (int m = LPE / 2; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
    }
    if (!live) continue;
    if (sub == 0) {
      if (anyc) {
        T c, dc;
        cosine_cutoff<T>(r, P.cl, P.cu, c, dc);
        T g = G.c[0] ? G.c[0][e] : T(0);
        if (G.c[1]) g += G.c[1][e];
        if (G.c[2]) g += G.c[2][e];
        acc += g * dc;
      }
      gr[e] = acc;
    }
    // the unit vector's Jacobian: component j = sub - 1 by lanes 1..3 of the group (LPE >= 4)
    const int j = sub - 1;
    if (j >= 0 && j < 3) {
      T out = T(0);
      if (gu) {
        const T x = P.dl[3 * e], y = P.dl[3 * e + 1], zz = P.dl[3 * e + 2];
        const T a = gu[3 * e], b = gu[3 * e + 1], c = gu[3 * e + 2];
        const T gj = j == 0 ? a : j == 1 ? b : c;
        if (P.src[e] == P.dst[e]) {
          out = gj;
        } else {
          const T n = sqrt(x * x + y * y + zz * zz);
          const T dot = (x * a + y * b + zz * c) / n;
          const T uj = (j == 0 ? x : j == 1 ? y : zz) / n;
          out = (gj - uj * dot) / n;
        }
      }
      gdl[3 * e + j] = out;
    }
  }
}

// Second order of k_bwd (force-loss training): the VJP of (g_dl, g_r) = bwd(dl, r, gf, gC, gu) for
// cotangents (gg_dl, gg_r).  With u = dl/n (n = |dl|, non-self edges), P = I - u u^T, g_dl = P gu / n:
//   d_gf[k] = gg_r f_k'(r)      d_gC = gg_r C'(r)      d_r = gg_r (sum_k gf_k f_k''(r) + gC C''(r))
//   d_gu    = P gg_dl / n       d_dl = -[(u.gu) P gg + (u.gg) P gu + A u] / n^2,
//   A = gg.gu - (u.gg)(u.gu);   self edges: d_gu = gg_dl, d_dl = 0.  Output pointers may be NULL.
template <typename T>
__global__ __launch_bounds__(256) void k_bwd2(Cfg<T> P, const T* __restrict__ gf, const T* __restrict__ gC,
                                              const T* __restrict__ gu, const T* __restrict__ ggdl,
                                              const T* __restrict__ ggr, T* __restrict__ dgf, T* __restrict__ dgC,
                                              T* __restrict__ dgu, T* __restrict__ dr, T* __restrict__ ddl) {
  const int lane = lane_id();
  const int nw = gridDim.x * (blockDim.x / TMD_WAVE);
  for (int e = blockIdx.x * (blockDim.x / TMD_WAVE) + threadIdx.x / TMD_WAVE; e < P.E; e += nw) {
    const T r = P.r[e];
    const T g_r = ggr ? ggr[e] : T(0);
    T acc = T(0);
    if (dgf || (dr && gf)) {
      for (int k = lane; k < P.R; k += TMD_WAVE) {
        T v, dv, d2v;
        basis2(P, r, k, v, dv, d2v);
        if (dgf) dgf[(long long)e * P.R + k] = g_r * dv;
        if (gf) acc += gf[(long long)e * P.R + k] * d2v;
      }
      if (dr && gf) acc = wave_sum(acc);
    }
    if (lane != 0) continue;
    if (dgC || dr) {
      T c, dc, d2c;
      cosine_cutoff2<T>(r, P.cl, P.cu, c, dc, d2c);
      if (dgC) dgC[e] = g_r * dc;
      if (dr) dr[e] = g_r * (acc + (gC ? gC[e] * d2c : T(0)));
    }
    if (!dgu && !ddl) continue;
    const T a = ggdl ? ggdl[3 * e] : T(0), b = ggdl ? ggdl[3 * e + 1] : T(0), c = ggdl ? ggdl[3 * e + 2] : T(0);
    T o[3] = {a, b, c}, d[3] = {T(0), T(0), T(0)};
    if (P.src[e] != P.dst[e]) {
      const T x = P.dl[3 * e], y = P.dl[3 * e + 1], z = P.dl[3 * e + 2];
      const T n = sqrt(x * x + y * y + z * z);
      const T u[3] = {x / n, y / n, z / n};
      const T ug = u[0] * a + u[1] * b + u[2] * c;
      const T gv[3] = {gu ? gu[3 * e] : T(0), gu ? gu[3 * e + 1] : T(0), gu ? gu[3 * e + 2] : T(0)};
      const T uq = u[0] * gv[0] + u[1] * gv[1] + u[2] * gv[2];
      const T A = a * gv[0] + b * gv[1] + c * gv[2] - ug * uq;
      const T in2 = T(1) / (n * n);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const T pg = o[j] - u[j] * ug, pq = gv[j] - u[j] * uq;
        d[j] = -(uq * pg + ug * pq + A * u[j]) * in2;
        o[j] = pg / n;
      }
    }
    if (dgu) {
      dgu[3 * e] = o[0]; dgu[3 * e + 1] = o[1]; dgu[3 * e + 2] = o[2];
    }
    if (ddl) {
      ddl[3 * e] = d[0]; ddl[3 * e + 1] = d[1]; ddl[3 * e + 2] = d[2];
    }
  }
}

// d f_k / d r of the edges rows[p] (rows NULL: p itself), [n_rows][R]: the edge-feature derivative the
// ET force pass contracts with the projection gradient (et_stack, "dr mode")
template <typename T>
__global__ void k_deriv(Cfg<T> P, const int32_t* __restrict__ rows, int n_rows, T* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n_rows * P.R) return;
  const int p = (int)(i / P.R), k = (int)(i % P.R);
  const int e = rows ? rows[p] : p;
  T v, dv;
  basis(P, P.r[e], k, v, dv);
  out[i] = dv;
}

template <typename T>
static Cfg<T> make(int E, int R, int type, const int32_t* src, const int32_t* dst, const void* dl,
                   const void* r, const void* mu, const void* beta, double cl, double cu) {
  Cfg<T> P;
  P.E = E; P.R = R; P.type = type; P.src = src; P.dst = dst;
  P.dl = (const T*)dl; P.r = (const T*)r; P.mu = (const T*)mu; P.beta = (const T*)beta;
  P.cl = (T)cl; P.cu = (T)cu; P.alpha = (T)(5.0 / (cu - cl));
  return P;
}

}  // namespace geom
}  // namespace tmd

using namespace tmd;

static int geom_fwd(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src, const int32_t* dst,
                    const void* deltas, const void* dist, const void* mu, const void* beta, double cutoff_lower,
                    double cutoff_upper, void* rbf, void* cutoff, void* unit, const int32_t* rows, int n_rows,
                    void* rbf_rows, void* drbf_rows, void* stream) {
  if (n_edges <= 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  long long work = rbf ? (long long)n_edges * num_rbf : n_edges;
  if (rows) work = std::max(work, (long long)n_rows * num_rbf);
  const int tb = 256;
  dim3 g((unsigned)((work + tb - 1) / tb));
  if (dtype == TMDNET_F32) {
    auto P = geom::make<float>(n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower, cutoff_upper);
    hipLaunchKernelGGL(geom::k_fwd<float>, g, dim3(tb), 0, st, P, (float*)rbf, (float*)cutoff, (float*)unit, rows,
                       n_rows, (float*)rbf_rows, (float*)drbf_rows);
  } else if (dtype == TMDNET_F64) {
    auto P = geom::make<double>(n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower, cutoff_upper);
    hipLaunchKernelGGL(geom::k_fwd<double>, g, dim3(tb), 0, st, P, (double*)rbf, (double*)cutoff, (double*)unit, rows,
                       n_rows, (double*)rbf_rows, (double*)drbf_rows);
  } else {
    return kUnsupported;
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_edge_geom_fwd(int dtype, int n_edges, int num_rbf, int rbf_type,
                                    const int32_t* src, const int32_t* dst, const void* deltas,
                                    const void* dist, const void* mu, const void* beta,
                                    double cutoff_lower, double cutoff_upper, void* rbf, void* cutoff,
                                    void* unit, void* stream) {
  return geom_fwd(dtype, n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower, cutoff_upper,
                  rbf, cutoff, unit, nullptr, 0, nullptr, nullptr, stream);
}

extern "C" int tmdnet_edge_geom_fwd_rows(int dtype, int n_edges, int num_rbf, int rbf_type,
                                         const int32_t* src, const int32_t* dst, const void* deltas,
                                         const void* dist, const void* mu, const void* beta,
                                         double cutoff_lower, double cutoff_upper, void* rbf, void* cutoff,
                                         void* unit, const int32_t* rows, int n_rows, void* rbf_rows,
                                         void* stream) {
  if (!rows || n_rows < 0 || (n_rows > 0 && !rbf_rows)) return kBadArgument;
  return geom_fwd(dtype, n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower, cutoff_upper,
                  rbf, cutoff, unit, rows, n_rows, rbf_rows, nullptr, stream);
}

extern "C" int tmdnet_edge_geom_fwd_rows2(int dtype, int n_edges, int num_rbf, int rbf_type,
                                          const int32_t* src, const int32_t* dst, const void* deltas,
                                          const void* dist, const void* mu, const void* beta,
                                          double cutoff_lower, double cutoff_upper, void* rbf, void* cutoff,
                                          void* unit, const int32_t* rows, int n_rows, void* rbf_rows,
                                          void* drbf_rows, void* stream) {
  if (!rows || n_rows < 0 || (n_rows > 0 && (!rbf_rows || !drbf_rows))) return kBadArgument;
  return geom_fwd(dtype, n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower, cutoff_upper,
                  rbf, cutoff, unit, rows, n_rows, rbf_rows, drbf_rows, stream);
}

extern "C" int tmdnet_edge_geom_bwd_multi(int dtype, int n_edges, int num_rbf, int rbf_type,
                                          const int32_t* src, const int32_t* dst, const void* deltas,
                                          const void* dist, const void* mu, const void* beta,
                                          double cutoff_lower, double cutoff_upper, const void* grad_rbf,
                                          const void* grad_rbf2, const void* grad_rbf3, const void* grad_cutoff,
                                          const void* grad_cutoff2, const void* grad_cutoff3, const void* grad_unit,
                                          void* grad_dist, void* grad_deltas, void* stream) {
  if (n_edges <= 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const int tb = 256;
  // lane-parallel form when R splits into 16-byte lane chunks of 4..64 lanes per edge (every config: R = 16,
  // 32, 64); the wave-per-edge form otherwise.  Gradient rows must be 16-byte aligned (contiguous [E][R]).
  const int kpl = dtype == TMDNET_F32 ? 4 : 2, lpe = num_rbf / kpl;
  const bool aligned = !((((uintptr_t)grad_rbf) | ((uintptr_t)grad_rbf2) | ((uintptr_t)grad_rbf3)) & 15);
  const bool vec = num_rbf % kpl == 0 && (lpe == 4 || lpe == 8 || lpe == 16 || lpe == 32 || lpe == 64) && aligned;
  const long long waves = vec ? ((long long)n_edges * lpe + TMD_WAVE - 1) / TMD_WAVE : n_edges;
  const int blocks = (int)std::min<long long>((waves + 3) / 4, 256LL * 64);
#define TMD_GEOM_BWD(T_)                                                                                           \
  {                                                                                                                \
    auto P = geom::make<T_>(n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower, cutoff_upper); \
    geom::GIn<T_> G{{(const T_*)grad_rbf, (const T_*)grad_rbf2, (const T_*)grad_rbf3},                               \
                    {(const T_*)grad_cutoff, (const T_*)grad_cutoff2, (const T_*)grad_cutoff3}};                     \
    const T_* gu_ = (const T_*)grad_unit;                                                                          \
    T_* gr_ = (T_*)grad_dist;                                                                                      \
    T_* gd_ = (T_*)grad_deltas;                                                                                    \
    if (!grad_rbf && !grad_rbf2 && !grad_rbf3)                                                                    \
      hipLaunchKernelGGL(geom::k_bwd_e<T_>, dim3((unsigned)((n_edges + 255) / 256)), dim3(256), 0, st, P, G, gu_,     \
                         gr_, gd_);                                                                                \
    else if (!vec) hipLaunchKernelGGL(geom::k_bwd<T_>, dim3(blocks), dim3(tb), 0, st, P, G, gu_, gr_, gd_);       \
    else if (lpe == 4) hipLaunchKernelGGL((geom::k_bwd_v<T_, 4>), dim3(blocks), dim3(tb), 0, st, P, G, gu_, gr_, gd_);   \
    else if (lpe == 8) hipLaunchKernelGGL((geom::k_bwd_v<T_, 8>), dim3(blocks), dim3(tb), 0, st, P, G, gu_, gr_, gd_);   \
    else if (lpe == 16) hipLaunchKernelGGL((geom::k_bwd_v<T_, 16>), dim3(blocks), dim3(tb), 0, st, P, G, gu_, gr_, gd_); \
    else if (lpe == 32) hipLaunchKernelGGL((geom::k_bwd_v<T_, 32>), dim3(blocks), dim3(tb), 0, st, P, G, gu_, gr_, gd_); \
    else hipLaunchKernelGGL((geom::k_bwd_v<T_, 64>), dim3(blocks), dim3(tb), 0, st, P, G, gu_, gr_, gd_);                \
  }
  if (dtype == TMDNET_F32)
    TMD_GEOM_BWD(float)
  else if (dtype == TMDNET_F64)
    TMD_GEOM_BWD(double)
  else
    return kUnsupported;
#undef TMD_GEOM_BWD
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_edge_geom_bwd(int dtype, int n_edges, int num_rbf, int rbf_type,
                                    const int32_t* src, const int32_t* dst, const void* deltas,
                                    const void* dist, const void* mu, const void* beta,
                                    double cutoff_lower, double cutoff_upper, const void* grad_rbf,
                                    const void* grad_cutoff, const void* grad_unit, void* grad_dist,
                                    void* grad_deltas, void* stream) {
  return tmdnet_edge_geom_bwd_multi(dtype, n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta,
                                    cutoff_lower, cutoff_upper, grad_rbf, nullptr, nullptr, grad_cutoff, nullptr,
                                    nullptr, grad_unit, grad_dist, grad_deltas, stream);
}

extern "C" int tmdnet_rbf_deriv(int dtype, int num_rbf, int rbf_type, const void* dist, const void* mu,
                                const void* beta, double cutoff_lower, double cutoff_upper,
                                const int32_t* rows, int n_rows, void* out, void* stream) {
  if (n_rows < 0 || num_rbf <= 0 || !dist || !mu || !beta || !out) return kBadArgument;
  if (n_rows == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const long long work = (long long)n_rows * num_rbf;
  const dim3 g((unsigned)((work + 255) / 256));
  if (dtype == TMDNET_F32) {
    auto P = geom::make<float>(0, num_rbf, rbf_type, nullptr, nullptr, nullptr, dist, mu, beta, cutoff_lower,
                               cutoff_upper);
    hipLaunchKernelGGL(geom::k_deriv<float>, g, dim3(256), 0, st, P, rows, n_rows, (float*)out);
  } else if (dtype == TMDNET_F64) {
    auto P = geom::make<double>(0, num_rbf, rbf_type, nullptr, nullptr, nullptr, dist, mu, beta, cutoff_lower,
                                cutoff_upper);
    hipLaunchKernelGGL(geom::k_deriv<double>, g, dim3(256), 0, st, P, rows, n_rows, (double*)out);
  } else {
    return kUnsupported;
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_edge_geom_bwd2(int dtype, int n_edges, int num_rbf, int rbf_type,
                                     const int32_t* src, const int32_t* dst, const void* deltas,
                                     const void* dist, const void* mu, const void* beta,
                                     double cutoff_lower, double cutoff_upper, const void* grad_rbf,
                                     const void* grad_cutoff, const void* grad_unit, const void* gg_deltas,
                                     const void* gg_dist, void* d_grad_rbf, void* d_grad_cutoff,
                                     void* d_grad_unit, void* d_dist, void* d_deltas, void* stream) {
  if (n_edges < 0 || num_rbf <= 0 || !src || !dst || !deltas || !dist || !mu || !beta) return kBadArgument;
  if (n_edges == 0) return kOk;
  hipStream_t st = (hipStream_t)stream;
  const int tb = 256;
  const int blocks = (int)std::min<long long>(((long long)n_edges + 3) / 4, 256LL * 64);
#define TMD_GEOM_BWD2(T_)                                                                                      \
  {                                                                                                            \
    auto P = geom::make<T_>(n_edges, num_rbf, rbf_type, src, dst, deltas, dist, mu, beta, cutoff_lower,        \
                            cutoff_upper);                                                                     \
    hipLaunchKernelGGL(geom::k_bwd2<T_>, dim3(blocks), dim3(tb), 0, st, P, (const T_*)grad_rbf,                \
                       (const T_*)grad_cutoff, (const T_*)grad_unit, (const T_*)gg_deltas, (const T_*)gg_dist, \
                       (T_*)d_grad_rbf, (T_*)d_grad_cutoff, (T_*)d_grad_unit, (T_*)d_dist, (T_*)d_deltas);     \
  }
  if (dtype == TMDNET_F32)
    TMD_GEOM_BWD2(float)
  else if (dtype == TMDNET_F64)
    TMD_GEOM_BWD2(double)
  else
    return kUnsupported;
#undef TMD_GEOM_BWD2
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
