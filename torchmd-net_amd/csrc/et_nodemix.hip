// The node mixes of an ET layer with the elementwise passes between them folded in (reference
// EquivariantMultiHeadAttention.forward, models/torchmd_et.py:262-312, and the residual updates of
// TorchMD_ET.forward, torchmd_et.py:181-184).  At QM9 size every launch of the layer is latency-bound
// (~2 us of graph-launch floor plus one or two dependent memory round trips), so the two kernels here
// remove the stand-alone epilogue + LayerNorm pass of every layer:
//
//   k_oproj_epi: o = x_agg W_o^T + b_o on the f32 MFMA, one workgroup per 32 nodes x 16 CHANNELS: its
//     three 16-column blocks are the channel slice's o1 / o2 / o3 (rows c, H + c, 2H + c of W_o), so the
//     layer epilogue runs on the tile's own output (x_out = x + (vec1 . vec2) o2 + o3, vec_out = vec +
//     vec3 o1 + vec_agg) -- o is written too (the backward reads it).  The epilogue operands are loaded
//     before the K loop, under its latency.
//   k_ln_mix: [q|k|v] = LayerNorm(x) W^T + b and vec_proj(vec) in one grouped launch; a 32-row tile of
//     the first problem spans the whole K = H (split over its 4 waves), so the tile forms the row
//     statistics itself (two passes: mean, then centred variance, across waves through LDS) and
//     normalises its A fragments in registers before the MFMAs.  The first column tile writes xn,
//     mean and rstd (the backward's and the weight gradients' operands).
//
// Both keep tmdnet_gemm_f32's per-wave K slices and its wave-order partial sum (+ bias after), so o is
// bit-identical to the unfused o_proj GEMM, and x_out / vec_out to tmdnet_et_epilogue_ln_fwd's; the
// LayerNorm statistics are the same two-pass formulas summed in another order (last-ulp differences).
#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace nodemix {

using f4 = float __attribute__((ext_vector_type(4)));
constexpr int kNW = 4;  // waves per workgroup, K split kNW ways (H / 64 16-wide blocks per wave)

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// ---------------------------------------------------------------------------------------------------
struct EpiArgs {
  int M, H;
  const float *xa, *w, *b;               // x_agg [M][H], W_o [3H][H], b_o [3H]
  const float *x, *vec, *vecp, *veca;    // [M][H], [M][3][H], [M][3][3H] (nullable: first layer), [M][3][H]
  float *o, *xo, *veco;                  // [M][3H], [M][H], [M][3][H]
};

template <int PER>
__global__ __launch_bounds__(kNW * 64) void k_oproj_epi(EpiArgs A) {
  __shared__ float part[kNW][32][49];
  const int nch = A.H / 16;
  const int r0 = (blockIdx.x / nch) * 32, ch0 = (blockIdx.x % nch) * 16;
  const int tid = threadIdx.x, w = tid / 64, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int H = A.H;
  // the epilogue operands of this thread's two (node, channel) items, in flight under the K loop
  float ex[2], ev[2][3], eva[2][3], ep[2][9];
  const bool hv = A.vecp != nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i, t = min(r0 + (e >> 4), A.M - 1), ch = ch0 + (e & 15);
    ex[i] = A.x[(size_t)t * H + ch];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      eva[i][a] = A.veca[((size_t)t * 3 + a) * H + ch];
      ev[i][a] = hv ? A.vec[((size_t)t * 3 + a) * H + ch] : 0.f;
#pragma unroll
      for (int s = 0; s < 3; ++s) ep[i][3 * a + s] = hv ? A.vecp[(size_t)t * 9 * H + a * 3 * H + s * H + ch] : 0.f;
    }
  }
  const int ra = min(r0 + lr, A.M - 1), rb = min(r0 + 16 + lr, A.M - 1);
  f4 a[PER][2], bb[PER][3];
  const int kb0 = w * PER;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int k = (kb0 + u) * 16 + 4 * lk;
    a[u][0] = ld4(A.xa + (size_t)ra * H + k);
    a[u][1] = ld4(A.xa + (size_t)rb * H + k);
#pragma unroll
    for (int s = 0; s < 3; ++s) bb[u][s] = ld4(A.w + (size_t)(s * H + ch0 + lr) * H + k);
  }
  f4 acc[2][3];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int s = 0; s < 3; ++s) acc[x][s] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < PER; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int s = 0; s < 3; ++s)
          acc[x][s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][x][j], bb[u][s][j], acc[x][s], 0, 0, 0);
  // C map of a 16 x 16 block: row 4 (lane >> 4) + i, column lane & 15
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][16 * x + 4 * lk + i][16 * s + lr] = acc[x][s][i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i, r = e >> 4, c = e & 15;
    const int t = r0 + r, ch = ch0 + c;
    if (t >= A.M) continue;
    float o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll
    for (int q = 0; q < kNW; ++q) {
      o1 += part[q][r][c];
      o2 += part[q][r][16 + c];
      o3 += part[q][r][32 + c];
    }
    o1 += A.b[ch];
    o2 += A.b[H + ch];
    o3 += A.b[2 * H + ch];
    float* ot = A.o + (size_t)t * 3 * H;
    ot[ch] = o1;
    ot[H + ch] = o2;
    ot[2 * H + ch] = o3;
    float xc = ex[i];
    if (hv) {
      float dot = 0.f;
#pragma unroll
      for (int a = 0; a < 3; ++a) dot += ep[i][3 * a] * ep[i][3 * a + 1];
      xc += dot * o2 + o3;
#pragma unroll
      for (int a = 0; a < 3; ++a) A.veco[((size_t)t * 3 + a) * H + ch] = ev[i][a] + ep[i][3 * a + 2] * o1 + eva[i][a];
    } else {
      xc += o3;
#pragma unroll
      for (int a = 0; a < 3; ++a) A.veco[((size_t)t * 3 + a) * H + ch] = eva[i][a];
    }
    A.xo[(size_t)t * H + ch] = xc;
  }
}

// ---------------------------------------------------------------------------------------------------
struct MixProb {
  int M, N, tiles_n, tile0;
  const float *A, *W, *bias;  // A [M][H], W [N][H] (nn.Linear weight), bias [N] or null
  float* C;                   // [M][N]
};
struct MixArgs {
  int H, n;
  MixProb p[2];
  const float *lw, *lb;  // problem 0's LayerNorm (affine)
  float eps;
  float *xn, *mean, *rstd;
};

template <int PER>
__global__ __launch_bounds__(kNW * 64) void k_ln_mix(MixArgs A) {
  __shared__ float part[kNW][32][33];
  __shared__ float red[2][kNW][32];
  const int pi = (A.n > 1 && (int)blockIdx.x >= A.p[1].tile0) ? 1 : 0;
  const MixProb& P = A.p[pi];
  const int t = blockIdx.x - P.tile0;
  const int r0 = (t / P.tiles_n) * 32, c0 = (t % P.tiles_n) * 32;
  const int tid = threadIdx.x, w = tid / 64, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const int H = A.H;
  const int ra = min(r0 + lr, P.M - 1), rb = min(r0 + 16 + lr, P.M - 1);
  const int ca = min(c0 + lr, P.N - 1), cb = min(c0 + 16 + lr, P.N - 1);
  const int kb0 = w * PER;
  f4 a[PER][2], bb[PER][2];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int k = (kb0 + u) * 16 + 4 * lk;
    a[u][0] = ld4(P.A + (size_t)ra * H + k);
    a[u][1] = ld4(P.A + (size_t)rb * H + k);
    bb[u][0] = ld4(P.W + (size_t)ca * H + k);
    bb[u][1] = ld4(P.W + (size_t)cb * H + k);
  }
  if (pi == 0) {  // LayerNorm of the tile's rows (block-uniform branch)
    float s[2] = {0.f, 0.f};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
#pragma unroll
      for (int u = 0; u < PER; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[x] += a[u][x][j];
      s[x] += __shfl_xor(s[x], 16);
      s[x] += __shfl_xor(s[x], 32);
      if (lk == 0) red[0][w][16 * x + lr] = s[x];
    }
    __syncthreads();
    float mu[2], rs[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < kNW; ++q) v += red[0][q][16 * x + lr];
      mu[x] = v / float(H);
      float d = 0.f;
#pragma unroll
      for (int u = 0; u < PER; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) d += (a[u][x][j] - mu[x]) * (a[u][x][j] - mu[x]);
      d += __shfl_xor(d, 16);
      d += __shfl_xor(d, 32);
      if (lk == 0) red[1][w][16 * x + lr] = d;
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < kNW; ++q) v += red[1][q][16 * x + lr];
      rs[x] = 1.f / sqrtf(v / float(H) + A.eps);
    }
    const bool wr = c0 == 0;  // the first column tile stores xn / mean / rstd
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int k = (kb0 + u) * 16 + 4 * lk;
      const f4 g = ld4(A.lw + k), h = ld4(A.lb + k);
#pragma unroll
      for (int x = 0; x < 2; ++x) {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[u][x][j] = (a[u][x][j] - mu[x]) * rs[x] * g[j] + h[j];
        const int row = r0 + 16 * x + lr;
        if (wr && row < P.M) *reinterpret_cast<f4*>(A.xn + (size_t)row * H + k) = a[u][x];
      }
    }
    if (wr && w == 0 && lk == 0) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int row = r0 + 16 * x + lr;
        if (row < P.M) {
          A.mean[row] = mu[x];
          A.rstd[row] = rs[x];
        }
      }
    }
  }
  f4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < PER; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][x][j], bb[u][y][j], acc[x][y], 0, 0, 0);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][16 * x + 4 * lk + i][16 * y + lr] = acc[x][y][i];
  __syncthreads();
  for (int e = tid; e < 32 * 32; e += kNW * 64) {
    const int r = e >> 5, c = e & 31;
    const int gr = r0 + r, gc = c0 + c;
    if (gr >= P.M || gc >= P.N) continue;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < kNW; ++q) v += part[q][r][c];
    if (P.bias) v += P.bias[gc];
    P.C[(size_t)gr * P.N + gc] = v;
  }
}

// ---------------------------------------------------------------------------------------------------
// The force pass's mirror image: k_lnbwd_oproj = the LayerNorm backward of layer l (+ its residual), the
// epilogue backward of layer l-1 and g_xa(l-1) = g_o(l-1) W_o(l-1) in one launch (replaces
// tmdnet_ln_bwd_epilogue + tmdnet_gemm_f32 of the o_proj input gradient).  A workgroup owns 32 nodes x
// 32 columns of g_xa, K = 3H: it forms its 32 rows of g_o itself -- 32 threads per node row, 4 channels
// each, every operand of the row (g_xn, x, the residual, g_vec, vecp, o) loaded in one round trip, the
// LayerNorm row sums over the row's 32 lanes -- into LDS as the GEMM's A tile.  The first column tile
// also stores g_x, g_o and g_vecp (the next layer's and the recorded backward's operands).  H = 128.
constexpr int kLH = 128;
constexpr int kLNW = 16;   // waves (the prologue: 2 node rows per wave)
constexpr int kLMW = 12;   // of which the GEMM's: 24 16-wide K blocks, 2 per wave
constexpr int kLAS = 3 * kLH + 4;  // A-tile row stride (floats)

struct LnBwdArgs {
  int M;
  const float *gxn, *x, *mean, *rstd, *lw, *gres;  // gres nullable (no residual: the model's out_norm)
  const float *gvec, *vecp, *o, *w;                 // vecp nullable (layer l-1 = 0: vec == 0)
  float *gx, *gvecp, *go, *gxa;
};

__global__ __launch_bounds__(kLNW * 64) void k_lnbwd_oproj(LnBwdArgs A) {
  __shared__ __attribute__((aligned(16))) float At[32 * kLAS];
  __shared__ float part[kLMW][32][33];
  constexpr int H = kLH, ntc = H / 32;
  const int r0 = (blockIdx.x / ntc) * 32, c0 = (blockIdx.x % ntc) * 32;
  const int tid = threadIdx.x, w = tid / 64, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  // the GEMM's B fragments (W_o [3H][H], rows k, columns c0 + 16 y + lr): independent of the prologue
  float bb[2][2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bb[u][y][j] = w < kLMW ? A.w[(size_t)((2 * w + u) * 16 + 4 * lk + j) * H + c0 + 16 * y + lr] : 0.f;
  // prologue: node row r, channels 4q .. 4q + 3
  const int r = tid >> 5, q = tid & 31, c = 4 * q;
  const int t = min(r0 + r, A.M - 1);
  const bool hv = A.vecp != nullptr;
  const f4 gn = ld4(A.gxn + (size_t)t * H + c), xv = ld4(A.x + (size_t)t * H + c), lw = ld4(A.lw + c);
  const f4 gr = A.gres ? ld4(A.gres + (size_t)t * H + c) : f4{0.f, 0.f, 0.f, 0.f};
  f4 gv[3], v1[3], v2[3], v3[3], o1, o2;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    gv[a] = ld4(A.gvec + ((size_t)t * 3 + a) * H + c);
    if (hv) {
      const float* vp = A.vecp + (size_t)t * 9 * H + a * 3 * H + c;
      v1[a] = ld4(vp);
      v2[a] = ld4(vp + H);
      v3[a] = ld4(vp + 2 * H);
    }
  }
  if (hv) {
    o1 = ld4(A.o + (size_t)t * 3 * H + c);
    o2 = ld4(A.o + (size_t)t * 3 * H + H + c);
  }
  const float mu = A.mean[t], rs = A.rstd[t];
  f4 xh, gh;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xh[i] = (xv[i] - mu) * rs;
    gh[i] = gn[i] * lw[i];
    s1 += gh[i];
    s2 += gh[i] * xh[i];
  }
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) {  // the row's 32 lanes (one half of the wave)
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  const float m1 = s1 / float(H), m2 = s2 / float(H);
  const bool wr = c0 == 0 && r0 + r < A.M;
  float* at = At + r * kLAS;
  f4 g, gdot, go1;
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = gr[i] + rs * (gh[i] - m1 - xh[i] * m2);
  if (hv) {
    f4 dot = f4{0.f, 0.f, 0.f, 0.f};
    go1 = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dot[i] += v1[a][i] * v2[a][i];
        go1[i] += gv[a][i] * v3[a][i];
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) gdot[i] = g[i] * dot[i];
    if (wr) {
      float* gvp = A.gvecp + (size_t)t * 9 * H + c;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        f4 e1, e2, e3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float gd = g[i] * o2[i];
          e1[i] = gd * v2[a][i];
          e2[i] = gd * v1[a][i];
          e3[i] = gv[a][i] * o1[i];
        }
        *reinterpret_cast<f4*>(gvp + a * 3 * H) = e1;
        *reinterpret_cast<f4*>(gvp + a * 3 * H + H) = e2;
        *reinterpret_cast<f4*>(gvp + a * 3 * H + 2 * H) = e3;
      }
    }
  } else {
    go1 = gdot = f4{0.f, 0.f, 0.f, 0.f};
  }
  *reinterpret_cast<f4*>(at + c) = go1;
  *reinterpret_cast<f4*>(at + H + c) = gdot;
  *reinterpret_cast<f4*>(at + 2 * H + c) = g;
  if (wr) {
    *reinterpret_cast<f4*>(A.gx + (size_t)t * H + c) = g;
    float* gt = A.go + (size_t)t * 3 * H + c;
    *reinterpret_cast<f4*>(gt) = go1;
    *reinterpret_cast<f4*>(gt + H) = gdot;
    *reinterpret_cast<f4*>(gt + 2 * H) = g;
  }
  __syncthreads();
  if (w < kLMW) {
    f4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = (2 * w + u) * 16 + 4 * lk;
      const f4 a0 = *reinterpret_cast<const f4*>(At + lr * kLAS + k);
      const f4 a1 = *reinterpret_cast<const f4*>(At + (16 + lr) * kLAS + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], bb[u][0][j], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], bb[u][1][j], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], bb[u][0][j], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], bb[u][1][j], acc[1][1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[w][16 * x + 4 * lk + i][16 * y + lr] = acc[x][y][i];
  }
  __syncthreads();
  {
    const int rr = tid >> 5, cc = tid & 31;
    if (r0 + rr < A.M) {
      float v = 0.f;
#pragma unroll
      for (int qq = 0; qq < kLMW; ++qq) v += part[qq][rr][cc];
      A.gxa[(size_t)(r0 + rr) * H + c0 + cc] = v;
    }
  }
}

inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

}  // namespace nodemix
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_et_oproj_epilogue_f32(int n_nodes, int hidden, const void* x_agg, const void* o_w,
                                            const void* o_b, const void* x, const void* vec, const void* vecp,
                                            const void* vec_agg, void* o, void* x_out, void* vec_out,
                                            void* stream) {
  if (n_nodes < 0 || hidden <= 0) return kBadArgument;
  if (n_nodes == 0) return kOk;
  if (!x_agg || !o_w || !o_b || !x || !vec_agg || !o || !x_out || !vec_out || (vecp && !vec)) return kBadArgument;
  if (hidden % 64 || hidden > 256) return kUnsupported;
  if (!nodemix::aligned16(x_agg) || !nodemix::aligned16(o_w)) return kUnsupported;
  nodemix::EpiArgs A{n_nodes, hidden, (const float*)x_agg, (const float*)o_w, (const float*)o_b,
                     (const float*)x, (const float*)vec, (const float*)vecp, (const float*)vec_agg,
                     (float*)o, (float*)x_out, (float*)vec_out};
  const dim3 g((unsigned)(((n_nodes + 31) / 32) * (hidden / 16)));
  hipStream_t st = (hipStream_t)stream;
  switch (hidden / 64) {
    case 1: hipLaunchKernelGGL(nodemix::k_oproj_epi<1>, g, dim3(256), 0, st, A); break;
    case 2: hipLaunchKernelGGL(nodemix::k_oproj_epi<2>, g, dim3(256), 0, st, A); break;
    case 3: hipLaunchKernelGGL(nodemix::k_oproj_epi<3>, g, dim3(256), 0, st, A); break;
    default: hipLaunchKernelGGL(nodemix::k_oproj_epi<4>, g, dim3(256), 0, st, A); break;
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_et_ln_mix_f32(int n_nodes, int hidden, const void* x, const void* ln_w, const void* ln_b,
                                    double eps, const void* w, const void* b, int n_out, void* out, void* xn,
                                    void* mean, void* rstd, const void* vec, const void* vec_w, int n_vec_out,
                                    void* vec_out, void* stream) {
  if (n_nodes < 0 || hidden <= 0 || n_out <= 0) return kBadArgument;
  if (n_nodes == 0) return kOk;
  if (!x || !ln_w || !ln_b || !w || !out || !xn || !mean || !rstd) return kBadArgument;
  if (vec && (!vec_w || !vec_out || n_vec_out <= 0)) return kBadArgument;
  if (hidden % 64 || hidden > 256) return kUnsupported;
  for (const void* p : {x, w, ln_w, ln_b, (const void*)xn, vec, vec_w})
    if (p && !nodemix::aligned16(p)) return kUnsupported;
  nodemix::MixArgs A{};
  A.H = hidden;
  A.n = vec ? 2 : 1;
  A.lw = (const float*)ln_w;
  A.lb = (const float*)ln_b;
  A.eps = (float)eps;
  A.xn = (float*)xn;
  A.mean = (float*)mean;
  A.rstd = (float*)rstd;
  A.p[0] = {n_nodes, n_out, (n_out + 31) / 32, 0, (const float*)x, (const float*)w, (const float*)b, (float*)out};
  int tiles = ((n_nodes + 31) / 32) * A.p[0].tiles_n;
  if (vec) {
    A.p[1] = {3 * n_nodes, n_vec_out, (n_vec_out + 31) / 32, tiles, (const float*)vec, (const float*)vec_w, nullptr,
              (float*)vec_out};
    tiles += ((3 * n_nodes + 31) / 32) * A.p[1].tiles_n;
  }
  hipStream_t st = (hipStream_t)stream;
  switch (hidden / 64) {
    case 1: hipLaunchKernelGGL(nodemix::k_ln_mix<1>, dim3(tiles), dim3(256), 0, st, A); break;
    case 2: hipLaunchKernelGGL(nodemix::k_ln_mix<2>, dim3(tiles), dim3(256), 0, st, A); break;
    case 3: hipLaunchKernelGGL(nodemix::k_ln_mix<3>, dim3(tiles), dim3(256), 0, st, A); break;
    default: hipLaunchKernelGGL(nodemix::k_ln_mix<4>, dim3(tiles), dim3(256), 0, st, A); break;
  }
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_et_lnbwd_oproj_f32(int n_nodes, int hidden, const void* grad_xn, const void* x,
                                         const void* mean, const void* rstd, const void* ln_w, const void* grad_res,
                                         const void* grad_vec, const void* vecp, const void* o, const void* o_w,
                                         void* grad_x, void* grad_vecp, void* grad_o, void* grad_xa, void* stream) {
  if (n_nodes < 0 || hidden <= 0) return kBadArgument;
  if (n_nodes == 0) return kOk;
  if (!grad_xn || !x || !mean || !rstd || !ln_w || !grad_vec || !o_w || !grad_x || !grad_o || !grad_xa)
    return kBadArgument;
  if (vecp && (!o || !grad_vecp)) return kBadArgument;
  if (hidden != nodemix::kLH) return kUnsupported;
  for (const void* p : {grad_xn, x, ln_w, grad_res, grad_vec, vecp, o, (const void*)grad_x, (const void*)grad_vecp,
                        (const void*)grad_o})
    if (p && !nodemix::aligned16(p)) return kUnsupported;
  nodemix::LnBwdArgs A{n_nodes, (const float*)grad_xn, (const float*)x, (const float*)mean, (const float*)rstd,
                       (const float*)ln_w, (const float*)grad_res, (const float*)grad_vec, (const float*)vecp,
                       (const float*)o, (const float*)o_w, (float*)grad_x, (float*)grad_vecp, (float*)grad_o,
                       (float*)grad_xa};
  const dim3 g((unsigned)(((n_nodes + 31) / 32) * (nodemix::kLH / 32)));
  hipLaunchKernelGGL(nodemix::k_lnbwd_oproj, g, dim3(nodemix::kLNW * 64), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
