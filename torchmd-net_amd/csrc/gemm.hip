// Grouped small fp32 GEMM on the f32 MFMA (v_mfma_f32_16x16x4_f32) for the node-level feature mixes
// of the ET layer (reference EquivariantMultiHeadAttention q/k/v, vec_proj, o_proj Linears,
// torchmd_et.py:272-312, and their input gradients).  At QM9 batch size these GEMMs are tiny
// (M = atoms ~ 700, N, K <= 640): the library kernels they replace spend most of their ~6-8 us in
// a serial K loop over few workgroups.  Here:
//   * up to four independent problems share ONE launch (q|k|v with vec_proj in the forward,
//     vec_proj^T with [q|k|v]^T in the backward) -- one kernel boundary instead of two;
//   * a workgroup owns a 32 x 32 output tile with K split over its 4 (K < 256) or 16 waves, the
//     partial tiles summed in LDS; a wave issues all loads of its K slice up front (16-byte loads
//     along K): about one memory round trip per tile, then 2 x 2 MFMA tiles per k-step (a 64 x 64
//     tile with a quadrant per wave over the whole K measured slower);
//   * the K order inside an MFMA k-step is a free relabelling (A and B use the same one): lane l
//     feeds k = k0 + 4 (l >> 4) + j at step j, so a lane's four A (and NT-B) values of a 16-wide
//     K block are ONE float4 load.
//   C = beta * C + A op(B) + bias,  A [M][K] (lda), op(B) = B^T with B [N][K] (nn.Linear weight,
//   `trans_b`) or B [K][N];  exact fp32 (MFMA f32 is an fmaf chain; only the summation order differs
//   from the library GEMM).
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "tmdnet.h"

namespace tmd {
namespace gemm {

struct Prob {
  int M, N, K, lda, ldb, ldc, trans_b, beta;
  const float* A;
  const float* B;
  const float* bias;
  float* C;
  int tiles_n, tile0;
};

struct Group {
  Prob p[4];
  int n;
};

using f4 = float __attribute__((ext_vector_type(4)));

template <int KB>  // 16-wide K blocks per wave (unrolled, loads first)
__device__ __forceinline__ void wave_tile(const Prob& P, int r0, int c0, int kb0, int nkb, f4 (&acc)[2][2]) {
  const int lane = lane_id();
  const int lr = lane & 15, lk = lane >> 4;
  const int ra = min(r0 + lr, P.M - 1), rb = min(r0 + 16 + lr, P.M - 1);
  const int ca = min(c0 + lr, P.N - 1), cb = min(c0 + 16 + lr, P.N - 1);
  for (int b0 = 0; b0 < nkb; b0 += KB) {
    f4 a[KB][2], bb[KB][2];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int k = (kb0 + min(b0 + u, nkb - 1)) * 16 + 4 * lk;
      a[u][0] = *reinterpret_cast<const f4*>(P.A + (size_t)ra * P.lda + k);
      a[u][1] = *reinterpret_cast<const f4*>(P.A + (size_t)rb * P.lda + k);
      if (P.trans_b) {
        bb[u][0] = *reinterpret_cast<const f4*>(P.B + (size_t)ca * P.ldb + k);
        bb[u][1] = *reinterpret_cast<const f4*>(P.B + (size_t)cb * P.ldb + k);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bb[u][0][j] = P.B[(size_t)(k + j) * P.ldb + ca];
          bb[u][1][j] = P.B[(size_t)(k + j) * P.ldb + cb];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      if (b0 + u >= nkb) break;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0][j], bb[u][0][j], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0][j], bb[u][1][j], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1][j], bb[u][0][j], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1][j], bb[u][1][j], acc[1][1], 0, 0, 0);
      }
    }
  }
}

__device__ __forceinline__ void slice(const Prob& P, int r0, int c0, int kb0, int mine, f4 (&acc)[2][2]) {
  switch (min(mine, 8)) {  // a K slice of up to 8 blocks is loaded in one go
    case 0: break;
    case 1: wave_tile<1>(P, r0, c0, kb0, mine, acc); break;
    case 2: wave_tile<2>(P, r0, c0, kb0, mine, acc); break;
    case 3: wave_tile<3>(P, r0, c0, kb0, mine, acc); break;
    case 4: wave_tile<4>(P, r0, c0, kb0, mine, acc); break;
    case 5: wave_tile<5>(P, r0, c0, kb0, mine, acc); break;
    case 6: wave_tile<6>(P, r0, c0, kb0, mine, acc); break;
    case 7: wave_tile<7>(P, r0, c0, kb0, mine, acc); break;
    default: wave_tile<8>(P, r0, c0, kb0, mine, acc); break;
  }
}

__device__ __forceinline__ void store(const Prob& P, int gr, int gc, float v) {
  if (gr >= P.M || gc >= P.N) return;
  if (P.bias) v += P.bias[gc];
  float* out = P.C + (size_t)gr * P.ldc + gc;
  if (P.beta) v += *out;
  *out = v;
}

template <int NW>  // waves per 32 x 32 tile, K split NW ways
__global__ __launch_bounds__(NW * 64) void k_gemm(Group G) {
  __shared__ float part[NW][32][33];
  int pi = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < G.n && (int)blockIdx.x >= G.p[i].tile0) pi = i;
  const Prob& P = G.p[pi];
  const int t = blockIdx.x - P.tile0;
  const int w = threadIdx.x / TMD_WAVE, lane = lane_id();
  const int nkb = P.K / 16;  // 16-wide K blocks
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // C/D map of the 16x16 MFMA tile: col = lane & 15, row = 4 (lane >> 4) + i
  const int r0 = (t / P.tiles_n) * 32, c0 = (t % P.tiles_n) * 32;
  const int per = (nkb + NW - 1) / NW;  // blocks per wave
  const int kb0 = w * per;
  slice(P, r0, c0, kb0, max(0, min(per, nkb - kb0)), acc);
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][bi * 16 + 4 * (lane >> 4) + i][bj * 16 + (lane & 15)] = acc[bi][bj][i];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += blockDim.x) {
    const int r = e >> 5, c = e & 31;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) v += part[i][r][c];
    store(P, r0 + r, c0 + c, v);
  }
}

}  // namespace gemm
}  // namespace tmd

using namespace tmd;

extern "C" int tmdnet_gemm_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream) {
  if (n_problems < 1 || n_problems > 4 || !dims || !ptrs) return kBadArgument;
  gemm::Group G{};
  G.n = n_problems;
  int tiles = 0;
  for (int i = 0; i < n_problems; ++i) {
    const int* d = dims + 8 * i;
    gemm::Prob& P = G.p[i];
    P.M = d[0]; P.N = d[1]; P.K = d[2]; P.lda = d[3]; P.ldb = d[4]; P.ldc = d[5];
    P.trans_b = d[6]; P.beta = d[7];
    P.A = (const float*)ptrs[4 * i];
    P.B = (const float*)ptrs[4 * i + 1];
    P.bias = (const float*)ptrs[4 * i + 2];
    P.C = (float*)ptrs[4 * i + 3];
    if (P.M <= 0 || P.N <= 0 || P.K <= 0 || !P.A || !P.B || !P.C) return kBadArgument;
    if (P.K % 64 || P.lda % 4 || (P.trans_b && P.ldb % 4) || P.lda < P.K || P.ldc < P.N) return kUnsupported;
    if ((((uintptr_t)P.A) & 15) || (P.trans_b && (((uintptr_t)P.B) & 15))) return kUnsupported;
    // (a 64 x 64 tile with the whole K per wave measured slower for every ET shape at QM9 size --
    // 16.5 vs 13 us for [q|k|v] + vec_proj: f32 MFMA is 1/16 of the bf16 rate, so the per-wave MFMA
    // chain, not the loads, sets the tile time; split K keeps four or more waves on every tile)
    const int tile = 32;
    P.tiles_n = (P.N + tile - 1) / tile;
    P.tile0 = tiles;
    tiles += ((P.M + tile - 1) / tile) * P.tiles_n;
  }
  // K split over 16 waves from K = 256 (the backward's K = 3H / 5H products): a wave's slice is 2-3
  // K blocks, one load batch, and 4x the waves hide the load latency (4 waves below: the K = H
  // mixes).  Measured C2 step: 4/4 waves 1.062 ms, 4/8 1.044, 4/16 1.039, 2/16 1.064, 8/8 1.069.
  static int nw_small = 4, nw_large = 16;  // TMDNET_GEMM_NW="small,large" (tuning)
  static const bool env_read = [] {
    if (const char* e = getenv("TMDNET_GEMM_NW")) sscanf(e, "%d,%d", &nw_small, &nw_large);
    return true;
  }();
  (void)env_read;
  int kmax = 0;
  for (int i = 0; i < n_problems; ++i) kmax = max(kmax, G.p[i].K);
  const int nw = kmax >= 256 ? nw_large : nw_small;
  hipStream_t st = (hipStream_t)stream;
  if (nw <= 2) hipLaunchKernelGGL(gemm::k_gemm<2>, dim3(tiles), dim3(128), 0, st, G);
  else if (nw >= 16) hipLaunchKernelGGL(gemm::k_gemm<16>, dim3(tiles), dim3(1024), 0, st, G);
  else if (nw >= 8) hipLaunchKernelGGL(gemm::k_gemm<8>, dim3(tiles), dim3(512), 0, st, G);
  else hipLaunchKernelGGL(gemm::k_gemm<4>, dim3(tiles), dim3(256), 0, st, G);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
