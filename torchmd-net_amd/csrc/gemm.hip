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
  // epilogue extensions (tmdnet_gemm_ex_f32; all off for tmdnet_gemm_f32): v = acc + bias (+ C) ->
  // pre[r][c] = v (the pre-activation a backward needs) -> v = silu(v) (act) -> v *= rscale[r] ->
  // v *= silu'(dpre[r][c]) (a backward chain: the next-lower layer's activation derivative) -> C
  int act, ldx;  // ldx: row stride of pre / dpre
  float* pre;
  const float* rscale;
  const float* dpre;
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

// KMAX: 8 blocks per load batch for the 4- / 8-wave kernels; 4 for the 16-wave kernel, whose
// 1024-thread blocks cap a wave at 128 VGPRs (an 8-block batch alone is 128 VGPRs of loads: it
// spilled 75 VGPRs; the 16-wave slices of the ET shapes are 2-3 blocks anyway)
template <int KMAX>
__device__ __forceinline__ void slice(const Prob& P, int r0, int c0, int kb0, int mine, f4 (&acc)[2][2]) {
  switch (min(mine, KMAX)) {  // a K slice of up to KMAX blocks is loaded in one go
    case 0: break;
    case 1: wave_tile<1>(P, r0, c0, kb0, mine, acc); break;
    case 2: wave_tile<2>(P, r0, c0, kb0, mine, acc); break;
    case 3: wave_tile<3>(P, r0, c0, kb0, mine, acc); break;
    case 4: wave_tile<4>(P, r0, c0, kb0, mine, acc); break;
    case 5: if constexpr (KMAX >= 5) wave_tile<5>(P, r0, c0, kb0, mine, acc); break;
    case 6: if constexpr (KMAX >= 6) wave_tile<6>(P, r0, c0, kb0, mine, acc); break;
    case 7: if constexpr (KMAX >= 7) wave_tile<7>(P, r0, c0, kb0, mine, acc); break;
    default: if constexpr (KMAX >= 8) wave_tile<8>(P, r0, c0, kb0, mine, acc); break;
  }
}

// EX: the tmdnet_gemm_ex_f32 epilogue switches; plain tmdnet_gemm_f32 launches compile them out
// (they cost the latency-bound node mixes ~5 % per launch when tested per element)
template <bool EX>
__device__ __forceinline__ void store(const Prob& P, int gr, int gc, float v) {
  if (gr >= P.M || gc >= P.N) return;
  if (P.bias) v += P.bias[gc];
  float* out = P.C + (size_t)gr * P.ldc + gc;
  if (P.beta) v += *out;
  if constexpr (EX) {
    if (P.pre) P.pre[(size_t)gr * P.ldx + gc] = v;
    if (P.act) v = Silu<float>(v).s;
    if (P.rscale) v *= P.rscale[gr];
    if (P.dpre) {
      const float x = P.dpre[(size_t)gr * P.ldx + gc];
      v *= Silu<float>(x).d(x);
    }
  }
  *out = v;
}

// NW waves per 32 x 32 tile, K split NW ways; KMAX = the load batch (K blocks) the launch's longest
// per-wave slice needs: the register file is sized for the largest batch the kernel can issue, so a
// K = 128 mix (2 blocks per wave) compiled with an 8-block batch ran at 160 VGPRs = 2 waves per SIMD
template <int NW, int KMAX, bool EX = true>
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
  slice<KMAX>(P, r0, c0, kb0, max(0, min(per, nkb - kb0)), acc);
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
    store<EX>(P, r0 + r, c0 + c, v);
  }
}

// ---------------------------------------------------------------------------------------------------
// Grouped "TN" fp32 MFMA GEMM for weight gradients: C (+)= A^T B summed over ROWS (K = atoms, edges,
// ...), A [K][M], B [K][N], C [M][N] -- the shape of every Linear's weight gradient (sum over samples
// of g (x) input).  The library picks a few-workgroup tile with a serial K loop for these (e.g. 64 us
// for [128 x 678]^T [678 x 257]); here a workgroup owns a 32 x 32 tile of C and splits K over its waves
// (partials summed in LDS), and up to TN_MAX problems (every layer's [q|k|v] / o_proj / vec_proj
// weights, or a head's six weights) share ONE launch.  Per problem, a second row segment (A2, B2, K2)
// continues the K sum -- e.g. the force-loss second order's extra terms of the same weight -- and
// `ones` (per segment) makes B's column N-1 a column of ones, i.e. C's last column the bias gradient
// (sum of A over the rows).  Loads are scalar along the rows (the contiguous direction of A and B is
// the output dimension): one k row of a 32-wide tile is a 128-byte segment.
constexpr int TN_MAX = 32;
// 16-row blocks whose loads are issued together per iteration (the loop is one memory round trip per
// 16 * TN_UB rows: a wave's row slice of an edge sum is ~800-1600 rows)
constexpr int TN_UB = 4;

struct ProbTN {
  int M, N, K, K2, lda, ldb, lda2, ldb2, ldc, beta, ones1, ones2, tiles_n, tile0;
  int onehot;  // A is an int64 index vector: A[k][m] = (A[k] == m) (embedding-table gradients)
  // 64-tile kernels: this problem's split-K factor, first workgroup, tile count, first partial tile
  int S, wg0, ntiles;
  long long part0;
  const float* A;
  const float* B;
  const float* A2;
  const float* B2;
  float* C;
  float* Cb;  // non-NULL: column N-1 (the ones / bias column) goes to Cb[m] instead of C[m][N-1]
  const int* rows;  // non-NULL (64-tile kernels): only rows < *rows of each segment are summed (device count)
};

struct GroupTN {
  ProbTN p[TN_MAX];
  int n;
  int S;        // split-K factor: S workgroups per tile, each over a chunk of the rows
  float* part;  // S > 1: partial tiles [tiles][S][32 * 32], summed in order by k_tn_reduce
};

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_gemm_tn(GroupTN G) {
  __shared__ float part[NW][32][33];
  const int tg = blockIdx.x / G.S, sk = blockIdx.x % G.S;  // tile, row chunk
  int pi = 0;
  for (int i = 1; i < G.n; ++i)
    if (tg >= G.p[i].tile0) pi = i;
  const ProbTN& P = G.p[pi];
  const int t = tg - P.tile0;
  const int w = threadIdx.x / TMD_WAVE, lane = lane_id();
  const int lr = lane & 15, lk = lane >> 4;
  const int r0 = (t / P.tiles_n) * 32, c0 = (t % P.tiles_n) * 32;
  // (a device row count shortens both segments: the chunks split the rows actually summed)
  const int cnt = P.rows ? max(0, *P.rows) : P.K + P.K2;
  const int K1 = min(P.K, cnt), KT = K1 + min(P.K2, cnt);
  // this workgroup's rows (16-row blocks split evenly over the S chunks), then this wave's share
  const int nkt = (KT + 15) / 16, cper = (nkt + G.S - 1) / G.S;
  const int c_lo = min(KT, sk * cper * 16), c_hi = min(KT, (sk + 1) * cper * 16);
  const int nkb = (c_hi - c_lo + 15) / 16, per = (nkb + NW - 1) / NW;
  const int k_lo = min(c_hi, c_lo + w * per * 16), k_hi = min(c_hi, c_lo + (w + 1) * per * 16);
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int ma = r0 + lr, mb = r0 + 16 + lr, na = c0 + lr, nb = c0 + 16 + lr;
  const bool va = ma < P.M, vb = mb < P.M;
  const bool anyones = P.ones1 || P.ones2;
  for (int seg = 0; seg < 2; ++seg) {  // the two row segments (wave-uniform)
    const int s0 = seg ? K1 : 0, s1 = seg ? KT : K1;
    const int lo = max(k_lo, s0), hi = min(k_hi, s1);
    if (lo >= hi) continue;
    const float* A = seg ? P.A2 : P.A;
    const float* B = seg ? P.B2 : P.B;
    const int lda = seg ? P.lda2 : P.lda, ldb = seg ? P.ldb2 : P.ldb;
    const bool ones = seg ? P.ones2 : P.ones1;
    // B column kind per lane: 0 read, 1 constant one, 2 zero
    const int kda = na >= P.N ? 2 : (anyones && na == P.N - 1) ? (ones ? 1 : 2) : 0;
    const int kdb = nb >= P.N ? 2 : (anyones && nb == P.N - 1) ? (ones ? 1 : 2) : 0;
    const int64_t* zi = P.onehot ? reinterpret_cast<const int64_t*>(A) : nullptr;  // (wave-uniform)
    const float* pa0 = zi ? nullptr : A + (va ? ma : 0);
    const float* pa1 = zi ? nullptr : A + (vb ? mb : 0);
    const float* pb0 = kda == 0 ? B + na : nullptr;
    const float* pb1 = kdb == 0 ? B + nb : nullptr;
    const float ca = kda == 1 ? 1.f : 0.f, cb = kdb == 1 ? 1.f : 0.f;
    for (int kb = lo; kb < hi; kb += 16 * TN_UB) {  // TN_UB 16-row blocks in flight
      float a[TN_UB][2][4], b[TN_UB][2][4];
#pragma unroll
      for (int u = 0; u < TN_UB; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = kb + 16 * u + 4 * lk + j;
          const bool kv = k < hi;
          const size_t ro = (size_t)(kv ? k - s0 : 0);
          if (zi) {
            const int64_t zk = kv ? zi[ro] : -1;
            a[u][0][j] = (va && zk == ma) ? 1.f : 0.f;
            a[u][1][j] = (vb && zk == mb) ? 1.f : 0.f;
          } else {
            a[u][0][j] = (kv && va) ? pa0[ro * lda] : 0.f;
            a[u][1][j] = (kv && vb) ? pa1[ro * lda] : 0.f;
          }
          b[u][0][j] = !kv ? 0.f : pb0 ? pb0[ro * ldb] : ca;
          b[u][1][j] = !kv ? 0.f : pb1 ? pb1[ro * ldb] : cb;
        }
#pragma unroll
      for (int u = 0; u < TN_UB; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0][j], b[u][0][j], acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0][j], b[u][1][j], acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1][j], b[u][0][j], acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1][j], b[u][1][j], acc[1][1], 0, 0, 0);
        }
    }
  }
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][bi * 16 + 4 * (lane >> 4) + i][bj * 16 + (lane & 15)] = acc[bi][bj][i];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += blockDim.x) {
    const int r = e >> 5, c = e & 31;
    const int gr = r0 + r, gc = c0 + c;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) v += part[i][r][c];
    if (G.S > 1) {  // partial tile; k_tn_reduce sums the S chunks in order (deterministic)
      G.part[((size_t)tg * G.S + sk) * 1024 + e] = v;
      continue;
    }
    if (gr >= P.M || gc >= P.N) continue;
    float* out = (P.Cb && gc == P.N - 1) ? P.Cb + gr : P.C + (size_t)gr * P.ldc + gc;
    if (P.beta) v += *out;
    *out = v;
  }
}

__global__ __launch_bounds__(256) void k_tn_reduce(GroupTN G, int tiles) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tiles * 1024) return;
  const int tg = i >> 10, e = i & 1023;
  int pi = 0;
  for (int j = 1; j < G.n; ++j)
    if (tg >= G.p[j].tile0) pi = j;
  const ProbTN& P = G.p[pi];
  const int t = tg - P.tile0;
  const int gr = (t / P.tiles_n) * 32 + (e >> 5), gc = (t % P.tiles_n) * 32 + (e & 31);
  if (gr >= P.M || gc >= P.N) return;
  const float* src = G.part + (size_t)tg * G.S * 1024 + e;
  float v = 0.f;
#pragma unroll 8
  for (int s = 0; s < G.S; ++s) v += src[(size_t)s * 1024];
  float* out = (P.Cb && gc == P.N - 1) ? P.Cb + gr : P.C + (size_t)gr * P.ldc + gc;
  if (P.beta) v += *out;
  *out = v;
}

// ---------------------------------------------------------------------------------------------------
// The same grouped TN GEMM with 64 x 64 tiles and 16-byte loads ("v" kernel; used when every operand
// row is 16-byte aligned).  The MFMA's output-row / output-column labels are a free permutation: lane
// (c, kq) of a 16x16x4 step feeds A[k0 + kq][m0 + 4c + mb] into block mb and B[k0 + kq][n0 + 4c + nb]
// into block nb, so ONE float4 load of A and one of B per 4 rows feed 16 MFMAs (the scalar kernel
// above: 4 loads per 4 MFMAs -- it is load-issue-bound on the node-weight shapes).  The ones column
// is not a GEMM column here: the bias is the row sum of A, accumulated from the same A registers by
// the first column tile.
constexpr int TV = 64;
constexpr int TV_PART = TV * TV + TV;  // partial tile + bias partials (split-K)

// Workgroup -> (problem, tile, row chunk) of the 64-tile kernels.  Each problem has its own split-K factor
// (every workgroup gets about the same number of rows: a 3N-row vec_proj problem is not split like an
// N-row one), and within a problem the chunk is the slow index, so the workgroups resident together read
// whole rows of A (every tile's column strip of the same row chunk) instead of long columns.
struct TNLoc {
  int pi, t, sk;
};
__device__ __forceinline__ TNLoc tn_locate(const GroupTN& G) {
  const int b = blockIdx.x;
  int pi = 0;
  for (int i = 1; i < G.n; ++i)
    if (b >= G.p[i].wg0) pi = i;
  const ProbTN& P = G.p[pi];
  const int l = b - P.wg0;
  return TNLoc{pi, l % P.ntiles, l / P.ntiles};
}
// this chunk's partial tile (S > 1), summed in chunk order by k_tn_reduce_v
__device__ __forceinline__ float* tn_part(const GroupTN& G, const ProbTN& P, int t, int sk) {
  return P.S > 1 ? G.part + ((size_t)P.part0 + (size_t)t * P.S + sk) * TV_PART : nullptr;
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_gemm_tn_v(GroupTN G) {
  __shared__ float red[NW][TV][TV + 1];
  __shared__ float redb[NW][TV];
  const TNLoc L = tn_locate(G);
  const ProbTN& P = G.p[L.pi];
  const int t = L.t, sk = L.sk;
  const int w = threadIdx.x / TMD_WAVE, lane = lane_id();
  const int c = lane & 15, kq = lane >> 4;
  const int m0 = (t / P.tiles_n) * TV, n0 = (t % P.tiles_n) * TV;
  const bool anyones = P.ones1 || P.ones2;
  const int Nr = anyones ? P.N - 1 : P.N;  // columns of B that are read (the ones column is the row sum)
  const bool do_bias = anyones && (t % P.tiles_n) == 0;
  // (a device row count shortens both segments: the chunks split the rows actually summed)
  const int cnt = P.rows ? max(0, *P.rows) : P.K + P.K2;
  const int K1 = min(P.K, cnt), KT = K1 + min(P.K2, cnt);
  const int nkt = (KT + 15) / 16, cper = (nkt + P.S - 1) / P.S;
  const int c_lo = min(KT, sk * cper * 16), c_hi = min(KT, (sk + 1) * cper * 16);
  const int nkb = (c_hi - c_lo + 15) / 16, per = (nkb + NW - 1) / NW;
  const int k_lo = min(c_hi, c_lo + w * per * 16), k_hi = min(c_hi, c_lo + (w + 1) * per * 16);
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  f4 rs = f4{0.f, 0.f, 0.f, 0.f};
  const int ma = m0 + 4 * c, na = n0 + 4 * c;
  const bool mfull = ma + 3 < P.M, nfull = na + 3 < Nr;
  const bool gemm = n0 < Nr;  // a bias-only tile (B = ones only) skips the MFMAs
  for (int seg = 0; seg < 2; ++seg) {
    const int s0 = seg ? K1 : 0, s1 = seg ? KT : K1;
    const int lo = max(k_lo, s0), hi = min(k_hi, s1);
    if (lo >= hi) continue;
    const float* A = seg ? P.A2 : P.A;
    const float* B = seg ? P.B2 : P.B;
    const int lda = seg ? P.lda2 : P.lda, ldb = seg ? P.ldb2 : P.ldb;
    const bool bias_seg = do_bias && (seg ? P.ones2 : P.ones1);
    const int64_t* zi = P.onehot ? reinterpret_cast<const int64_t*>(A) : nullptr;
    for (int kb = lo; kb < hi; kb += 16) {  // four 4-row MFMA steps, all loads first
      f4 a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + 4 * u + kq;
        const bool kv = k < hi;
        const size_t ro = (size_t)(kv ? k - s0 : 0);
        if (zi) {
          const int64_t zk = kv ? zi[ro] : -1;
#pragma unroll
          for (int i = 0; i < 4; ++i) a[u][i] = (zk == ma + i && ma + i < P.M) ? 1.f : 0.f;
        } else if (kv && mfull) {
          a[u] = *reinterpret_cast<const f4*>(A + ro * lda + ma);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[u][i] = (kv && ma + i < P.M) ? A[ro * lda + ma + i] : 0.f;
        }
        if (!gemm || !B) {
          b[u] = f4{0.f, 0.f, 0.f, 0.f};
        } else if (kv && nfull) {
          b[u] = *reinterpret_cast<const f4*>(B + ro * ldb + na);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) b[u][i] = (kv && na + i < Nr) ? B[ro * ldb + na + i] : 0.f;
        }
      }
      if (bias_seg) {
#pragma unroll
        for (int u = 0; u < 4; ++u) rs += a[u];
      }
      if (gemm) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][mb], b[u][nb], acc[mb][nb], 0, 0, 0);
      }
    }
  }
  // C layout of a 16x16 block: lane holds rows 4 (lane >> 4) + i, column lane & 15 (MFMA labels)
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][4 * (4 * kq + i) + mb][4 * c + nb] = acc[mb][nb][i];
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      rs[i] = v;
    }
    if (kq == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) redb[w][4 * c + i] = rs[i];
    }
  }
  __syncthreads();
  float* part = tn_part(G, P, t, sk);
  for (int e = threadIdx.x; e < TV * TV; e += blockDim.x) {
    const int r = e >> 6, cc = e & 63;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) v += red[i][r][cc];
    if (part) {
      part[e] = v;
      continue;
    }
    const int m = m0 + r, n = n0 + cc;
    if (m >= P.M || n >= Nr) continue;
    float* out = P.C + (size_t)m * P.ldc + n;
    if (P.beta) v += *out;
    *out = v;
  }
  if (do_bias) {
    for (int r = threadIdx.x; r < TV; r += blockDim.x) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) v += redb[i][r];
      if (part) {
        part[TV * TV + r] = v;
        continue;
      }
      const int m = m0 + r;
      if (m >= P.M) continue;
      float* out = P.Cb ? P.Cb + m : P.C + (size_t)m * P.ldc + (P.N - 1);
      if (P.beta) v += *out;
      *out = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_tn_reduce_v(GroupTN G, int tiles) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tiles * TV_PART) return;
  const int tg = i / TV_PART, e = i - tg * TV_PART;
  int pi = 0;
  for (int j = 1; j < G.n; ++j)
    if (tg >= G.p[j].tile0) pi = j;
  const ProbTN& P = G.p[pi];
  if (P.S <= 1) return;  // written by the GEMM kernel itself
  const int t = tg - P.tile0;
  const int m0 = (t / P.tiles_n) * TV, n0 = (t % P.tiles_n) * TV;
  const bool anyones = P.ones1 || P.ones2;
  const int Nr = anyones ? P.N - 1 : P.N;
  float* out;
  if (e < TV * TV) {
    const int m = m0 + (e >> 6), n = n0 + (e & 63);
    if (m >= P.M || n >= Nr) return;
    out = P.C + (size_t)m * P.ldc + n;
  } else {
    const int m = m0 + (e - TV * TV);
    if (!anyones || (t % P.tiles_n) != 0 || m >= P.M) return;
    out = P.Cb ? P.Cb + m : P.C + (size_t)m * P.ldc + (P.N - 1);
  }
  const float* src = G.part + ((size_t)P.part0 + (size_t)t * P.S) * TV_PART + e;
  float v = 0.f;
#pragma unroll 8
  for (int s = 0; s < P.S; ++s) v += src[(size_t)s * TV_PART];
  if (P.beta) v += *out;
  *out = v;
}

// The "v" kernel with the row loop software-pipelined and a small reduction buffer (A/B switch
// TMDNET_TN_V=1 keeps k_gemm_tn_v).  k_gemm_tn_v issues a 16-row block's loads and then its MFMAs, so every
// block waits out a full memory latency, and its per-wave reduction tiles (NW x 64 x 65 floats, 66 KB)
// hold a CU to two workgroups.  Here the next block's A / B rows are in flight while the MFMAs consume the
// current ones (two register sets, the loop unrolled by two), and the waves fold their tiles into ONE
// 64 x (16 NB + 1) buffer in wave order (deterministic: the same order every run).  NB = 16-column blocks
// per tile: 2 when every problem reads <= 32 columns of B (the dk/dv weight gradient: 4096 x 32 over the
// edge pairs), so no MFMA runs on the zero half of a 64-wide tile.  The tile numbering and the partial
// layout are k_gemm_tn_v's (64 x 64 + 64; with NB = 2 the one column tile is n0 = 0 and the reduction
// never reads columns >= Nr), so k_tn_reduce_v and the workspace size serve both.
template <int NW, int NB, bool PIPE>
__global__ __launch_bounds__(NW * 64) void k_gemm_tn_v2(GroupTN G) {
  constexpr int TN = 16 * NB;
  __shared__ float red[TV][TN + 1];
  __shared__ float redb[TV];
  const TNLoc L = tn_locate(G);
  const ProbTN& P = G.p[L.pi];
  const int t = L.t, sk = L.sk;
  const int w = threadIdx.x / TMD_WAVE, lane = lane_id();
  const int c = lane & 15, kq = lane >> 4;
  const int m0 = (t / P.tiles_n) * TV, n0 = (t % P.tiles_n) * TV;
  const bool anyones = P.ones1 || P.ones2;
  const int Nr = anyones ? P.N - 1 : P.N;
  const bool do_bias = anyones && (t % P.tiles_n) == 0;
  // (a device row count shortens both segments: the chunks split the rows actually summed)
  const int cnt = P.rows ? max(0, *P.rows) : P.K + P.K2;
  const int K1 = min(P.K, cnt), KT = K1 + min(P.K2, cnt);
  const int nkt = (KT + 15) / 16, cper = (nkt + P.S - 1) / P.S;
  const int c_lo = min(KT, sk * cper * 16), c_hi = min(KT, (sk + 1) * cper * 16);
  const int nkb = (c_hi - c_lo + 15) / 16, per = (nkb + NW - 1) / NW;
  const int k_lo = min(c_hi, c_lo + w * per * 16), k_hi = min(c_hi, c_lo + (w + 1) * per * 16);
  f4 acc[4][NB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  f4 rs = f4{0.f, 0.f, 0.f, 0.f};
  // MFMA labels: lane c feeds A row m0 + 4c + mb into block mb and B column n0 + NB c + nb into block nb
  const int ma = m0 + 4 * c, na = n0 + NB * c;
  const bool mfull = ma + 3 < P.M, nfull = na + NB - 1 < Nr;
  const bool gemm = n0 < Nr;
  for (int seg = 0; seg < 2; ++seg) {
    const int s0 = seg ? K1 : 0, s1 = seg ? KT : K1;
    const int lo = max(k_lo, s0), hi = min(k_hi, s1);
    if (lo >= hi) continue;
    const float* A = seg ? P.A2 : P.A;
    const float* B = seg ? P.B2 : P.B;
    const int lda = seg ? P.lda2 : P.lda, ldb = seg ? P.ldb2 : P.ldb;
    const bool bias_seg = do_bias && (seg ? P.ones2 : P.ones1);
    const int64_t* zi = P.onehot ? reinterpret_cast<const int64_t*>(A) : nullptr;
    auto load = [&](int kb, f4 (&a)[4], f4 (&b)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + 4 * u + kq;
        const bool kv = k < hi;
        const size_t ro = (size_t)(kv ? k - s0 : 0);
        if (zi) {
          const int64_t zk = kv ? zi[ro] : -1;
#pragma unroll
          for (int i = 0; i < 4; ++i) a[u][i] = (zk == ma + i && ma + i < P.M) ? 1.f : 0.f;
        } else if (kv && mfull) {
          a[u] = *reinterpret_cast<const f4*>(A + ro * lda + ma);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[u][i] = (kv && ma + i < P.M) ? A[ro * lda + ma + i] : 0.f;
        }
        b[u] = f4{0.f, 0.f, 0.f, 0.f};
        if (!gemm || !B) {
        } else if (kv && nfull) {
          if constexpr (NB == 4) {
            b[u] = *reinterpret_cast<const f4*>(B + ro * ldb + na);
          } else {
            const float2 v = *reinterpret_cast<const float2*>(B + ro * ldb + na);
            b[u][0] = v.x;
            b[u][1] = v.y;
          }
        } else {
#pragma unroll
          for (int i = 0; i < NB; ++i) b[u][i] = (kv && na + i < Nr) ? B[ro * ldb + na + i] : 0.f;
        }
      }
    };
    auto mma = [&](const f4 (&a)[4], const f4 (&b)[4]) {
      if (bias_seg) {
#pragma unroll
        for (int u = 0; u < 4; ++u) rs += a[u];
      }
      if (gemm) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][mb], b[u][nb], acc[mb][nb], 0, 0, 0);
      }
    };
    f4 a0[4], b0[4], a1[4], b1[4];
    if constexpr (!PIPE) {
      for (int kb = lo; kb < hi; kb += 16) {
        load(kb, a0, b0);
        mma(a0, b0);
      }
      continue;
    }
    load(lo, a0, b0);
    for (int kb = lo; kb < hi; kb += 32) {
      const bool more = kb + 16 < hi;
      if (more) load(kb + 16, a1, b1);
      mma(a0, b0);
      if (!more) break;
      if (kb + 32 < hi) load(kb + 32, a0, b0);
      mma(a1, b1);
    }
  }
  // fold the waves' tiles in wave order (C layout of a 16x16 block: lane holds rows 4 (lane >> 4) + i,
  // column lane & 15 in the MFMA labels)
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      rs[i] = v;
    }
  }
  for (int i = 0; i < NW; ++i) {
    if (w == i) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float& r = red[4 * (4 * kq + j) + mb][NB * c + nb];
            r = i ? r + acc[mb][nb][j] : acc[mb][nb][j];
          }
      if (do_bias && kq == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) redb[4 * c + j] = i ? redb[4 * c + j] + rs[j] : rs[j];
      }
    }
    __syncthreads();
  }
  float* part = tn_part(G, P, t, sk);
  for (int e = threadIdx.x; e < TV * TN; e += blockDim.x) {
    const int r = e / TN, cc = e - r * TN;
    const float v = red[r][cc];
    if (part) {
      part[r * TV + cc] = v;
      continue;
    }
    const int m = m0 + r, n = n0 + cc;
    if (m >= P.M || n >= Nr) continue;
    float* out = P.C + (size_t)m * P.ldc + n;
    *out = P.beta ? *out + v : v;
  }
  if (do_bias) {
    for (int r = threadIdx.x; r < TV; r += blockDim.x) {
      const float v = redb[r];
      if (part) {
        part[TV * TV + r] = v;
        continue;
      }
      const int m = m0 + r;
      if (m >= P.M) continue;
      float* out = P.Cb ? P.Cb + m : P.C + (size_t)m * P.ldc + (P.N - 1);
      *out = P.beta ? *out + v : v;
    }
  }
}

}  // namespace gemm

// ---------------------------------------------------------------------------------------------------
// The ET dk/dv projection  C [M][N] = A [M][K] W[N][K]^T (+ bias)  with K = num_rbf = 32 or 64 (the
// pair rows' RBF times every layer's stacked dk/dv weight, reference torchmd_et.py:282-291; also its
// r-derivative and, in the force-loss second order, the adjoint gb_f W^T).  The f32-input MFMA
// (v_mfma_f32_16x16x4_f32) delivers 1/16 of the bf16 rate, so this runs on the bf16 MFMA with fp32
// accuracy: every operand is split EXACTLY into three bf16 pieces x = x0 + x1 + x2 (truncation: each
// piece takes the next 8 significant bits, x - x0 and x - x0 - x1 are exact in fp32), and the six
// products x_i y_j with i + j <= 2 -- each exact in the fp32 accumulator -- are summed, small terms
// first.  The dropped x1 y2 + x2 y1 + x2 y2 are below 2^-23 |x||y|: the result carries fp32 GEMM
// error (tests/test_gpu_second_order.py: error vs fp64 against the library fp32 GEMM's).
// 6 MFMAs of 16 x 16 x 32 per 16 x 16 x 32 block of the product = 2.5 PF / 6 ~ 400 TF of fp32 work;
// at K = 64 that is above the rate at which the output (4 bytes per 128 FLOP) can be written, so the
// kernel is bound by the C stream.
// Roles: the MFMA's A operand is the W tile (rows n), its B operand is A^T (columns m), so a lane's
// four accumulator rows are four consecutive n of one output row m -> one 16-byte store.
namespace proj {

using u4 = unsigned __attribute__((ext_vector_type(4)));
using bf8 = __bf16 __attribute__((ext_vector_type(8)));
using f4 = float __attribute__((ext_vector_type(4)));

struct Args {
  int M, N, lda, ldc;
  long long pstride;       // elements between the three pieces of Wp
  const float* A;
  const unsigned short* Wp;
  const float* bias;
  float* C;
};

// the three truncated bf16 pieces of x, as fp32 bit patterns with the low half zero
__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
  h = __float_as_uint(x) & 0xffff0000u;
  const float r1 = x - __uint_as_float(h);
  m = __float_as_uint(r1) & 0xffff0000u;
  l = __float_as_uint(r1 - __uint_as_float(m)) & 0xffff0000u;
}

// 8 consecutive fp32 (two 16-byte loads) -> the three bf16 fragments of one MFMA operand
__device__ __forceinline__ void split8(const float4& a, const float4& b, bf8 (&f)[3]) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  unsigned h[8], m[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) split3(x[j], h[j], m[j], l[j]);
  u4 H, M, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // element 2p in the low half of register p
    H[p] = (h[2 * p] >> 16) | h[2 * p + 1];
    M[p] = (m[2 * p] >> 16) | m[2 * p + 1];
    L[p] = (l[2 * p] >> 16) | l[2 * p + 1];
  }
  f[0] = __builtin_bit_cast(bf8, H);
  f[1] = __builtin_bit_cast(bf8, M);
  f[2] = __builtin_bit_cast(bf8, L);
}

// W [N][K] fp32 -> its three exact bf16 pieces Wp [3][N][K] (once per weight, shared by every GEMM
// that multiplies by it: the projection, its r-derivative and the second-order adjoint)
__global__ __launch_bounds__(256) void k_proj_split(int N, int K, const float* W, int ldw, unsigned short* Wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // one float4 of W
  if (i >= N * K / 4) return;
  const int n = i / (K / 4), k = (i % (K / 4)) * 4;
  const float4 v = *reinterpret_cast<const float4*>(W + (size_t)n * ldw + k);
  const float x[4] = {v.x, v.y, v.z, v.w};
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split3(x[j], h[j], m[j], l[j]);
  const size_t o = (size_t)n * K + k, ps = (size_t)N * K;
  *reinterpret_cast<uint2*>(Wp + o) = make_uint2((h[0] >> 16) | h[1], (h[2] >> 16) | h[3]);
  *reinterpret_cast<uint2*>(Wp + ps + o) = make_uint2((m[0] >> 16) | m[1], (m[2] >> 16) | m[3]);
  *reinterpret_cast<uint2*>(Wp + 2 * ps + o) = make_uint2((l[0] >> 16) | l[1], (l[2] >> 16) | l[3]);
}

// KS = K / 32 MFMA k-steps.  A workgroup (4 waves) owns BN columns -- their W pieces (from the
// pre-split Wp) and bias staged in LDS -- and 64 MB rows, a wave MB 16-row blocks of A split into
// registers.  After the one barrier the waves read W fragments from LDS only: a global load inside
// the column loop would wait behind the wave's own output stores (loads and stores share vmcnt).
// Grid: x = column tiles (fast: the tiles of one row block run together and re-read its A rows from
// L2), y = row tiles.
// (Output stores staged per wave through LDS as whole 128-byte lines were measured and dropped: the
// L2 already merges the half-line pieces of adjacent column blocks; nontemporal stores too:
// C2 step 0.885 -> 0.913 ms.)
template <int KS, int MB, int BN>
__global__ __launch_bounds__(256) void k_proj_x3(Args P) {
  constexpr int K = 32 * KS, LD = K + 8;  // LDS row pitch in bf16 (16-byte pad: rows shift banks)
  __shared__ __attribute__((aligned(16))) unsigned short w[3][BN][LD];
  __shared__ __attribute__((aligned(16))) float sb[BN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * BN;
  const int m0 = (blockIdx.y * 4 + wave) * (16 * MB);
  const int nr = min(BN, P.N - n0);
  const int kq = 8 * (lane >> 4);
  // A rows first (their latency overlaps the W tile copy): lane holds row m0 + 16 mb + (lane & 15),
  // k = 32 ks + kq + 0..7
  float4 ar[MB][KS][2];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const float* r = P.A + (size_t)min(m0 + 16 * mb + (lane & 15), P.M - 1) * P.lda + kq;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      ar[mb][ks][0] = *reinterpret_cast<const float4*>(r + 32 * ks);
      ar[mb][ks][1] = *reinterpret_cast<const float4*>(r + 32 * ks + 4);
    }
  }
  // W tile (3 pieces x BN rows x K bf16, 16-byte chunks; rows past N clamp) and bias -> LDS: all of the
  // thread's loads first, then the stores (one memory round trip, not one per chunk)
  constexpr int CH = K / 8;  // 16-byte chunks per row
  constexpr int NL = (3 * BN * CH + 255) / 256;
  u4 stg[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int p = c / (BN * CH), rc = c % (BN * CH), n = rc / CH, k = (rc % CH) * 8;
    if (c < 3 * BN * CH)
      stg[i] = *reinterpret_cast<const u4*>(P.Wp + p * P.pstride + (size_t)min(n0 + n, P.N - 1) * K + k);
  }
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int p = c / (BN * CH), rc = c % (BN * CH), n = rc / CH, k = (rc % CH) * 8;
    if (c < 3 * BN * CH) *reinterpret_cast<u4*>(&w[p][n][k]) = stg[i];
  }
  if (threadIdx.x < BN) sb[threadIdx.x] = P.bias ? P.bias[min(n0 + (int)threadIdx.x, P.N - 1)] : 0.f;
  bf8 a[MB][KS][3];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) split8(ar[mb][ks][0], ar[mb][ks][1], a[mb][ks]);
  __syncthreads();
  if (m0 >= P.M) return;  // (after the barrier: every wave took part in the tile copy)
  for (int nb = 0; nb < nr; nb += 16) {
    bf8 b[KS][3];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        b[ks][p] = *reinterpret_cast<const bf8*>(&w[p][nb + (lane & 15)][32 * ks + kq]);
    f4 acc[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb] = f4{0.f, 0.f, 0.f, 0.f};
    // small terms first: (W piece, A piece) = (2,0) (1,1) (0,2) (1,0) (0,1) (0,0)
    constexpr int TW[6] = {2, 1, 0, 1, 0, 0}, TA[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][TW[t]], a[mb][ks][TA[t]], acc[mb], 0, 0, 0);
    const int nl = nb + 4 * (lane >> 4);
    const f4 bv = *reinterpret_cast<const f4*>(&sb[nl]);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = m0 + 16 * mb + (lane & 15);
      if (m < P.M) *reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n0 + nl) = acc[mb] + bv;
    }
  }
}

// B [K][N] (row-major, ldb) -> the three exact bf16 pieces of B^T, Bp [3][N][K]: the split of a weight that
// multiplies from the right untransposed (an input gradient g_y W of a Linear y = x W^T), so that
// k_gemm_x3 reads it as the k-contiguous [N][K] operand.  One thread per 4 consecutive k of one n.
__global__ __launch_bounds__(256) void k_split_t(int N, int K, const float* B, int ldb, unsigned short* Bp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * (K / 4)) return;
  const int k = (i / N) * 4, n = i % N;  // consecutive threads: consecutive n (coalesced reads of B rows)
  const float x[4] = {B[(size_t)k * ldb + n], B[(size_t)(k + 1) * ldb + n], B[(size_t)(k + 2) * ldb + n],
                      B[(size_t)(k + 3) * ldb + n]};
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split3(x[j], h[j], m[j], l[j]);
  const size_t o = (size_t)n * K + k, ps = (size_t)N * K;
  *reinterpret_cast<uint2*>(Bp + o) = make_uint2((h[0] >> 16) | h[1], (h[2] >> 16) | h[3]);
  *reinterpret_cast<uint2*>(Bp + ps + o) = make_uint2((m[0] >> 16) | m[1], (m[2] >> 16) | m[3]);
  *reinterpret_cast<uint2*>(Bp + 2 * ps + o) = make_uint2((l[0] >> 16) | l[1], (l[2] >> 16) | l[3]);
}

// Large-M fp32 GEMM on the bf16 MFMA at fp32 accuracy (the node feature mixes of C5-size systems, where
// the grouped split-K k_gemm runs out of its envelope): C [M][N] = beta C + A [M][K] Bp^T + bias, Bp the
// pre-split [3][N][K] pieces (k_proj_split of a Linear weight, or k_split_t of an untransposed right
// operand).  k_proj_x3's scheme -- A split into three bf16 pieces in registers, the six products with
// i + j <= 2 summed small first, W as the MFMA's A operand so a lane's four accumulator rows are four
// consecutive output columns (one 16-byte store) -- with K walked in 128- (or 64-) wide chunks (any K % 32 == 0:
// the input gradients have K = 3H / 5H): per chunk the workgroup stages its BN columns' pieces of the
// chunk in LDS (two barriers) and each wave splits its MB 16-row blocks of the chunk; the accumulators of
// all BN columns stay in registers across chunks.
struct XArgs {
  int M, N, K, lda, ldc, beta;
  int nx, ny, remap;  // column / row tiles; remap: 1-D grid dealt XCD-major (see k_gemm_x3)
  const float* A;
  const unsigned short* Bp;
  const float* bias;
  float* C;
  // epilogue extensions (tmdnet_gemm_x3_ex_f32, k_gemm's tmdnet_gemm_ex_f32 semantics): v = acc + bias (+ C)
  // -> pre[r][c] = v -> v = silu(v) (act) -> v *= rscale[r] -> v *= silu'(dpre[r][c]) -> C
  int act, ldx;
  float* pre;
  const float* rscale;
  const float* dpre;
  // WS != 0: the right operand as fp32, split into its three pieces while it is staged in LDS (no separate
  // split launch, nothing cached that an in-place weight update could leave stale): WS = 1 a [N][K] Linear
  // weight (C = A W^T), WS = 2 a [K][N] right operand (C = A W); row stride ldw
  const float* W;
  int ldw;
};
template <int MB, int BN, int PD, int WS = 0>
__global__ __launch_bounds__(256) void k_gemm_x3(XArgs P) {
  // K chunk staged per barrier pair: 128 (64 at BN = 128) -> ~52 KB of LDS, 3 workgroups per CU
  constexpr int KC = BN >= 128 ? 64 : 128, LD = KC + 8, NB = BN / 16, SPC = KC / 32;
  // A prefetch depth in k-steps: the loads of step s + PD are issued when step s is split, so ~PD steps of
  // MFMA work (PD x 6 x NB x MB MFMAs) cover the HBM latency of a row block.  Measured (tools/x3_time.py,
  // C5 shapes): the narrow input-gradient form (BN = 128, K = 3H / 5H) gains from PD = 4 (vec_bwd 132 ->
  // 114 us), the wide forward form (BN = 64, K = H) loses (the ring's registers cost it a wave per SIMD:
  // 75 -> 100 us), so it keeps PD = 1
  __shared__ __attribute__((aligned(16))) unsigned short w[3][BN][LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int bx = blockIdx.x, by = blockIdx.y;
  if (P.remap) {
    // The hardware deals consecutive workgroups round-robin to the 8 XCDs, so the nx column tiles of one
    // row block -- which all read the same A rows -- would land on nx different XCDs (nx fetches of A from
    // HBM / MALL, one per XCD L2).  Dealt XCD-major instead: XCD x (= b % 8) walks the contiguous tile range
    // [start(x), start(x) + count(x)) in order, so a row block's column tiles run on one XCD, together.
    const int T = P.nx * P.ny, b = blockIdx.x, x = b & 7, q = T >> 3, r = T & 7;
    const int t = x * q + min(x, r) + (b >> 3);
    bx = t % P.nx;
    by = t / P.nx;
  }
  const int n0 = bx * BN;
  const int m0 = (by * 4 + wave) * (16 * MB);
  const int kq = 8 * (lane >> 4);
  const size_t ps = (size_t)P.N * P.K;
  f4 acc[NB][MB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f4{0.f, 0.f, 0.f, 0.f};
  // A rows of this wave: row m0 + 16 mb + (lane & 15), k = 32 s + kq .. + 7 (two 16-byte loads per k-step
  // and row block), in a ring of PD k-steps
  const float* arow[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) arow[mb] = P.A + (size_t)min(m0 + 16 * mb + (lane & 15), P.M - 1) * P.lda + kq;
  const int nks_all = P.K / 32;
  float4 an[PD][MB][2];
#pragma unroll
  for (int d = 0; d < PD; ++d)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int ko = 32 * min(d, nks_all - 1);
      an[d][mb][0] = *reinterpret_cast<const float4*>(arow[mb] + ko);
      an[d][mb][1] = *reinterpret_cast<const float4*>(arow[mb] + ko + 4);
    }
  constexpr int TW[6] = {2, 1, 0, 1, 0, 0}, TA[6] = {0, 1, 2, 0, 1, 0};
  for (int s0 = 0; s0 < nks_all; s0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int st_ = s0 + d;
      if (st_ < nks_all) {
        if (st_ % SPC == 0) {
          // the chunk's pieces: every 16-byte load of the thread issued before the first LDS store (one
          // memory round trip per chunk; a load -> store loop serialises ~12 of them)
          const int kc = 32 * st_;
          const int nks = min(KC, P.K - kc) / 32;
          constexpr int CH = KC / 8, NL = 3 * BN * CH / 256;
          const int ch = nks * 4;  // 16-byte chunks per row of this K chunk
          if constexpr (WS == 0) {
            u4 stg[NL];
#pragma unroll
            for (int i = 0; i < NL; ++i) {
              const int c = threadIdx.x + 256 * i;
              const int p = c / (BN * CH), rc = c % (BN * CH), n = rc / CH, k = (rc % CH) * 8;
              stg[i] = k < 8 * ch
                           ? *reinterpret_cast<const u4*>(P.Bp + p * ps + (size_t)min(n0 + n, P.N - 1) * P.K + kc + k)
                           : u4{0u, 0u, 0u, 0u};
            }
            __syncthreads();  // the previous chunk's LDS reads are done
#pragma unroll
            for (int i = 0; i < NL; ++i) {
              const int c = threadIdx.x + 256 * i;
              const int p = c / (BN * CH), rc = c % (BN * CH), n = rc / CH, k = (rc % CH) * 8;
              *reinterpret_cast<u4*>(&w[p][n][k]) = stg[i];
            }
          } else if constexpr (WS == 1) {
            // 8 consecutive k of one weight row per chunk: two 16-byte loads, split8 -> three 16-byte LDS stores
            constexpr int NC = BN * CH / 256;
            float4 lo[NC], hi[NC];
#pragma unroll
            for (int i = 0; i < NC; ++i) {
              const int c = threadIdx.x + 256 * i;
              const int n = c / CH, k = (c % CH) * 8;
              if (k < 8 * ch) {
                const float* r = P.W + (size_t)min(n0 + n, P.N - 1) * P.ldw + kc + k;
                lo[i] = *reinterpret_cast<const float4*>(r);
                hi[i] = *reinterpret_cast<const float4*>(r + 4);
              } else {
                lo[i] = hi[i] = make_float4(0.f, 0.f, 0.f, 0.f);
              }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NC; ++i) {
              const int c = threadIdx.x + 256 * i;
              const int n = c / CH, k = (c % CH) * 8;
              bf8 f[3];
              split8(lo[i], hi[i], f);
#pragma unroll
              for (int p = 0; p < 3; ++p) *reinterpret_cast<bf8*>(&w[p][n][k]) = f[p];
            }
          } else {
            // W [K][N]: 4 consecutive n of one k row per 16-byte load, written transposed (2-byte LDS stores)
            constexpr int NC = KC * BN / 4 / 256, QN = BN / 4;
            float4 v[NC];
#pragma unroll
            for (int i = 0; i < NC; ++i) {
              const int c = threadIdx.x + 256 * i;
              const int k = c / QN, n4 = (c % QN) * 4;
              v[i] = (k < 32 * nks && n0 + n4 < P.N)
                         ? *reinterpret_cast<const float4*>(P.W + (size_t)(kc + k) * P.ldw + n0 + n4)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NC; ++i) {
              const int c = threadIdx.x + 256 * i;
              const int k = c / QN, n4 = (c % QN) * 4;
              const float x[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                unsigned h, m, l;
                split3(x[j], h, m, l);
                w[0][n4 + j][k] = (unsigned short)(h >> 16);
                w[1][n4 + j][k] = (unsigned short)(m >> 16);
                w[2][n4 + j][k] = (unsigned short)(l >> 16);
              }
            }
          }
          __syncthreads();
        }
        bf8 a[MB][3];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) split8(an[d][mb][0], an[d][mb][1], a[mb]);
        const int ko = 32 * min(st_ + PD, nks_all - 1);  // (clamped: the tail reloads the last step)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          an[d][mb][0] = *reinterpret_cast<const float4*>(arow[mb] + ko);
          an[d][mb][1] = *reinterpret_cast<const float4*>(arow[mb] + ko + 4);
        }
        const int kl = 32 * (st_ % SPC);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          bf8 b[3];
#pragma unroll
          for (int q = 0; q < 3; ++q) b[q] = *reinterpret_cast<const bf8*>(&w[q][16 * nb + (lane & 15)][kl + kq]);
#pragma unroll
          for (int t = 0; t < 6; ++t)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[TW[t]], a[mb][TA[t]], acc[nb][mb], 0, 0, 0);
        }
      }
    }
  }
  if (m0 >= P.M) return;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = n0 + 16 * nb + 4 * (lane >> 4);
    if (n >= P.N) continue;
    const f4 bv = P.bias ? *reinterpret_cast<const f4*>(P.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = m0 + 16 * mb + (lane & 15);
      if (m >= P.M) continue;
      f4* out = reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n);
      f4 v = acc[nb][mb] + bv;
      if (P.beta) v += *out;
      if (P.pre) *reinterpret_cast<f4*>(P.pre + (size_t)m * P.ldx + n) = v;
      if (P.act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = Silu<float>(v[j]).s;
      }
      if (P.rscale) v *= P.rscale[m];
      if (P.dpre) {
        const f4 x = *reinterpret_cast<const f4*>(P.dpre + (size_t)m * P.ldx + n);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= Silu<float>(x[j]).d(x[j]);
      }
      *out = v;
    }
  }
}

}  // namespace proj

// ---------------------------------------------------------------------------------------------------
// The grouped TN GEMM (C (+)= A^T B [+ A2^T B2], bias = column sums of A) on the bf16 MFMA at fp32
// accuracy (A/B switch TMDNET_TN_V=4): every operand value is split EXACTLY into three bf16 pieces
// (proj::split3) and the six products with i + j <= 2 are accumulated in fp32, as tmdnet_proj_f32 does
// -- 6 bf16 MFMAs per 16 x 16 x 32 block = 2.7x the fp32 MFMA's rate.  Both operands arrive k-major
// (row k holds every m / n) while an MFMA fragment is 8 consecutive k of one m / n, so each 32-row step
// goes through LDS: coalesced float4 loads, split in registers, written transposed into three bf16
// planes per operand; the four waves (2 x 2 over the 64 x 64 tile) read 16-byte fragments.  The next
// step's rows are loaded before the current step's MFMAs.  Tile numbering, split-K partial layout and
// epilogue are k_gemm_tn_v's (k_tn_reduce_v sums the partials).  Not for one-hot A (the v kernel).
// Measured (tools/tn_time.py, C2 training shapes): SLOWER than the fp32-MFMA k_gemm_tn_v -- dk/dv 4096 x 64
// over 6.6k + 13.2k rows 264 vs 142 us, node weights 259 vs 147 us: the transposed 2-byte LDS stores, the
// in-register splits and two barriers per 32-row step cost more than the MFMA time they save at these
// 64-wide outputs.  Kept as the A/B form; the default stays k_gemm_tn_v.
namespace tnx3 {

using gemm::GroupTN;
using gemm::ProbTN;
using gemm::TV;
using gemm::TV_PART;
using gemm::TNLoc;
using gemm::tn_locate;
using gemm::tn_part;
using bf8 = __bf16 __attribute__((ext_vector_type(8)));
using f4 = float __attribute__((ext_vector_type(4)));
constexpr int KB = 32, LDK = KB + 8;  // rows per step; LDS pitch (bf16) of a transposed row

__global__ __launch_bounds__(256) void k_gemm_tn_x3(GroupTN G) {
  __shared__ __attribute__((aligned(16))) unsigned short la[3][TV][LDK];
  __shared__ __attribute__((aligned(16))) unsigned short lb[3][TV][LDK];
  __shared__ float rsum[16][TV];
  const TNLoc L = tn_locate(G);
  const ProbTN& P = G.p[L.pi];
  const int t = L.t, sk = L.sk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = (t / P.tiles_n) * TV, n0 = (t % P.tiles_n) * TV;
  const bool anyones = P.ones1 || P.ones2;
  const int Nr = anyones ? P.N - 1 : P.N;
  const bool do_bias = anyones && (t % P.tiles_n) == 0;
  const bool gemm = n0 < Nr;
  // (a device row count shortens both segments: the chunks split the rows actually summed)
  const int cnt = P.rows ? max(0, *P.rows) : P.K + P.K2;
  const int K1 = min(P.K, cnt), KT = K1 + min(P.K2, cnt);
  const int nks = (KT + KB - 1) / KB, cper = (nks + P.S - 1) / P.S;
  const int c_lo = min(KT, sk * cper * KB), c_hi = min(KT, (sk + 1) * cper * KB);
  // this thread's two float4 of each 32 x 64 operand tile: row kr[j], columns q4 .. q4 + 3
  const int q4 = (tid & 15) * 4, kr0 = tid >> 4;  // rows kr0 and kr0 + 16
  const int ma = m0 + q4, na = n0 + q4;
  const bool mfull = ma + 3 < P.M, nfull = na + 3 < Nr;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  f4 rs = f4{0.f, 0.f, 0.f, 0.f};
  for (int seg = 0; seg < 2; ++seg) {
    const int s0 = seg ? K1 : 0, s1 = seg ? KT : K1;
    const int lo = max(c_lo, s0), hi = min(c_hi, s1);
    if (lo >= hi) continue;
    const float* A = seg ? P.A2 : P.A;
    const float* B = seg ? P.B2 : P.B;
    const int lda = seg ? P.lda2 : P.lda, ldb = seg ? P.ldb2 : P.ldb;
    const bool bias_seg = do_bias && (seg ? P.ones2 : P.ones1);
    auto load = [&](int kb, f4 (&a)[2], f4 (&b)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = kb + kr0 + 16 * j;
        const bool kv = k < hi;
        const size_t ro = (size_t)(kv ? k - s0 : 0);
        if (kv && mfull) {
          a[j] = *reinterpret_cast<const f4*>(A + ro * lda + ma);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[j][i] = (kv && ma + i < P.M) ? A[ro * lda + ma + i] : 0.f;
        }
        if (!gemm || !B) {
          b[j] = f4{0.f, 0.f, 0.f, 0.f};
        } else if (kv && nfull) {
          b[j] = *reinterpret_cast<const f4*>(B + ro * ldb + na);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) b[j][i] = (kv && na + i < Nr) ? B[ro * ldb + na + i] : 0.f;
        }
      }
    };
    // split into the three pieces and store transposed: plane[p][column][row]
    auto stage = [&](const f4 (&a)[2], const f4 (&b)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int kr = kr0 + 16 * j;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          unsigned h, m, l;
          proj::split3(a[j][i], h, m, l);
          la[0][q4 + i][kr] = (unsigned short)(h >> 16);
          la[1][q4 + i][kr] = (unsigned short)(m >> 16);
          la[2][q4 + i][kr] = (unsigned short)(l >> 16);
          proj::split3(b[j][i], h, m, l);
          lb[0][q4 + i][kr] = (unsigned short)(h >> 16);
          lb[1][q4 + i][kr] = (unsigned short)(m >> 16);
          lb[2][q4 + i][kr] = (unsigned short)(l >> 16);
        }
      }
    };
    f4 a[2], b[2];
    load(lo, a, b);
    for (int kb = lo; kb < hi; kb += KB) {
      if (bias_seg) rs += a[0] + a[1];
      __syncthreads();  // the previous step's fragments are read
      stage(a, b);
      __syncthreads();
      if (kb + KB < hi) load(kb + KB, a, b);  // next rows in flight during the MFMAs
      if (gemm) {
        bf8 fa[2][3], fb[2][3];
        const int ko = 8 * (lane >> 4);
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            fa[x][p] = *reinterpret_cast<const bf8*>(&la[p][32 * wm + 16 * x + (lane & 15)][ko]);
            fb[x][p] = *reinterpret_cast<const bf8*>(&lb[p][32 * wn + 16 * x + (lane & 15)][ko]);
          }
        constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};  // small terms first
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
              acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[x][TA[q]], fb[y][TB[q]], acc[x][y], 0, 0, 0);
      }
    }
  }
  float* part = tn_part(G, P, t, sk);
  if (gemm) {  // lane holds C[m = 4 (lane >> 4) + i][n = lane & 15] of each 16 x 16 block
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 32 * wm + 16 * x + 4 * (lane >> 4) + i, c = 32 * wn + 16 * y + (lane & 15);
          const float v = acc[x][y][i];
          if (part) {
            part[r * TV + c] = v;
            continue;
          }
          const int m = m0 + r, n = n0 + c;
          if (m >= P.M || n >= Nr) continue;
          float* out = P.C + (size_t)m * P.ldc + n;
          *out = P.beta ? *out + v : v;
        }
  } else if (part) {  // a bias-only tile: its partial's GEMM block is zero
    for (int e = tid; e < TV * TV; e += 256) part[e] = 0.f;
  }
  if (do_bias) {  // column sums of A: the 16 row lanes of each column quad, in order
    *reinterpret_cast<f4*>(&rsum[kr0][q4]) = rs;
    __syncthreads();
    if (tid < TV) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) v += rsum[i][tid];
      if (part) {
        part[TV * TV + tid] = v;
      } else {
        const int m = m0 + tid;
        if (m < P.M) {
          float* out = P.Cb ? P.Cb + m : P.C + (size_t)m * P.ldc + (P.N - 1);
          *out = P.beta ? *out + v : v;
        }
      }
    }
  }
}

}  // namespace tnx3

// ---------------------------------------------------------------------------------------------------
// The grouped TN GEMM on the bf16 MFMA at fp32 accuracy with NO LDS staging (TMDNET_TN_V=5).  The k index
// of an MFMA is a summation label, so a lane may feed ANY 8 rows as its k group as long as its A and B
// fragments use the same rows: lane (c, g) loads rows kb + 8g + j (j < 8), A columns m0 + 4c .. + 3 and B
// columns n0 + 4c .. + 3 as float4 (coalesced 256-byte row segments per 16 lanes), and the 8 values of
// A column m0 + 4c + mb ARE the lane's fragment of 16 x 16 block mb (MFMA row label c) -- k_gemm_tn_v's
// label permutation with 8 k per lane instead of one.  Each value is split in registers into its three
// exact bf16 pieces (proj::split3) and the six piece products with i + j <= 2 run as 16x16x32 bf16 MFMAs:
// 96 MFMAs of 16 cycles per 32-row step of a 64 x 64 tile against the f32 kernel's 128 of 32.  The split
// of a step happens before the next step's loads are issued (the raw registers are then free), so the
// loads fly during the MFMAs.  Tile numbering, split-K partial layout, bias (A's column sums from the raw
// values) and the cross-wave reduction are k_gemm_tn_v's.  Not for one-hot A.
namespace tnx3r {

using gemm::GroupTN;
using gemm::ProbTN;
using gemm::TV;
using gemm::TV_PART;
using gemm::TNLoc;
using gemm::tn_locate;
using gemm::tn_part;
using bf8 = __bf16 __attribute__((ext_vector_type(8)));
using f4 = float __attribute__((ext_vector_type(4)));
using u4 = unsigned __attribute__((ext_vector_type(4)));
constexpr int KS = 32;  // rows per step (4 k groups x 8)

// element i of 8 float4 (rows k .. k + 7 of the lane's group) -> the three bf16 fragments
__device__ __forceinline__ void split_col(const f4 (&x)[8], int i, bf8 (&f)[3]) {
  unsigned h[8], m[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) proj::split3(x[j][i], h[j], m[j], l[j]);
  u4 H, M, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // element 2p in the low half of register p
    H[p] = (h[2 * p] >> 16) | h[2 * p + 1];
    M[p] = (m[2 * p] >> 16) | m[2 * p + 1];
    L[p] = (l[2 * p] >> 16) | l[2 * p + 1];
  }
  f[0] = __builtin_bit_cast(bf8, H);
  f[1] = __builtin_bit_cast(bf8, M);
  f[2] = __builtin_bit_cast(bf8, L);
}

template <int NW>
__global__ __launch_bounds__(NW * 64, 2) void k_gemm_tn_x3r(GroupTN G) {
  __shared__ float red[NW][TV][TV + 1];
  __shared__ float redb[NW][TV];
  const TNLoc L = tn_locate(G);
  const ProbTN& P = G.p[L.pi];
  const int t = L.t, sk = L.sk;
  const int w = threadIdx.x / TMD_WAVE, lane = lane_id();
  const int c = lane & 15, kg = lane >> 4;
  const int m0 = (t / P.tiles_n) * TV, n0 = (t % P.tiles_n) * TV;
  const bool anyones = P.ones1 || P.ones2;
  const int Nr = anyones ? P.N - 1 : P.N;
  const bool do_bias = anyones && (t % P.tiles_n) == 0;
  // (a device row count shortens both segments: the chunks split the rows actually summed)
  const int cnt = P.rows ? max(0, *P.rows) : P.K + P.K2;
  const int K1 = min(P.K, cnt), KT = K1 + min(P.K2, cnt);
  const int nkt = (KT + KS - 1) / KS, cper = (nkt + P.S - 1) / P.S;
  const int c_lo = min(KT, sk * cper * KS), c_hi = min(KT, (sk + 1) * cper * KS);
  const int nkb = (c_hi - c_lo + KS - 1) / KS, per = (nkb + NW - 1) / NW;
  const int k_lo = min(c_hi, c_lo + w * per * KS), k_hi = min(c_hi, c_lo + (w + 1) * per * KS);
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  f4 rs = f4{0.f, 0.f, 0.f, 0.f};
  const int ma = m0 + 4 * c, na = n0 + 4 * c;
  const bool mfull = ma + 3 < P.M, nfull = na + 3 < Nr;
  const bool gemm = n0 < Nr;
  for (int seg = 0; seg < 2; ++seg) {
    const int s0 = seg ? K1 : 0, s1 = seg ? KT : K1;
    const int lo = max(k_lo, s0), hi = min(k_hi, s1);
    if (lo >= hi) continue;
    const float* A = seg ? P.A2 : P.A;
    const float* B = seg ? P.B2 : P.B;
    const int lda = seg ? P.lda2 : P.lda, ldb = seg ? P.ldb2 : P.ldb;
    const bool bias_seg = do_bias && (seg ? P.ones2 : P.ones1);
    const bool rb = gemm && B;
    auto load = [&](int kb, f4 (&a)[8], f4 (&b)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kb + 8 * kg + j;
        const bool kv = k < hi;
        const size_t ro = (size_t)(kv ? k - s0 : 0);
        if (kv && mfull) {
          a[j] = *reinterpret_cast<const f4*>(A + ro * lda + ma);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[j][i] = (kv && ma + i < P.M) ? A[ro * lda + ma + i] : 0.f;
        }
        if (!rb) {
          b[j] = f4{0.f, 0.f, 0.f, 0.f};
        } else if (kv && nfull) {
          b[j] = *reinterpret_cast<const f4*>(B + ro * ldb + na);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) b[j][i] = (kv && na + i < Nr) ? B[ro * ldb + na + i] : 0.f;
        }
      }
    };
    f4 a[8], b[8];
    load(lo, a, b);
    for (int kb = lo; kb < hi; kb += KS) {
      if (bias_seg) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rs += a[j];
      }
      bf8 fa[4][3], fb[4][3];
      if (gemm) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          split_col(a, i, fa[i]);
          split_col(b, i, fb[i]);
        }
      }
      if (kb + KS < hi) load(kb + KS, a, b);  // in flight during this step's MFMAs
      if (gemm) {
        constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};  // small terms first
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
              acc[mb][nb] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mb][TA[q]], fb[nb][TB[q]], acc[mb][nb], 0, 0, 0);
      }
    }
  }
  // C layout of a 16x16 block: lane holds MFMA rows 4 (lane >> 4) + i, column lane & 15 (labels as above)
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][4 * (4 * kg + i) + mb][4 * c + nb] = acc[mb][nb][i];
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      rs[i] = v;
    }
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) redb[w][4 * c + i] = rs[i];
    }
  }
  __syncthreads();
  float* part = tn_part(G, P, t, sk);
  for (int e = threadIdx.x; e < TV * TV; e += blockDim.x) {
    const int r = e >> 6, cc = e & 63;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) v += red[i][r][cc];
    if (part) {
      part[e] = v;
      continue;
    }
    const int m = m0 + r, n = n0 + cc;
    if (m >= P.M || n >= Nr) continue;
    float* out = P.C + (size_t)m * P.ldc + n;
    if (P.beta) v += *out;
    *out = v;
  }
  if (do_bias) {
    for (int r = threadIdx.x; r < TV; r += blockDim.x) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) v += redb[i][r];
      if (part) {
        part[TV * TV + r] = v;
        continue;
      }
      const int m = m0 + r;
      if (m >= P.M) continue;
      float* out = P.Cb ? P.Cb + m : P.C + (size_t)m * P.ldc + (P.N - 1);
      if (P.beta) v += *out;
      *out = v;
    }
  }
}

}  // namespace tnx3r

namespace emb {
constexpr int MAX_TABLES = 4;
struct Tables {
  int n_tables, H4;  // H / 4
  const float* t[MAX_TABLES];
  int ldt[MAX_TABLES];
  float* out[MAX_TABLES];
  int ldo[MAX_TABLES];
};
// out_t[k][:] = table_t[z[k]][:] for every table sharing z: one thread per float4 of one output row
// (x = node-major float4 index, y = table).  An index outside [0, num_types) is an error of the caller
// (nn.Embedding raises): the debug build asserts it, the release build writes zeros.
__global__ __launch_bounds__(256) void k_embed_fwd(int n, int num_types, const int64_t* __restrict__ z, Tables T) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int t = blockIdx.y;
  if (i >= (long long)n * T.H4) return;
  const int k = (int)(i / T.H4), c = (int)(i % T.H4);
  const long long m = z[k];
  TMD_DCHECK(m >= 0 && m < num_types);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (m >= 0 && m < num_types) v = reinterpret_cast<const float4*>(T.t[t] + (size_t)m * T.ldt[t])[c];
  reinterpret_cast<float4*>(T.out[t] + (size_t)k * T.ldo[t])[c] = v;
}
}  // namespace emb
}  // namespace tmd

using namespace tmd;

static int gemm_run(gemm::Group& G, void* stream);

extern "C" int tmdnet_gemm_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream) {
  if (n_problems < 1 || n_problems > 4 || !dims || !ptrs) return kBadArgument;
  gemm::Group G{};
  G.n = n_problems;
  for (int i = 0; i < n_problems; ++i) {
    const int* d = dims + 8 * i;
    gemm::Prob& P = G.p[i];
    P.M = d[0]; P.N = d[1]; P.K = d[2]; P.lda = d[3]; P.ldb = d[4]; P.ldc = d[5];
    P.trans_b = d[6]; P.beta = d[7];
    P.A = (const float*)ptrs[4 * i];
    P.B = (const float*)ptrs[4 * i + 1];
    P.bias = (const float*)ptrs[4 * i + 2];
    P.C = (float*)ptrs[4 * i + 3];
  }
  return gemm_run(G, stream);
}

extern "C" int tmdnet_gemm_ex_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream) {
  if (n_problems < 1 || n_problems > 4 || !dims || !ptrs) return kBadArgument;
  gemm::Group G{};
  G.n = n_problems;
  for (int i = 0; i < n_problems; ++i) {
    const int* d = dims + 10 * i;
    gemm::Prob& P = G.p[i];
    P.M = d[0]; P.N = d[1]; P.K = d[2]; P.lda = d[3]; P.ldb = d[4]; P.ldc = d[5];
    P.trans_b = d[6]; P.beta = d[7]; P.act = d[8]; P.ldx = d[9];
    const void* const* q = ptrs + 7 * i;
    P.A = (const float*)q[0];
    P.B = (const float*)q[1];
    P.bias = (const float*)q[2];
    P.C = (float*)q[3];
    P.pre = (float*)q[4];
    P.rscale = (const float*)q[5];
    P.dpre = (const float*)q[6];
    if (P.act != 0 && P.act != 1) return kUnsupported;
    if ((P.pre || P.dpre) && P.ldx < P.N) return kBadArgument;
  }
  return gemm_run(G, stream);
}

static int gemm_run(gemm::Group& G, void* stream) {
  const int n_problems = G.n;
  int tiles = 0;
  for (int i = 0; i < n_problems; ++i) {
    gemm::Prob& P = G.p[i];
    if (P.M <= 0 || P.N <= 0 || P.K <= 0 || !P.A || !P.B || !P.C) return kBadArgument;
    // K in 16-wide blocks (a wave's K slice may be empty: K = 32 over 4 waves leaves two idle)
    if (P.K % 16 || P.lda % 4 || (P.trans_b && P.ldb % 4) || P.lda < P.K || P.ldc < P.N) return kUnsupported;
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
  // K blocks per wave of the longest problem -> the smallest load batch that covers it in one go
  // (a longer slice loops over batches, so any KMAX is correct; the choice only sizes registers)
  const int per = (kmax / 16 + nw - 1) / nw;
  hipStream_t st = (hipStream_t)stream;
  bool ex = false;  // any epilogue extension (tmdnet_gemm_ex_f32) in this launch
  for (int i = 0; i < n_problems; ++i)
    ex = ex || G.p[i].pre || G.p[i].act || G.p[i].rscale || G.p[i].dpre;
#define TMD_GEMM_LAUNCH(NW_, KB_)                                                                   \
  if (ex) hipLaunchKernelGGL((gemm::k_gemm<NW_, KB_, true>), dim3(tiles), dim3(NW_ * 64), 0, st, G); \
  else hipLaunchKernelGGL((gemm::k_gemm<NW_, KB_, false>), dim3(tiles), dim3(NW_ * 64), 0, st, G)
  if (nw <= 2) TMD_GEMM_LAUNCH(2, 8);
  else if (nw >= 16) {
    // (the 16-wave launches measured equal with 1-, 2- and 3-block batches: one 1024-thread block per
    // CU at any of them; TMDNET_GEMM_KB16 forces one)
    static const int kb16 = [] { const char* e = getenv("TMDNET_GEMM_KB16"); return e ? atoi(e) : 0; }();
    const int kb = kb16 ? kb16 : per;
    if (kb <= 1) TMD_GEMM_LAUNCH(16, 1);
    else if (kb == 2) TMD_GEMM_LAUNCH(16, 2);
    else if (kb == 3) TMD_GEMM_LAUNCH(16, 3);
    else TMD_GEMM_LAUNCH(16, 4);
  } else if (nw >= 8) {
    if (per <= 2) TMD_GEMM_LAUNCH(8, 2);
    else TMD_GEMM_LAUNCH(8, 8);
  } else {
    // a 2-block slice loaded one block at a time: 46 VGPRs = 8 waves per SIMD instead of 84 = 4,
    // and the second load is hidden by the other resident tiles (ET-QM9 training step: the 32
    // K = H launches 257 -> 232 us; TMDNET_GEMM_KB4=2 restores the one-batch load)
    static const int kb4 = [] { const char* e = getenv("TMDNET_GEMM_KB4"); return e ? atoi(e) : 1; }();
    if (per <= 2 && kb4 <= 1) TMD_GEMM_LAUNCH(4, 1);
    else if (per <= 2) TMD_GEMM_LAUNCH(4, 2);
    else if (per <= 4) TMD_GEMM_LAUNCH(4, 4);
    else TMD_GEMM_LAUNCH(4, 8);
  }
#undef TMD_GEMM_LAUNCH
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// split-K factor: few tiles over many rows (e.g. a 128 x 64 weight over 12.5k edges is 8 tiles)
// leave most CUs idle; S 4-wave workgroups per tile (~1024 workgroups in all), each wave >= 64 rows
static int tn_target() {  // A/B switch TMDNET_TN_TARGET: workgroups aimed at by the split (default 1024)
  const char* te = getenv("TMDNET_TN_TARGET");
  return te ? max(64, atoi(te)) : 1024;
}

static int tn_split(int tiles, int kmax, int target = tn_target()) {
  int S = (target + tiles - 1) / tiles;
  S = min(S, max(1, kmax / (4 * 64)));
  return max(1, min(S, 64));
}

// the 16-byte-load kernel needs every A / B row 16-byte aligned (one-hot A: any)
static bool tn_vec_ok(const gemm::GroupTN& G) {
  static const bool off = getenv("TMDNET_TN_SCALAR") != nullptr;  // A/B switch
  if (off) return false;
  auto al = [](const void* p, int ld) { return !p || ((((uintptr_t)p) & 15) == 0 && ld % 4 == 0); };
  for (int i = 0; i < G.n; ++i) {
    const gemm::ProbTN& P = G.p[i];
    if (P.Cb && !(P.ones1 || P.ones2)) return false;  // a read column N-1 redirected to Cb: the 32-tile kernel
    if (!(P.onehot || al(P.A, P.lda)) || !al(P.B, P.ldb)) return false;
    if (P.K2 > 0 && (!al(P.A2, P.lda2) || !al(P.B2, P.ldb2))) return false;
  }
  return true;
}

// (re)number the tiles for tile edge T; returns the tile count
static int tn_tiles(gemm::GroupTN& G, int T) {
  int tiles = 0;
  for (int i = 0; i < G.n; ++i) {
    gemm::ProbTN& P = G.p[i];
    const int nr = (T == gemm::TV && (P.ones1 || P.ones2)) ? P.N - 1 : P.N;
    P.tiles_n = max(1, (nr + T - 1) / T);
    P.tile0 = tiles;
    tiles += ((P.M + T - 1) / T) * P.tiles_n;
  }
  return tiles;
}

// The 64-tile kernels' split: rows per workgroup = the group's (tile x row) work over ~target workgroups, at
// least 4 waves x 64 rows, and S = ceil(rows of the problem / that) per problem (<= 64), so the workgroups of
// a 3N-row problem and of an N-row one take about equally long (one S for the group left the vec_proj
// tiles of the node weight gradients three times longer than the others).  Shapes only (the workspace
// query uses it too).  Returns the workgroup count; parts = partial tiles of the S > 1 problems.
struct TNShape {
  int M, Nr, KT;
};
static int tn_plan_v(int n, const TNShape* sh, bool split, int* S, int* ntiles, long long* part0, long long& parts) {
  long long work = 0;
  for (int i = 0; i < n; ++i) {
    ntiles[i] = ((sh[i].M + gemm::TV - 1) / gemm::TV) * max(1, (sh[i].Nr + gemm::TV - 1) / gemm::TV);
    work += (long long)ntiles[i] * sh[i].KT;
  }
  const long long target = tn_target(), rows = max(256LL, (work + target - 1) / target);
  int wgs = 0;
  parts = 0;
  for (int i = 0; i < n; ++i) {
    S[i] = split ? (int)max(1LL, min(64LL, (sh[i].KT + rows - 1) / rows)) : 1;
    part0[i] = parts;
    if (S[i] > 1) parts += (long long)ntiles[i] * S[i];
    wgs += ntiles[i] * S[i];
  }
  return wgs;
}

static void launch_tn(gemm::GroupTN& G, int tiles, int kmax, float* ws, hipStream_t st) {
  if (tn_vec_ok(G)) {
    const int tv = tn_tiles(G, gemm::TV);
    TNShape sh[gemm::TN_MAX];
    int S[gemm::TN_MAX], nt[gemm::TN_MAX];
    long long p0[gemm::TN_MAX], parts = 0;
    for (int i = 0; i < G.n; ++i) {
      const gemm::ProbTN& P = G.p[i];
      sh[i] = TNShape{P.M, (P.ones1 || P.ones2) ? P.N - 1 : P.N, P.K + P.K2};
    }
    const int wgs = tn_plan_v(G.n, sh, ws != nullptr, S, nt, p0, parts);
    G.S = 1;
    for (int i = 0, w0 = 0; i < G.n; ++i) {
      gemm::ProbTN& P = G.p[i];
      P.S = S[i];
      P.ntiles = nt[i];
      P.part0 = p0[i];
      P.wg0 = w0;
      w0 += nt[i] * S[i];
      G.S = max(G.S, S[i]);  // (> 1: some problem writes partial tiles)
    }
    G.part = ws;
    bool narrow = true;  // every problem reads <= 32 columns of B
    for (int i = 0; i < G.n; ++i) {
      const gemm::ProbTN& P = G.p[i];
      narrow = narrow && ((P.ones1 || P.ones2) ? P.N - 1 : P.N) <= 32;
    }
    // (read per launch: tests compare the forms in one process).  Default: the pipelined 32-column form
    // for narrow groups (4096 x 32 over 6.6k + 6.6k rows: 80 vs 96 us), k_gemm_tn_v for 64-wide tiles
    // (the pipelined form at 2 waves per SIMD: 289 vs 210 us on the dk/dv weight gradient, 4096 x 64)
    const char* fe = getenv("TMDNET_TN_V");
    const int form = fe ? atoi(fe) : (narrow ? 2 : 1);
    bool onehot = false;
    for (int i = 0; i < G.n; ++i) onehot = onehot || G.p[i].onehot;
    if (form == 4 && !onehot) {
      hipLaunchKernelGGL(tnx3::k_gemm_tn_x3, dim3(wgs), dim3(256), 0, st, G);
    } else if (form == 5 && !onehot) {
      hipLaunchKernelGGL(tnx3r::k_gemm_tn_x3r<4>, dim3(wgs), dim3(256), 0, st, G);
    } else if (form == 2 || form == 3) {
      const bool pipe = form == 2;
      if (kmax >= 8192 && G.S == 1) {
        if (narrow) hipLaunchKernelGGL((gemm::k_gemm_tn_v2<8, 2, true>), dim3(tv), dim3(512), 0, st, G);
        else hipLaunchKernelGGL((gemm::k_gemm_tn_v2<8, 4, true>), dim3(tv), dim3(512), 0, st, G);
      } else if (narrow) {
        if (pipe) hipLaunchKernelGGL((gemm::k_gemm_tn_v2<4, 2, true>), dim3(wgs), dim3(256), 0, st, G);
        else hipLaunchKernelGGL((gemm::k_gemm_tn_v2<4, 2, false>), dim3(wgs), dim3(256), 0, st, G);
      } else {
        if (pipe) hipLaunchKernelGGL((gemm::k_gemm_tn_v2<4, 4, true>), dim3(wgs), dim3(256), 0, st, G);
        else hipLaunchKernelGGL((gemm::k_gemm_tn_v2<4, 4, false>), dim3(wgs), dim3(256), 0, st, G);
      }
    } else if (kmax >= 8192 && G.S == 1) {
      hipLaunchKernelGGL(gemm::k_gemm_tn_v<8>, dim3(tv), dim3(512), 0, st, G);
    } else {
      hipLaunchKernelGGL(gemm::k_gemm_tn_v<4>, dim3(wgs), dim3(256), 0, st, G);
    }
    if (G.S > 1)
      hipLaunchKernelGGL(gemm::k_tn_reduce_v, dim3((tv * gemm::TV_PART + 255) / 256), dim3(256), 0, st, G, tv);
    return;
  }
  tiles = tn_tiles(G, 32);
  G.S = ws ? tn_split(tiles, kmax) : 1;
  G.part = ws;
  // unsplit: K over 16 waves from 8192 rows (edge sums), 4 below (atom sums: a wave's slice stays long
  // enough to amortise the partial-tile reduction); split: 4 waves over each chunk
  if (kmax >= 8192 && G.S == 1) hipLaunchKernelGGL(gemm::k_gemm_tn<16>, dim3(tiles), dim3(1024), 0, st, G);
  else hipLaunchKernelGGL(gemm::k_gemm_tn<4>, dim3(tiles * G.S), dim3(256), 0, st, G);
  if (G.S > 1) hipLaunchKernelGGL(gemm::k_tn_reduce, dim3((tiles * 1024 + 255) / 256), dim3(256), 0, st, G, tiles);
}

// Embedding-table gradients (reference nn.Embedding backward, used by TorchMD_ET.embedding and
// NeighborEmbedding.embedding): out_t[m][c] (+)= sum_{k: z[k] == m} grad_t[k][c] for n_tables tables
// sharing the indices, as one-hot TN GEMMs in ONE launch -- deterministic (no atomics), no sort.
extern "C" int tmdnet_embedding_bwd_f32(int n, int H, int num_types, const int64_t* z, int n_tables,
                                        const void* const* grads, const int* ld_grads, void* const* outs,
                                        int accumulate, void* stream) {
  if (n < 0 || H <= 0 || num_types <= 0 || n_tables < 1 || n_tables > gemm::TN_MAX || !z || !grads || !outs)
    return kBadArgument;
  gemm::GroupTN G{};
  G.n = n_tables;
  int tiles = 0;
  for (int i = 0; i < n_tables; ++i) {
    gemm::ProbTN& P = G.p[i];
    if (!grads[i] || !outs[i] || (ld_grads && ld_grads[i] < H)) return kBadArgument;
    P.M = num_types; P.N = H; P.K = n; P.K2 = 0;
    P.lda = 1; P.ldb = ld_grads ? ld_grads[i] : H; P.ldc = H; P.beta = accumulate ? 1 : 0;
    P.onehot = 1;
    P.A = (const float*)z; P.B = (const float*)grads[i]; P.C = (float*)outs[i];
    P.tiles_n = (P.N + 31) / 32;
    P.tile0 = tiles;
    tiles += ((P.M + 31) / 32) * P.tiles_n;
  }
  launch_tn(G, tiles, n, nullptr, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// Embedding lookups of n_tables tables sharing the indices z (TorchMD_ET.embedding and
// NeighborEmbedding.embedding, reference torchmd_et.py:170, utils.py:92) in ONE launch.
extern "C" int tmdnet_embedding_fwd_f32(int n, int H, int num_types, const int64_t* z, int n_tables,
                                        const void* const* tables, const int* ld_tables, void* const* outs,
                                        const int* ld_outs, void* stream) {
  if (n < 0 || H <= 0 || num_types <= 0 || n_tables < 1 || n_tables > emb::MAX_TABLES || !tables || !outs)
    return kBadArgument;
  if (n == 0) return kOk;
  if (!z) return kBadArgument;
  if (H % 4) return kUnsupported;
  emb::Tables T{};
  T.n_tables = n_tables;
  T.H4 = H / 4;
  for (int i = 0; i < n_tables; ++i) {
    if (!tables[i] || !outs[i]) return kBadArgument;
    T.t[i] = (const float*)tables[i];
    T.out[i] = (float*)outs[i];
    T.ldt[i] = ld_tables ? ld_tables[i] : H;
    T.ldo[i] = ld_outs ? ld_outs[i] : H;
    if (T.ldt[i] < H || T.ldo[i] < H || T.ldt[i] % 4 || T.ldo[i] % 4) return kUnsupported;
    if ((((uintptr_t)tables[i]) | ((uintptr_t)outs[i])) & 15) return kUnsupported;
  }
  const long long items = (long long)n * T.H4;
  if (items > 2147483647LL * 256) return kUnsupported;
  const dim3 g((unsigned)((items + 255) / 256), n_tables);
  hipLaunchKernelGGL(emb::k_embed_fwd, g, dim3(256), 0,
                     (hipStream_t)stream, n, num_types, z, T);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// dims: 12 ints per problem {M, N, K, K2, lda, ldb, lda2, ldb2, ldc, beta, ones1, ones2};
// ptrs: 5 per problem {A, B, A2, B2, C} (A2 / B2 NULL when K2 = 0).
static int tn_group(int n_problems, const int* dims, const void* const* ptrs, int np, gemm::GroupTN& G, int& tiles,
                    int& kmax) {
  if (n_problems < 1 || n_problems > gemm::TN_MAX || !dims || !ptrs) return kBadArgument;
  G.n = n_problems;
  tiles = 0;
  kmax = 0;
  for (int i = 0; i < n_problems; ++i) {
    const int* d = dims + 12 * i;
    gemm::ProbTN& P = G.p[i];
    P.M = d[0]; P.N = d[1]; P.K = d[2]; P.K2 = d[3]; P.lda = d[4]; P.ldb = d[5]; P.lda2 = d[6]; P.ldb2 = d[7];
    P.ldc = d[8]; P.beta = d[9]; P.ones1 = d[10]; P.ones2 = d[11];
    const void* const* q = ptrs + (size_t)np * i;
    P.A = (const float*)q[0]; P.B = (const float*)q[1];
    P.A2 = (const float*)q[2]; P.B2 = (const float*)q[3]; P.C = (float*)q[4];
    P.Cb = np > 5 ? (float*)q[5] : nullptr;
    P.rows = np > 6 ? (const int*)q[6] : nullptr;
    if (P.M <= 0 || P.N <= 0 || P.K < 0 || P.K2 < 0 || !P.C || P.ldc < P.N - (P.Cb ? 1 : 0)) return kBadArgument;
    if ((P.K > 0 && (!P.A || (!P.B && !(P.ones1 && P.N == 1)) || P.lda < P.M)) ||
        (P.K2 > 0 && (!P.A2 || (!P.B2 && !(P.ones2 && P.N == 1)) || P.lda2 < P.M)))
      return kBadArgument;
    P.tiles_n = (P.N + 31) / 32;
    P.tile0 = tiles;
    tiles += ((P.M + 31) / 32) * P.tiles_n;
    kmax = max(kmax, P.K + P.K2);
  }
  return kOk;
}

static int gemm_tn(int n_problems, const int* dims, const void* const* ptrs, int np, void* workspace,
                   size_t workspace_bytes, void* stream) {
  gemm::GroupTN G{};
  int tiles = 0, kmax = 0;
  const int rc = tn_group(n_problems, dims, ptrs, np, G, tiles, kmax);
  if (rc != kOk) return rc;
  float* ws = (float*)workspace;
  if (ws && workspace_bytes < tmdnet_gemm_tn_workspace_bytes(n_problems, dims)) return kWorkspaceTooSmall;
  launch_tn(G, tiles, kmax, ws, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_gemm_tn_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream) {
  return gemm_tn(n_problems, dims, ptrs, 5, nullptr, 0, stream);
}

extern "C" size_t tmdnet_gemm_tn_workspace_bytes(int n_problems, const int* dims) {
  if (n_problems < 1 || n_problems > gemm::TN_MAX || !dims) return 0;
  int tiles = 0, kmax = 0;  // the shapes only (tn_group's tiling)
  for (int i = 0; i < n_problems; ++i) {
    const int* d = dims + 12 * i;
    tiles += ((d[0] + 31) / 32) * ((d[1] + 31) / 32);
    kmax = max(kmax, d[2] + d[3]);
  }
  TNShape sh[gemm::TN_MAX];  // the 64-tile kernels' plan (bias rides in the first column tile)
  for (int i = 0; i < n_problems; ++i) {
    const int* d = dims + 12 * i;
    sh[i] = TNShape{d[0], (d[10] || d[11]) ? d[1] - 1 : d[1], d[2] + d[3]};
  }
  int Sv[gemm::TN_MAX], nt[gemm::TN_MAX];
  long long p0[gemm::TN_MAX], parts = 0;
  tn_plan_v(n_problems, sh, true, Sv, nt, p0, parts);
  const int S = tn_split(tiles, kmax);
  const size_t b32 = S > 1 ? sizeof(float) * 1024 * (size_t)tiles * S : 0;
  const size_t bv = sizeof(float) * gemm::TV_PART * (size_t)parts;
  return max(b32, bv);
}

extern "C" int tmdnet_gemm_tn_f32_ws(int n_problems, const int* dims, const void* const* ptrs, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  return gemm_tn(n_problems, dims, ptrs, 6, workspace, workspace_bytes, stream);
}

extern "C" int tmdnet_gemm_tn_rows_f32_ws(int n_problems, const int* dims, const void* const* ptrs, void* workspace,
                                          size_t workspace_bytes, void* stream) {
  return gemm_tn(n_problems, dims, ptrs, 7, workspace, workspace_bytes, stream);
}

// Wp [3][N][K] (bf16 bit patterns) = the exact three-piece split of W [N][K] (ldw), see tmd::proj.
extern "C" int tmdnet_proj_split_f32(int N, int K, const void* W, int ldw, void* Wp, void* stream) {
  if (N <= 0 || K <= 0 || !W || !Wp) return kBadArgument;
  if (K % 4 || ldw < K || ldw % 4 || (((uintptr_t)W) & 15) || (((uintptr_t)Wp) & 7)) return kUnsupported;
  const int n4 = N * K / 4;
  hipLaunchKernelGGL(proj::k_proj_split, dim3((n4 + 255) / 256), dim3(256), 0, (hipStream_t)stream, N, K,
                     (const float*)W, ldw, (unsigned short*)Wp);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// C [M][N] = A [M][K] W [N][K]^T (+ bias [N]) from Wp = tmdnet_proj_split_f32(W) (rows of the pieces
// piece_stride elements apart: a row slice of a larger split is Wp + row0 * K with the full stride).
// fp32 in / out on the bf16 MFMA.  K = 32 or 64, N % 16 == 0, 16-byte aligned rows.
extern "C" int tmdnet_proj_f32(int M, int N, int K, const void* A, int lda, const void* Wp,
                               long long piece_stride, const void* bias, void* C, int ldc, void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || !A || !Wp || !C) return kBadArgument;
  if (M == 0) return kOk;
  if ((K != 32 && K != 64) || N % 16 || lda < K || ldc < N || lda % 4 || ldc % 4 || piece_stride < (long long)N * K)
    return kUnsupported;
  if ((((uintptr_t)A) | ((uintptr_t)Wp) | ((uintptr_t)C) | ((uintptr_t)bias)) & 15) return kUnsupported;
  static const int mb_env = getenv("TMDNET_PROJ_MB") ? atoi(getenv("TMDNET_PROJ_MB")) : 0;  // tuning
  static const int bn_env = getenv("TMDNET_PROJ_BN") ? atoi(getenv("TMDNET_PROJ_BN")) : 0;
  // measured (tools/proj_time.py): C2 [6613 x 64] x [64 x 4096] 38 us at 128 x 64 tiles (library 48);
  // C5 [1.36M x 64] x [64 x 512] 0.90 ms at 256 x 128 (library 1.07)
  const bool big = M >= 65536;
  const int mb_req = mb_env ? mb_env : (big ? 4 : 2), bn_req = bn_env ? bn_env : (big ? 128 : 64);
  // the tile that is actually instantiated for this K (the grid is derived from it, not from the
  // request: K = 32 has only 64-column tiles)
  const int bn = (K == 64 && bn_req >= 128) ? 128 : 64;
  const int mb = mb_req >= 4 ? 4 : (mb_req >= 2 || bn == 128 || K == 32) ? 2 : 1;
  proj::Args P{M, N, lda, ldc, piece_stride, (const float*)A, (const unsigned short*)Wp, (const float*)bias,
               (float*)C};
  const dim3 g((N + bn - 1) / bn, (M + 64 * mb - 1) / (64 * mb));
  hipStream_t st = (hipStream_t)stream;
#define TMD_PROJ(KS_, MB_, BN_) hipLaunchKernelGGL((proj::k_proj_x3<KS_, MB_, BN_>), g, dim3(256), 0, st, P)
  if (K == 64) {
    if (bn == 128) {
      if (mb == 4) TMD_PROJ(2, 4, 128); else TMD_PROJ(2, 2, 128);
    } else {
      if (mb == 4) TMD_PROJ(2, 4, 64); else if (mb == 2) TMD_PROJ(2, 2, 64); else TMD_PROJ(2, 1, 64);
    }
  } else {
    if (mb == 4) TMD_PROJ(1, 4, 64); else TMD_PROJ(1, 2, 64);
  }
#undef TMD_PROJ
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

extern "C" int tmdnet_split_t_f32(int N, int K, const void* B, int ldb, void* Bp, void* stream) {
  if (N <= 0 || K <= 0 || !B || !Bp) return kBadArgument;
  if (K % 4 || ldb < N || (((uintptr_t)Bp) & 7)) return kUnsupported;
  const int n = N * (K / 4);
  hipLaunchKernelGGL(proj::k_split_t, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, N, K,
                     (const float*)B, ldb, (unsigned short*)Bp);
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

// C [M][N] = beta C + A [M][K] Bp^T + bias (Bp: tmdnet_proj_split_f32 of a [N][K] weight, or
// tmdnet_split_t_f32 of a [K][N] right operand); fp32 in / out at fp32 accuracy on the bf16 MFMA.
// K % 32 == 0, N % 16 == 0, 16-byte aligned rows and pointers.
extern "C" int tmdnet_gemm_x3_f32(int M, int N, int K, const void* A, int lda, const void* Bp, const void* bias,
                                  void* C, int ldc, int beta, void* stream) {
  return tmdnet_gemm_x3_ex_f32(M, N, K, A, lda, Bp, bias, C, ldc, beta, 0, nullptr, nullptr, nullptr, 0, stream);
}

// tmdnet_gemm_x3_f32 with tmdnet_gemm_ex_f32's epilogue: pre (the pre-activation, row stride ldx), act (SiLU),
// rscale (per-row scale), dpre (times silu'(dpre), row stride ldx) -- the Linear + SiLU stacks of large
// systems (TensorNet's edge MLP over ~1M pair rows at C5) without separate activation passes.
static int gemm_x3_launch(int M, int N, int K, const void* A, int lda, const void* Bp, const void* W, int ldw, int ws,
                          const void* bias, void* C, int ldc, int beta, int act, void* pre, const void* rscale,
                          const void* dpre, int ldx, void* stream);

extern "C" int tmdnet_gemm_x3_ex_f32(int M, int N, int K, const void* A, int lda, const void* Bp, const void* bias,
                                     void* C, int ldc, int beta, int act, void* pre, const void* rscale,
                                     const void* dpre, int ldx, void* stream) {
  if (!Bp) return kBadArgument;
  return gemm_x3_launch(M, N, K, A, lda, Bp, nullptr, 0, 0, bias, C, ldc, beta, act, pre, rscale, dpre, ldx, stream);
}

// The same with the right operand given as fp32 and split inside the kernel while it is staged in LDS:
// trans_w = 1: W [N][K] (a Linear weight, C = A W^T); trans_w = 0: W [K][N] (C = A W).  ldw % 4 == 0,
// W 16-byte aligned.
extern "C" int tmdnet_gemm_x3w_f32(int M, int N, int K, const void* A, int lda, const void* W, int ldw, int trans_w,
                                   const void* bias, void* C, int ldc, int beta, int act, void* pre,
                                   const void* rscale, const void* dpre, int ldx, void* stream) {
  if (!W) return kBadArgument;
  if (ldw % 4 || (((uintptr_t)W) & 15) || ldw < (trans_w ? K : N)) return kUnsupported;
  return gemm_x3_launch(M, N, K, A, lda, nullptr, W, ldw, trans_w ? 1 : 2, bias, C, ldc, beta, act, pre, rscale,
                        dpre, ldx, stream);
}

static int gemm_x3_launch(int M, int N, int K, const void* A, int lda, const void* Bp, const void* W, int ldw, int ws,
                          const void* bias, void* C, int ldc, int beta, int act, void* pre, const void* rscale,
                          const void* dpre, int ldx, void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || !A || !C) return kBadArgument;
  if (M == 0) return kOk;
  if (K % 32 || N % 16 || lda < K || ldc < N || lda % 4 || ldc % 4) return kUnsupported;
  if ((((uintptr_t)A) | ((uintptr_t)Bp) | ((uintptr_t)C) | ((uintptr_t)bias)) & 15) return kUnsupported;
  if ((pre || dpre) && (ldx < N || ldx % 4 || ((((uintptr_t)pre) | ((uintptr_t)dpre)) & 15))) return kUnsupported;
  static const int remap_env = [] {
    const char* e = getenv("TMDNET_X3_REMAP");
    return e ? atoi(e) : 1;
  }();
  proj::XArgs P{M, N, K, lda, ldc, beta ? 1 : 0, 0, 0, 0, (const float*)A, (const unsigned short*)Bp,
                (const float*)bias, (float*)C, act ? 1 : 0, ldx, (float*)pre, (const float*)rscale,
                (const float*)dpre, (const float*)W, ldw};
  hipStream_t st = (hipStream_t)stream;
  // 64-column tiles for wide outputs (the forward mixes, N = 3H..5H), 128 for the narrow input gradients
  // (N = H: one column tile, A read once); 2 row blocks per wave (128 rows per workgroup).  Wide-form
  // alternatives measured slower at C5 (us for qkv / o / vec_proj): <2,64,1> 75.6 / 50.0 / 150.7,
  // <2,64,2> 93.8 / 58.3 / 167.3, <1,64,4> 106.1 / 65.2 / 192.0, <1,64,2> 96.6 / 59.2 / 181.9
  // TMDNET_X3_BN = 64 / 128 forces the tile width (A/B; read once per process)
  static const int bn_env = [] {
    const char* e = getenv("TMDNET_X3_BN");
    return e ? atoi(e) : 0;
  }();
  // auto: 128-column tiles for the narrow outputs (N < 256) and, for wide ones, from 131072 rows on (measured,
  // tools/x3_time.py / x3_tn_time.py: C5 ET vec_fwd 150k rows 155 -> 148 us, TensorNet's 1M-row edge MLP
  // 2110 -> 1836 us (256 -> 384), 1001 -> 854 (128 -> 256); at 50k rows the 64-wide form stays ahead: qkv_fwd
  // 79 vs 83, o_fwd 51 vs 56 us)
  const int bn = bn_env == 64 || bn_env == 128 ? bn_env
                                               : (N <= 64 ? 64 : (N < 256 || M >= 131072) ? 128 : 64);
  P.nx = (N + bn - 1) / bn;
  P.ny = (M + 127) / 128;
  P.remap = remap_env && P.nx > 1 && (long long)P.nx * P.ny < (1ll << 31);
  const dim3 g = P.remap ? dim3(P.nx * P.ny) : dim3(P.nx, P.ny);
#define TMD_X3(WS_)                                                               \
  if (bn == 64)                                                                   \
    hipLaunchKernelGGL((proj::k_gemm_x3<2, 64, 1, WS_>), g, dim3(256), 0, st, P);  \
  else                                                                            \
    hipLaunchKernelGGL((proj::k_gemm_x3<2, 128, 4, WS_>), g, dim3(256), 0, st, P);
  if (ws == 1) {
    TMD_X3(1)
  } else if (ws == 2) {
    TMD_X3(2)
  } else {
    TMD_X3(0)
  }
#undef TMD_X3
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}
