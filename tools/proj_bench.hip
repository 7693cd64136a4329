#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"
// Micro-benchmark of hand-written f32-MFMA variants of the ET edge-feature projection GEMM
// (C = A B^T + bias, K = num_rbf = 64; C2: 6613 x 4096, C5: 1360782 x 512).  NEGATIVE RESULT, kept
// as the record: register-resident K tiles (no LDS), transposed MFMA tiles with 16-byte stores,
// LDS-staged full-row stores, 32x32x2, and a persistent variant with the next A tile in flight all
// reach 44-74 TF (C2) / 47-65 TF (C5), against hipBLASLt's 74 / 85 TF on the same shapes, so the
// model keeps the library GEMM for this product.
// Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I torchmd-net_amd/csrc -I include tools/proj_bench.hip -o /tmp/pb && /tmp/pb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.h"
using namespace tmd;
using f4 = float __attribute__((ext_vector_type(4)));

struct Proj { int M, N, lda, ldb, ldc, tiles_n; const float* A; const float* B; const float* bias; float* C; };

// VAR 0: all MFMAs then all stores; 1: per n-block compute + store; 2: as 1 with nontemporal stores
template <int KB, int VAR>
__global__ __launch_bounds__(256, 2) void k_proj(Proj P) {
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lb / P.tiles_n, tn = lb - tm * P.tiles_n;
  const int w = threadIdx.x / 64, lane = lane_id();
  const int lr = lane & 15, lk = lane >> 4;
  const int m0 = tm * 64 + (w >> 1) * 32, n0 = tn * 128 + (w & 1) * 64;
  f4 a[2][KB], b[4][KB];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float* ar = P.A + (size_t)min(m0 + 16 * i + lr, P.M - 1) * P.lda + 4 * lk;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) a[i][kb] = *reinterpret_cast<const f4*>(ar + 16 * kb);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* br = P.B + (size_t)min(n0 + 16 * j + lr, P.N - 1) * P.ldb + 4 * lk;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) b[j][kb] = *reinterpret_cast<const f4*>(br + 16 * kb);
  }
  if (VAR == 0 || VAR >= 4) {
    f4 acc[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 16 * j + 4 * lk;
      const f4 bv = (P.bias && n < P.N) ? *reinterpret_cast<const f4*>(P.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
      acc[0][j] = bv; acc[1][j] = bv;
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][kb][q], a[i][kb][q], acc[i][j], 0, 0, 0);
    if (VAR == 5) {  // no stores unless a value is NaN (never): load + MFMA time
      bool bad = false;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) bad |= acc[i][j].x != acc[i][j].x;
      if (bad) P.C[0] = 1.f;
      return;
    }
    if (VAR == 4) {  // stage the wave tile in LDS, store whole 256-byte row segments
      __shared__ __align__(16) float st[4][32][68];
      float (*t)[68] = st[w];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<f4*>(&t[16 * i + lr][16 * j + 4 * lk]) = acc[i][j];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      const int c = (lane & 15) * 4, r0 = lane >> 4;
#pragma unroll
      for (int rr = 0; rr < 32; rr += 4) {
        const int m = m0 + rr + r0, n = n0 + c;
        const f4 v = *reinterpret_cast<const f4*>(&t[rr + r0][c]);
        if (m < P.M && n < P.N) *reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n) = v;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + 16 * i + lr;
      if (m >= P.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + 16 * j + 4 * lk;
        if (n < P.N) *reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n) = acc[i][j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 16 * j + 4 * lk;
      const f4 bv = (P.bias && n < P.N) ? *reinterpret_cast<const f4*>(P.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
      f4 acc[2] = {bv, bv};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][kb][q], a[i][kb][q], acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = m0 + 16 * i + lr;
        if (m < P.M && n < P.N) {
          f4* dst = reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n);
          if (VAR == 2) __builtin_nontemporal_store(acc[i], dst);
          else *dst = acc[i];
        }
      }
    }
  }
}

// VAR 6: the workgroup keeps its B (weight) fragment in registers and walks `per` M tiles, the next
// tile's A rows in flight while the current tile's MFMAs run (software pipeline, unrolled by 2)
template <int KB>
__global__ __launch_bounds__(256, 2) void k_proj_p(Proj P, int per) {
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int g = lb / P.tiles_n, tn = lb - g * P.tiles_n;
  const int mtn = (P.M + 63) / 64;
  const int mt0 = g * per, mt1 = min(mtn, mt0 + per);
  if (mt0 >= mt1) return;
  const int w = threadIdx.x / 64, lane = lane_id();
  const int lr = lane & 15, lk = lane >> 4;
  const int mo = (w >> 1) * 32, n0 = tn * 128 + (w & 1) * 64;
  f4 b[4][KB], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* br = P.B + (size_t)min(n0 + 16 * j + lr, P.N - 1) * P.ldb + 4 * lk;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) b[j][kb] = *reinterpret_cast<const f4*>(br + 16 * kb);
    const int n = n0 + 16 * j + 4 * lk;
    bv[j] = (P.bias && n < P.N) ? *reinterpret_cast<const f4*>(P.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
  }
  auto load = [&](int mt, f4 (&x)[2][KB]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* ar = P.A + (size_t)min(mt * 64 + mo + 16 * i + lr, P.M - 1) * P.lda + 4 * lk;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) x[i][kb] = *reinterpret_cast<const f4*>(ar + 16 * kb);
    }
  };
  auto tile = [&](int mt, const f4 (&x)[2][KB]) {
    f4 acc[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[0][j] = bv[j]; acc[1][j] = bv[j]; }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][kb][q], x[i][kb][q], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = mt * 64 + mo + 16 * i + lr;
      if (m >= P.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + 16 * j + 4 * lk;
        if (n < P.N) *reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n) = acc[i][j];
      }
    }
  };
  f4 a0[2][KB], a1[2][KB];
  load(mt0, a0);
  for (int mt = mt0; mt < mt1; mt += 2) {
    if (mt + 1 < mt1) load(mt + 1, a1);
    tile(mt, a0);
    if (mt + 1 >= mt1) break;
    if (mt + 2 < mt1) load(mt + 2, a0);
    tile(mt + 1, a1);
  }
}

// VAR 3: 32x32x2 MFMA, wave tile 32 (M) x 64 (N) as 2 blocks of 32x32 (N along MFMA rows)
template <int KB>
__global__ __launch_bounds__(256, 2) void k_proj32(Proj P) {
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lb / P.tiles_n, tn = lb - tm * P.tiles_n;
  const int w = threadIdx.x / 64, lane = lane_id();
  const int lr = lane & 31, lk = lane >> 5;
  const int m0 = tm * 64 + (w >> 1) * 32, n0 = tn * 128 + (w & 1) * 64;
  constexpr int K8 = KB * 2;  // 8-wide K blocks
  f4 a[K8], b[2][K8];
  const float* ar = P.A + (size_t)min(m0 + lr, P.M - 1) * P.lda + 4 * lk;
#pragma unroll
  for (int kb = 0; kb < K8; ++kb) a[kb] = *reinterpret_cast<const f4*>(ar + 8 * kb);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float* br = P.B + (size_t)min(n0 + 32 * j + lr, P.N - 1) * P.ldb + 4 * lk;
#pragma unroll
    for (int kb = 0; kb < K8; ++kb) b[j][kb] = *reinterpret_cast<const f4*>(br + 8 * kb);
  }
  using f16v = float __attribute__((ext_vector_type(16)));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // D[row = n][col = m]: lane holds rows 8(g) + 4 (lane>>5)... standard 32x32 map:
    // row = (i / 4) * 8 + 4 * (lane >> 5) + (i % 4), col = lane & 31, i < 16
    f16v acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = n0 + 32 * j + 8 * g + 4 * lk;
      const f4 bv = (P.bias && n < P.N) ? *reinterpret_cast<const f4*>(P.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
      acc[4 * g] = bv.x; acc[4 * g + 1] = bv.y; acc[4 * g + 2] = bv.z; acc[4 * g + 3] = bv.w;
    }
#pragma unroll
    for (int kb = 0; kb < K8; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(b[j][kb][q], a[kb][q], acc, 0, 0, 0);
    const int m = m0 + lr;
    if (m < P.M) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + 32 * j + 8 * g + 4 * lk;
        if (n < P.N)
          *reinterpret_cast<f4*>(P.C + (size_t)m * P.ldc + n) = f4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
      }
    }
  }
}

int main(int argc, char** argv) {
  const int shapes[2][2] = {{6613, 4096}, {1360782, 512}};
  const int K = 64;
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1];
    float *A, *B, *bias, *C;
    hipMalloc(&A, (size_t)M * K * 4); hipMalloc(&B, (size_t)N * K * 4); hipMalloc(&bias, N * 4);
    hipMalloc(&C, (size_t)M * N * 4);
    std::vector<float> h((size_t)M * K);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    hipMemcpy(A, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice);
    hipMemcpy(B, h.data(), (size_t)N * K * 4, hipMemcpyHostToDevice);
    hipMemcpy(bias, h.data(), N * 4, hipMemcpyHostToDevice);
    Proj P{M, N, K, K, N, (N + 127) / 128, A, B, bias, C};
    const dim3 g((unsigned)(((M + 63) / 64) * P.tiles_n)), bl(256);
    std::vector<float> ref((size_t)M * N), out((size_t)M * N);
    for (int var = 0; var < 9; ++var) {
      const int mtn = (M + 63) / 64;
      const int per = var == 6 ? 4 : var == 7 ? 8 : 16;
      const int groups = (mtn + per - 1) / per;
      const dim3 gp((unsigned)(groups * P.tiles_n));
      auto launch = [&]() {
        if (var >= 6) { hipLaunchKernelGGL((k_proj_p<4>), gp, bl, 0, 0, P, per); return; }
        if (var == 0) hipLaunchKernelGGL((k_proj<4, 0>), g, bl, 0, 0, P);
        else if (var == 4) hipLaunchKernelGGL((k_proj<4, 4>), g, bl, 0, 0, P);
        else if (var == 5) hipLaunchKernelGGL((k_proj<4, 5>), g, bl, 0, 0, P);
        else if (var == 1) hipLaunchKernelGGL((k_proj<4, 1>), g, bl, 0, 0, P);
        else if (var == 2) hipLaunchKernelGGL((k_proj<4, 2>), g, bl, 0, 0, P);
        else hipLaunchKernelGGL((k_proj32<4>), g, bl, 0, 0, P);
      };
      for (int i = 0; i < 3; ++i) launch();
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      const int reps = M > 100000 ? 10 : 50;
      hipEventRecord(e0);
      for (int i = 0; i < reps; ++i) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      hipMemcpy(var == 0 ? ref.data() : out.data(), C, (size_t)M * N * 4, hipMemcpyDeviceToHost);
      double md = 0;
      if (var && var != 5) for (size_t i = 0; i < out.size(); i += 97) md = fmax(md, fabs(out[i] - ref[i]));
      printf("M=%d N=%d var=%d  %.4f ms  %.1f TF  maxdiff_vs_var0=%g\n", M, N, var, ms, 2.0 * M * N * K / (ms * 1e-3) / 1e12, md);
    }
    hipFree(A); hipFree(B); hipFree(bias); hipFree(C);
  }
  return 0;
}
