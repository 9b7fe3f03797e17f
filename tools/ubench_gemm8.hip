// Microbenchmark: candidate GEMM main loops for the 8-wave tiles (bf16,
// A [M][K] and B [N][K] both K-major = the forward GEMM), against the
// production kernel through the C-ABI, at the bench shapes.  Random operands
// (uniform [-1, 1)), checked against a naive fp32 GPU GEMM.
//
// Loop "stagger" (STAG = 1): a ring of NBUF K-tiles (64 deep) filled by
// LDS-DMA with a counted vmcnt and ONE raw barrier per K-tile; the two wave
// groups (waves 0-3 / 4-7, one of each per SIMD) place that barrier at
// different points of their program -- group 0 after both 32-deep k-steps of
// a tile, group 1 between them -- so on every SIMD one wave issues MFMAs while
// its partner waits at the barrier or reads fragments.  Every fragment of a
// tile is read (lgkmcnt(0)) before the barrier that frees its buffer.
// STAG = 0: both groups place the barrier after both k-steps (lockstep).
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 \
//          -o build/ubench_gemm8 tools/ubench_gemm8.hip -Iinclude \
//          -Licra2021_multimodal_ad_amd -lmmad -Wl,-rpath,$PWD/icra2021_multimodal_ad_amd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "mmad.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
#define LDSP __attribute__((address_space(3)))

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void dma16(const void* src, char* dst) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(LDSP void*)dst);
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}

// one K-tile (64 bf16 = 128 B per row) of a K-major operand: ROWS rows,
// 16-B chunk j of row r at chunk j ^ ((r >> 1) & 7)
template <int ROWS, int NT>
__device__ __forceinline__ void issue_op(char* img, const bf16* G, int ld, int r0, int k0, int tid) {
  constexpr int CH = ROWS * 128 / 16 / NT;
  static_assert(CH >= 1 && ROWS * 128 % (16 * NT) == 0, "tile / threads");
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int p = NT * i + tid;
    const int row = p >> 3, j = (p & 7) ^ ((row >> 1) & 7);
    dma16(G + (size_t)(r0 + row) * ld + k0 + j * 8, img + (NT * i + (tid & ~63)) * 16);
  }
}
__device__ __forceinline__ bf16x8 frag(const char* img, int rbase, int kk, int lane) {
  const int m = rbase + (lane & 15), g = lane >> 4;
  return *(const bf16x8*)(img + m * 128 + (((kk * 4 + g) ^ ((m >> 1) & 7)) << 4));
}

// DI = 1: the next tile's LDS-DMA spread over the MFMAs of the following
// k-step instead of issued in one burst after the barrier.  NOMMA: 1 = no MFMA
// (fragment reads and the DMA ring only: the operand-feed ceiling); 2 = no
// MFMA and no fragment reads either (the DMA ring and its barriers alone).
// NW: waves per workgroup (8, or 4 for 128x64 / 128x128 wave tiles).
template <int BM, int BN, int WM, int WN, int NBUF, int STAG, int DI = 0, int NOMMA = 0, int NW = 8>
__global__ __launch_bounds__(64 * NW, 1) void gemm8(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                bf16* __restrict__ C, int M, int N, int K, int tiles_n,
                                                int group_m, int store) {
  constexpr int NT = 64 * NW;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(WM * WN == NW, "wave grid");
  constexpr int ABYTES = BM * 128, SLOT = (BM + BN) * 128;
  constexpr int NL = SLOT / 16 / NT;                       // DMA per thread per K-tile
  static_assert(NBUF * SLOT <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int grp = w >> 2;
  // XCD-aware grouped tile order (as the production kernel)
  const int nblk = gridDim.x, bid = blockIdx.x;
  int tm, tn;
  {
    const int q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
    const int lt = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_m = nblk / tiles_n;
    const int per_group = group_m * tiles_n;
    const int first_m = (lt / per_group) * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    tm = first_m + (lt % per_group) % gsz;
    tn = (lt % per_group) / gsz;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nt = K / 64;
  const int ra = wm * 16 * TM, rb = wn * 16 * TN;
  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* base = smem + (t % NBUF) * SLOT;
    issue_op<BM, NT>(base, A, K, m0, t * 64, tid);
    issue_op<BN, NT>(base + ABYTES, B, K, n0, t * 64, tid);
  };
  // chunk q (0..NL-1) of tile t's DMA: A chunks first, then B
  constexpr int CHA = BM * 128 / 16 / NT;
  auto issue_q = [&](int t, int q) {
    char* base = smem + (t % NBUF) * SLOT;
    if (q < CHA) {
      const int p = NT * q + tid, row = p >> 3, j = (p & 7) ^ ((row >> 1) & 7);
      dma16(A + (size_t)(m0 + row) * K + t * 64 + j * 8, base + (NT * q + (tid & ~63)) * 16);
    } else {
      const int qq = q - CHA;
      const int p = NT * qq + tid, row = p >> 3, j = (p & 7) ^ ((row >> 1) & 7);
      dma16(B + (size_t)(n0 + row) * K + t * 64 + j * 8, base + ABYTES + (NT * qq + (tid & ~63)) * 16);
    }
  };
  int pend = -1;   // DI: tile whose DMA is still to be issued during the next MFMAs
  // wait until tile t+1 has landed, given no issue after t+NBUF-1 exists
  auto wait_next = [&](int t) {
    const int later = min(nt - 1, t + NBUF - 1) - (t + 1);   // tiles issued after t+1
    if (later >= 2) wait_vm<2 * NL>();
    else if (later == 1) wait_vm<NL>();
    else wait_vm<0>();
  };
  bf16x8 fa[2][TM], fb[2][TN];
  auto rd = [&](int t, int kk, int s) {
    if constexpr (NOMMA >= 2) return;
    const char* base = smem + (t % NBUF) * SLOT;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[s][i] = frag(base, ra + i * 16, kk, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[s][j] = frag(base + ABYTES, rb + j * 16, kk, lane);
  };
  auto mfma = [&](int s, int i, int j) {
    if constexpr (NOMMA) {
      asm volatile("" :: "v"(fa[s][i]), "v"(fb[s][j]));
    } else {
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
    }
  };
  auto pend_issue = [&](int i) {     // DI: this row's share of the pending DMA
    if constexpr (DI) {
      if (pend >= 0) {
#pragma unroll
        for (int q = 0; q < NL; ++q)
          if (q * TM / NL == i) issue_q(pend, q);
        if (i == TM - 1) pend = -1;
      }
    }
  };
  auto mma = [&](int s) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma(s, i, j);
      pend_issue(i);
    }
  };
  // [A](t): MFMAs of k-step 0 with the k-step-1 reads between them
  auto stepA = [&](int t) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma(0, i, j);
      pend_issue(i);
      if constexpr (NOMMA < 2) {
        if (i == 0) {
          const char* base = smem + (t % NBUF) * SLOT;
#pragma unroll
          for (int j = 0; j < TN; ++j) fb[1][j] = frag(base + ABYTES, rb + j * 16, 1, lane);
        }
        fa[1][i] = frag(smem + (t % NBUF) * SLOT, ra + i * 16, 1, lane);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto stepB = [&]() {
    __builtin_amdgcn_s_setprio(1);
    mma(1);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_issue = [&](int t) {      // after the last read of tile t
    wait_next(t);
    wait_lgkm0();
    bar();
    if (t + NBUF < nt) {
      if constexpr (DI) pend = t + NBUF;
      else issue(t + NBUF);
    }
  };

  // prologue
#pragma unroll
  for (int s = 0; s < NBUF; ++s)
    if (s < nt) issue(s);
  if (nt >= NBUF) {
    if constexpr (NBUF == 2) wait_vm<NL>();
    else wait_vm<(NBUF - 1) * NL>();
  } else {
    wait_vm<0>();
  }
  bar();
  rd(0, 0, 0);
  if (STAG && grp == 1) {
    for (int t = 0; t < nt; ++t) {
      stepA(t);
      if (t + 1 < nt) {
        sync_issue(t);
        __builtin_amdgcn_s_setprio(1);
        mma(1);
        __builtin_amdgcn_s_setprio(0);
        rd(t + 1, 0, 0);
      } else {
        stepB();
      }
    }
  } else {
    for (int t = 0; t < nt; ++t) {
      stepA(t);
      stepB();
      if (t + 1 < nt) {
        sync_issue(t);
        rd(t + 1, 0, 0);
      }
    }
  }
  const int g = lane >> 4, c = lane & 15;
  if (!store) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][3];
    if (s == 1.2345e-30f) C[tid] = (bf16)s;
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + ra + i * 16 + 4 * g + r, col = n0 + rb + j * 16 + c;
        C[(size_t)row * N + col] = (bf16)acc[i][j][r];
      }
}

__global__ void init_k(bf16* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (bf16)((float)(h & 0xffffff) / 8388608.f - 1.f);
  }
}
__global__ void ref_k(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(size_t)m * K + k] * (float)B[(size_t)n * K + k];
  C[(size_t)m * N + n] = s;
}

template <int BM, int BN, int WM, int WN, int NBUF, int STAG, int DI = 0, int NOMMA = 0, int NW = 8>
static float run(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int store, int iters) {
  const int tiles_m = M / BM, tiles_n = N / BN, ntiles = tiles_m * tiles_n;
  int gm = (int)(sqrt(ntiles / 8.0 * BN / BM) + 0.5);
  gm = gm < 1 ? 1 : (gm > tiles_m ? tiles_m : gm);
  auto launch = [&]() {
    gemm8<BM, BN, WM, WN, NBUF, STAG, DI, NOMMA, NW><<<ntiles, 64 * NW>>>(A, B, C, M, N, K, tiles_n, gm, store);
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / iters;
}

static float max_err(const bf16* Cd, const float* Rd, int M, int N) {
  std::vector<bf16> c((size_t)M * N);
  std::vector<float> r((size_t)M * N);
  CK(hipMemcpy(c.data(), Cd, c.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), Rd, r.size() * 4, hipMemcpyDeviceToHost));
  float e = 0.f;
  for (size_t i = 0; i < c.size(); ++i) {
    const float d = fabsf((float)c[i] - r[i]) / (1.f + fabsf(r[i]));
    e = d > e ? d : e;
  }
  return e;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096;
  const int N = argc > 2 ? atoi(argv[2]) : 1664;
  const int K = argc > 3 ? atoi(argv[3]) : 2048;
  const int iters = argc > 4 ? atoi(argv[4]) : 50;
  const int check = argc > 5 ? atoi(argv[5]) : 1;
  bf16 *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&R, (size_t)M * N * 4));
  init_k<<<1024, 256>>>(A, (size_t)M * K, 1u);
  init_k<<<1024, 256>>>(B, (size_t)N * K, 2u);
  if (check) ref_k<<<dim3((N + 255) / 256, M), 256>>>(A, B, R, M, N, K);
  CK(hipDeviceSynchronize());
  const double fl = 2.0 * M * N * K;
  auto report = [&](const char* name, float us, bool chk) {
    float e = -1.f;
    if (chk && check) e = max_err(C, R, M, N);
    printf("%-34s M=%d N=%d K=%d: %8.2f us  %7.1f TFLOP/s  %.3f of 2.5 PF  err %.2e\n", name, M, N, K,
           us, fl / us * 1e-6, fl / us * 1e-6 / 2500.0, e);
    fflush(stdout);
  };
  // production kernel (C-ABI): forward GEMM, no activation / stats
  {
    float* bias;
    CK(hipMalloc(&bias, N * 4));
    CK(hipMemset(bias, 0, N * 4));
    for (int tile : {-1, 0, 1, 2, 6}) {
      mmad_tune_set(0, tile);
      auto f = [&]() { return mmad_fc_fwd(MMAD_BF16, M, N, K, M, N, K, A, B, bias, 0, 0.f, nullptr, nullptr, C, nullptr, 0); };
      for (int i = 0; i < 3; ++i)
        if (f()) { printf("prod err %s\n", mmad_last_error_string()); return 1; }
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) f();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      char nm[64];
      snprintf(nm, sizeof nm, "production fc_fwd tile %d", tile);
      report(nm, ms * 1e3f / iters, true);
    }
    mmad_tune_set(0, -1);
  }
#define RUN(BM_, BN_, WM_, WN_, NB_, ST_, DI_, NW_)                                               \
  if (M % BM_ == 0 && N % BN_ == 0) {                                                           \
    char nm[64];                                                                                \
    snprintf(nm, sizeof nm, "gemm8 %dx%d w%dx%d nb%d st%d di%d", BM_, BN_, WM_, WN_, NB_, ST_, DI_); \
    report(nm, run<BM_, BN_, WM_, WN_, NB_, ST_, DI_, 0, NW_>(A, B, C, M, N, K, 1, iters), true); \
    snprintf(nm, sizeof nm, "  (no store)");                                                    \
    report(nm, run<BM_, BN_, WM_, WN_, NB_, ST_, DI_, 0, NW_>(A, B, C, M, N, K, 0, iters), false); \
    snprintf(nm, sizeof nm, "  (no MFMA: feed ceiling)");                                       \
    report(nm, run<BM_, BN_, WM_, WN_, NB_, ST_, DI_, 1, NW_>(A, B, C, M, N, K, 0, iters), false); \
    snprintf(nm, sizeof nm, "  (no MFMA, no reads: DMA ring)");                                 \
    report(nm, run<BM_, BN_, WM_, WN_, NB_, ST_, DI_, 2, NW_>(A, B, C, M, N, K, 0, iters), false); \
  }
  RUN(256, 128, 4, 2, 3, 0, 1, 8)
  RUN(256, 128, 2, 2, 3, 0, 1, 4)
  RUN(256, 128, 2, 2, 3, 0, 0, 4)
  RUN(256, 256, 2, 4, 2, 0, 1, 8)
  RUN(256, 256, 2, 2, 2, 0, 1, 4)
  return 0;
}
