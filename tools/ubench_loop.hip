// Microbenchmark: GEMM main-loop structures (glds ring + MFMA) on the bench
// AE's GEMM shapes, to pick the production tiling.  Garbage-in (zeros), the
// output is a checksum only; timing is what matters.
// Variants: BM x BN block tile, WM x WN waves (2 waves/SIMD at 8 waves),
// NS-stage LDS ring (BK = 64 bf16), SK split-K slices, PF = register prefetch
// of the next k-step's fragments.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/ubench_loop tools/ubench_loop.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
#define LDSP __attribute__((address_space(3)))

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int ROWS, int NT>
__device__ __forceinline__ void issue(char* img, const __bf16* G, int ld, int r0, int k0, int tid) {
  constexpr int CH = ROWS * 128 / 16 / NT;
  static_assert(CH >= 1, "tile too small for thread count");
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int p = NT * i + tid;
    const int row = p >> 3, j = (p & 7) ^ ((row >> 1) & 7);
    const __bf16* src = G + (size_t)(r0 + row) * ld + k0 + j * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (LDSP void*)(img + (NT * i + (tid & ~63)) * 16), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag(const char* img, int r, int kk, int lane) {
  const int m = r + (lane & 15);
  const int c = (kk * 4 + (lane >> 4)) ^ ((m >> 1) & 7);
  return *(const bf16x8*)(img + m * 128 + c * 16);
}

template <int BM, int BN, int WM, int WN, int NS, int PF>
__global__ __launch_bounds__(64 * WM * WN, 1) void kloop(const __bf16* A, const __bf16* B, int K, int tiles_n,
                                                        int sk, float* out) {
  constexpr int NT = 64 * WM * WN;
  constexpr int SA = BM * 128, SB = BN * 128, SLOT = SA + SB;
  constexpr int NL = (BM + BN) * 128 / 16 / NT;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 16x16 tiles per wave
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const int wr = (w / WN) * (BM / WM), wc = (w % WN) * (BN / WN);
  const int slice = blockIdx.x % sk, tile = blockIdx.x / sk;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int kper = K / sk, kbase = slice * kper;
  const int nt = kper / 64;
  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    issue<BM, NT>(smem + s * SLOT, A, K, tm * BM, kbase + s * 64, tid);
    issue<BN, NT>(smem + s * SLOT + SA, B, K, tn * BN, kbase + s * 64, tid);
  }
  for (int t = 0; t < nt; ++t) {
    if (t + NS - 2 < nt) wait_vm<(NS - 2) * NL>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nt) {
      const int s = t + NS - 1;
      issue<BM, NT>(smem + (s % NS) * SLOT, A, K, tm * BM, kbase + s * 64, tid);
      issue<BN, NT>(smem + (s % NS) * SLOT + SA, B, K, tn * BN, kbase + s * 64, tid);
    }
    const char* sa = smem + (t % NS) * SLOT;
    const char* sb = sa + SA;
    if constexpr (PF) {
      bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa0[i] = frag(sa, wr + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb0[j] = frag(sb, wc + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa1[i] = frag(sa, wr + i * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb1[j] = frag(sb, wc + j * 16, 1, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[i], fb0[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag(sa, wr + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag(sb, wc + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 12345.f) out[0] = s;
}

template <int BM, int BN, int WM, int WN, int NS, int PF>
void run(const __bf16* A, const __bf16* B, int M, int N, int K, int sk, float* out) {
  if (M % BM || N % BN || (K / sk) % 64) return;
  const int tn = N / BN, grid = (M / BM) * tn * sk;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) kloop<BM, BN, WM, WN, NS, PF><<<grid, 64 * WM * WN>>>(A, B, K, tn, sk, out);
  const int it = 20;
  (void)hipEventRecord(e0);
  for (int i = 0; i < it; ++i) kloop<BM, BN, WM, WN, NS, PF><<<grid, 64 * WM * WN>>>(A, B, K, tn, sk, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it;
  printf("  %3dx%3d w%dx%d ns%d pf%d sk%d grid=%4d %8.2f us %7.1f TF\n", BM, BN, WM, WN, NS, PF, sk, grid, us,
         2.0 * M * N * K / us / 1e6);
}

void shape(const __bf16* A, const __bf16* B, int M, int N, int K, float* out) {
  printf("M=%d N=%d K=%d\n", M, N, K);
  for (int sk : {1, 2, 4}) {
    run<128, 128, 2, 2, 4, 0>(A, B, M, N, K, sk, out);
    run<128, 128, 2, 2, 4, 1>(A, B, M, N, K, sk, out);
    run<128, 128, 2, 4, 4, 0>(A, B, M, N, K, sk, out);
    run<128, 128, 4, 2, 4, 0>(A, B, M, N, K, sk, out);
    run<256, 128, 4, 2, 3, 0>(A, B, M, N, K, sk, out);
    run<256, 128, 4, 2, 3, 1>(A, B, M, N, K, sk, out);
    run<256, 128, 2, 2, 3, 0>(A, B, M, N, K, sk, out);
    run<128, 256, 2, 4, 3, 0>(A, B, M, N, K, sk, out);
    run<64, 128, 2, 2, 5, 0>(A, B, M, N, K, sk, out);
    run<64, 128, 2, 2, 5, 1>(A, B, M, N, K, sk, out);
  }
}

__global__ void init_k(__bf16* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (__bf16)((float)(h & 0xffff) / 32768.f - 1.f);
  }
}

int main(int argc, char** argv) {
  __bf16 *A, *B;
  float* out;
  (void)hipMalloc(&A, (size_t)4096 * 4096 * 2);
  (void)hipMalloc(&B, (size_t)4096 * 4096 * 2);
  (void)hipMalloc(&out, 64);
  init_k<<<1024, 256>>>(A, (size_t)4096 * 4096, 1u);
  init_k<<<1024, 256>>>(B, (size_t)4096 * 4096, 7u);
  (void)hipDeviceSynchronize();
  const int Bt = argc > 1 ? atoi(argv[1]) : 1024;
  shape(A, B, Bt, 1664, 2048, out);   // L0 fwd
  shape(A, B, Bt, 1280, 1664, out);   // L1 fwd
  shape(A, B, Bt, 896, 1280, out);    // L2 fwd
  shape(A, B, 1664, 2048, Bt, out);   // L0 dW (K = batch)
  return 0;
}
