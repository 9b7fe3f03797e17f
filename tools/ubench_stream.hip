// Microbenchmark: operand-streaming rate of the GEMM main loop without MFMA.
// Each block streams a BM x K (K-major) panel of A and a BN x K panel of B
// through an NS-stage LDS ring, exactly the GEMM's global->LDS traffic, and
// optionally runs MFMAs on garbage LDS (mode 2) or both (mode 3).
// Build: hipcc -O3 --offload-arch=gfx950 -o build/ubench_stream tools/ubench_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
#define LDSP __attribute__((address_space(3)))

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// one stage of one K-major operand: ROWS rows x 128 B, 16 B per lane, lane-linear LDS
template <int ROWS, int NT>
__device__ __forceinline__ void issue(char* img, const __bf16* G, int ld, int r0, int k0, int tid) {
  constexpr int CH = ROWS * 128 / 16 / NT;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int p = NT * i + tid;
    const int row = p >> 3, j = (p & 7) ^ ((row >> 1) & 7);
    const __bf16* src = G + (size_t)(r0 + row) * ld + k0 + j * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (LDSP void*)(img + (NT * i + (tid & ~63)) * 16), 16, 0, 0);
  }
}

template <int BM, int BN, int NS, int NT, int MODE>
__global__ __launch_bounds__(NT, 1) void kstream(const __bf16* A, const __bf16* B, int K, int tiles_n, float* out) {
  constexpr int SA = BM * 128, SB = BN * 128, SLOT = SA + SB;
  constexpr int NL = (BM + BN) * 128 / 16 / NT;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int nt = K / 64;
  floatx4 acc[4][4];
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0, 0, 0, 0};
  if (MODE & 1) {
    for (int s = 0; s < NS - 1; ++s) {
      issue<BM, NT>(smem + s * SLOT, A, K, tm * BM, s * 64, tid);
      issue<BN, NT>(smem + s * SLOT + SA, B, K, tn * BN, s * 64, tid);
    }
  }
  for (int t = 0; t < nt; ++t) {
    if (MODE & 1) {
      if (t + NS - 2 < nt) wait_vm<(NS - 2) * NL>(); else wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if ((MODE & 1) && t + NS - 1 < nt) {
      const int s = t + NS - 1;
      issue<BM, NT>(smem + (s % NS) * SLOT, A, K, tm * BM, s * 64, tid);
      issue<BN, NT>(smem + (s % NS) * SLOT + SA, B, K, tn * BN, s * 64, tid);
    }
    if (MODE & 2) {
      // wave tile 64x64 per wave (16 MFMA per k32), reads like the GEMM
      const char* sa = smem + (t % NS) * SLOT;
      const char* sb = sa + SA;
      const int wr = (w % (BM / 64)) * 64, wc = (w / (BM / 64)) * 64 % BN;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = *(const bf16x8*)(sa + (wr + i * 16 + (lane & 15)) * 128 + ((kk * 4 + (lane >> 4)) ^ (lane & 7)) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(sb + (wc + j * 16 + (lane & 15)) * 128 + ((kk * 4 + (lane >> 4)) ^ (lane & 7)) * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  float s = 0;
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 12345.f) out[0] = s;
}

template <int BM, int BN, int NS, int NT, int MODE>
void run(const char* name, const __bf16* A, const __bf16* B, int M, int N, int K, float* out) {
  const int tn = N / BN, grid = (M / BM) * tn;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) kstream<BM, BN, NS, NT, MODE><<<grid, NT>>>(A, B, K, tn, out);
  const int it = 20;
  hipEventRecord(e0);
  for (int i = 0; i < it; ++i) kstream<BM, BN, NS, NT, MODE><<<grid, NT>>>(A, B, K, tn, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it;
  const double bytes = (double)grid * (BM + BN) * K * 2;
  const double fl = 2.0 * M * N * K;
  printf("%-28s M=%5d N=%5d K=%5d grid=%4d  %8.2f us  L2->LDS %6.2f TB/s (%5.1f GB/s/blk)  %7.1f TF(eq)\n",
         name, M, N, K, grid, us, bytes / us / 1e6, bytes / grid / us / 1e3, fl / us / 1e6);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 1024;
  const int N = 1664, K = 2048;
  __bf16 *A, *B; float* out;
  hipMalloc(&A, (size_t)4096 * K * 2);
  hipMalloc(&B, (size_t)2048 * K * 2);
  hipMalloc(&out, 64);
  hipMemset(A, 0, (size_t)4096 * K * 2);
  hipMemset(B, 0, (size_t)2048 * K * 2);
  const int N2 = 1792;  // multiple of 256 for the 256-wide tiles
  run<64, 128, 5, 256, 1>("load 64x128 ns5 t256", A, B, M, N, K, out);
  run<128, 128, 4, 256, 1>("load 128x128 ns4 t256", A, B, M, N, K, out);
  run<128, 128, 4, 512, 1>("load 128x128 ns4 t512", A, B, M, N, K, out);
  run<128, 128, 3, 256, 1>("load 128x128 ns3 t256", A, B, M, N, K, out);
  run<256, 128, 3, 256, 1>("load 256x128 ns3 t256", A, B, M, N, K, out);
  run<256, 128, 3, 512, 1>("load 256x128 ns3 t512", A, B, M, N, K, out);
  run<256, 256, 2, 512, 1>("load 256x256 ns2 t512", A, B, M, N2, K, out);
  run<128, 128, 4, 256, 2>("mfma 128x128 (no load)", A, B, M, N, K, out);
  run<128, 128, 4, 256, 3>("both 128x128 ns4", A, B, M, N, K, out);
  run<256, 128, 3, 512, 3>("both 256x128 ns3 t512", A, B, M, N, K, out);
  run<256, 256, 2, 1024, 3>("both 256x256 ns2 t1024", A, B, M, N2, K, out);
  return 0;
}
