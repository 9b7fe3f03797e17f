// Microbenchmark: GEMM main-loop structures on gfx950 (both operands K-major,
// bf16, 16x16x32 MFMA), one block per CU, zero operands.
//   PIPE 0: per stage: wait stage t, barrier, issue t+NS-1, read all frags of
//           a 32-deep step then its MFMAs (the v3 kernel's loop)
//   PIPE 1: fragment registers double-buffered one 32-deep step ahead, one
//           barrier per stage placed between the stage's two MFMA groups,
//           all NS slots in flight (issue t+NS right after the barrier)
//   MODE bit0: operand streaming (global_load_lds), bit1: LDS reads + MFMA
//   S: split-K factor (grid = tiles * S, each block covers K / S)
// Build: hipcc -O3 --offload-arch=gfx950 -o build/ubench_pipe tools/ubench_pipe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
#define LDSP __attribute__((address_space(3)))

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

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

template <int TM, int TN>
__device__ __forceinline__ void read_frags(const char* sa, const char* sb, int ra, int rb, int kk, int lane,
                                           bf16x8 (&fa)[TM], bf16x8 (&fb)[TN]) {
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = ra + i * 16 + (lane & 15);
    fa[i] = *(const bf16x8*)(sa + m * 128 + (((kk * 4 + g) ^ ((m >> 1) & 7)) << 4));
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = rb + j * 16 + (lane & 15);
    fb[j] = *(const bf16x8*)(sb + n * 128 + (((kk * 4 + g) ^ ((n >> 1) & 7)) << 4));
  }
}

template <int TM, int TN>
__device__ __forceinline__ void mfmas(floatx4 (&acc)[TM][TN], const bf16x8 (&fa)[TM], const bf16x8 (&fb)[TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
}

// half H of the wave tile's MFMAs (rows i in [H*TM/2, (H+1)*TM/2))
template <int TM, int TN, int H>
__device__ __forceinline__ void mfmas_half(floatx4 (&acc)[TM][TN], const bf16x8 (&fa)[TM], const bf16x8 (&fb)[TN]) {
#pragma unroll
  for (int i = H * TM / 2; i < (H + 1) * TM / 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
}

template <int BM, int BN, int WM, int WN, int NS, int MODE, int PIPE, int PRIO>
__global__ __launch_bounds__(WM * WN * 64, 2) void kpipe(const __bf16* A, const __bf16* B, int K, int tiles_n,
                                                          int S, float* out) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int SA = BM * 128, SB = BN * 128, SLOT = SA + SB;
  constexpr int NL = (BM + BN) * 128 / 16 / NT;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const int wm = w / WN, wn = w % WN;
  const int nblk = gridDim.x, bid = blockIdx.x;
  int lt;
  {
    const int q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
    lt = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tile = lt / S, sk = lt % S;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int Ks = K / S, kbase = sk * Ks;
  const int nt = Ks / 64;
  const int ra = wm * 16 * TM, rb = wn * 16 * TN;
  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0, 0, 0, 0};
  auto iss = [&](int s) {
    char* base = smem + (s % NS) * SLOT;
    issue<BM, NT>(base, A, K, tm * BM, kbase + s * 64, tid);
    issue<BN, NT>(base + SA, B, K, tn * BN, kbase + s * 64, tid);
  };
  if constexpr (PIPE == 0) {
    if (MODE & 1)
      for (int s = 0; s < NS - 1; ++s)
        if (s < nt) iss(s);
    for (int t = 0; t < nt; ++t) {
      if (MODE & 1) {
        if (t + NS - 2 < nt) wait_vm<(NS - 2) * NL>(); else wait_vm<0>();
      }
      barrier();
      if ((MODE & 1) && t + NS - 1 < nt) iss(t + NS - 1);
      if (MODE & 2) {
        const char* sa = smem + (t % NS) * SLOT;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 fa[TM], fb[TN];
          read_frags<TM, TN>(sa, sa + SA, ra, rb, kk, lane, fa, fb);
          if (PRIO) __builtin_amdgcn_s_setprio(1);
          mfmas<TM, TN>(acc, fa, fb);
          if (PRIO) __builtin_amdgcn_s_setprio(0);
        }
      }
    }
  } else {
    // prologue: all NS slots in flight
    if (MODE & 1)
      for (int s = 0; s < NS; ++s)
        if (s < nt) iss(s);
    bf16x8 f0a[TM], f0b[TN], f1a[TM], f1b[TN];
    if (MODE & 1) {
      if (nt > NS - 1) wait_vm<(NS - 1) * NL>(); else wait_vm<0>();
    }
    barrier();
    if (MODE & 2) read_frags<TM, TN>(smem, smem + SA, ra, rb, 0, lane, f0a, f0b);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): no SMEM left in flight at the loop
    // one stage: F1 <- (t, kk1); MFMA(F0); [wait t+1, barrier, refill slot t,
    // F0 <- (t+1, kk0)]; MFMA(F1).  Straight-line bodies (no LDS op under a
    // branch) so the compiler's lgkmcnt stays counted.
    auto step = [&](int t, auto issue_c, auto last_c) {
      constexpr bool ISSUE = decltype(issue_c)::value, LAST = decltype(last_c)::value;
      const char* sa = smem + (t % NS) * SLOT;
      if (MODE & 2) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
        mfmas_half<TM, TN, 0>(acc, f0a, f0b);
        __builtin_amdgcn_sched_barrier(0);
        read_frags<TM, TN>(sa, sa + SA, ra, rb, 1, lane, f1a, f1b);
        __builtin_amdgcn_sched_barrier(0);
        mfmas_half<TM, TN, 1>(acc, f0a, f0b);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (!LAST) {
        if (MODE & 1) {
          if constexpr (ISSUE) {
            wait_vm<(NS - 2) * NL>();
          } else {
            const int rem = nt - t - 2;   // stages that may stay in flight
            if (rem >= 2 && NS >= 4) wait_vm<2 * NL>();
            else if (rem >= 1) wait_vm<NL>();
            else wait_vm<0>();
          }
        }
        wait_lgkm0();
        barrier();
        if constexpr (ISSUE) { if (MODE & 1) iss(t + NS); }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (MODE & 2) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
        mfmas_half<TM, TN, 0>(acc, f1a, f1b);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!LAST) {
          const char* sn = smem + ((t + 1) % NS) * SLOT;
          read_frags<TM, TN>(sn, sn + SA, ra, rb, 0, lane, f0a, f0b);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfmas_half<TM, TN, 1>(acc, f1a, f1b);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    int t = 0;
    for (; t < nt - NS; ++t) step(t, T_{}, F_{});
    for (; t < nt - 1; ++t) step(t, F_{}, F_{});
    step(nt - 1, F_{}, T_{});
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 12345.f) out[0] = s;
}

template <int BM, int BN, int WM, int WN, int NS, int MODE, int PIPE, int PRIO = 0>
void run(const char* name, const __bf16* A, const __bf16* B, int M, int N, int K, int S, float* out) {
  constexpr int NT = WM * WN * 64;
  const int tn = N / BN, grid = (M / BM) * tn * S;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) kpipe<BM, BN, WM, WN, NS, MODE, PIPE, PRIO><<<grid, NT>>>(A, B, K, tn, S, out);
  const int it = 20;
  (void)hipEventRecord(e0);
  for (int i = 0; i < it; ++i) kpipe<BM, BN, WM, WN, NS, MODE, PIPE, PRIO><<<grid, NT>>>(A, B, K, tn, S, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it;
  const double bytes = (double)grid * (BM + BN) * (K / S) * 2;
  const double fl = 2.0 * M * N * K;
  printf("%-34s M=%5d N=%5d K=%5d S=%d grid=%4d %8.2f us  L2->LDS %6.2f TB/s  %7.1f TF (%4.1f%%)\n", name, M, N, K,
         S, grid, us, bytes / us / 1e6, fl / us / 1e6, fl / us / 1e6 / 25.0);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 1024;
  const int N = 1664, K = 2048;
  __bf16 *A, *B;
  float* out;
  (void)hipMalloc(&A, (size_t)4096 * K * 2);
  (void)hipMalloc(&B, (size_t)2048 * K * 2);
  (void)hipMalloc(&out, 64);
  (void)hipMemset(A, 0, (size_t)4096 * K * 2);
  (void)hipMemset(B, 0, (size_t)2048 * K * 2);
  // 128x128, 4 waves (wave tile 64x64)
  run<128, 128, 2, 2, 4, 2, 0>("mfma  128x128 w4 pipe0", A, B, M, N, K, 1, out);
  run<128, 128, 2, 2, 4, 2, 1>("mfma  128x128 w4 pipe1", A, B, M, N, K, 1, out);
  run<128, 128, 2, 2, 4, 2, 1, 1>("mfma  128x128 w4 pipe1 prio", A, B, M, N, K, 1, out);
  run<128, 128, 2, 2, 4, 3, 0>("both  128x128 w4 pipe0", A, B, M, N, K, 1, out);
  run<128, 128, 2, 2, 4, 3, 1>("both  128x128 w4 pipe1", A, B, M, N, K, 1, out);
  run<128, 128, 2, 2, 4, 3, 1>("both  128x128 w4 pipe1", A, B, M, N, K, 2, out);
  run<128, 128, 2, 2, 4, 1, 1>("load  128x128 w4 pipe1", A, B, M, N, K, 2, out);
  run<128, 128, 2, 2, 4, 3, 1, 1>("both  128x128 w4 pipe1 prio", A, B, M, N, K, 2, out);
  run<128, 128, 2, 2, 3, 3, 1>("both  128x128 w4 pipe1 ns3", A, B, M, N, K, 2, out);
  // 128x128, 8 waves (wave tile 64x32)
  run<128, 128, 2, 4, 4, 2, 0>("mfma  128x128 w8 pipe0", A, B, M, N, K, 1, out);
  run<128, 128, 2, 4, 4, 2, 1>("mfma  128x128 w8 pipe1", A, B, M, N, K, 1, out);
  run<128, 128, 2, 4, 4, 3, 1>("both  128x128 w8 pipe1", A, B, M, N, K, 2, out);
  // 256x128, 8 waves (wave tile 64x64)
  run<256, 128, 4, 2, 3, 2, 0>("mfma  256x128 w8 pipe0", A, B, M, N, K, 1, out);
  run<256, 128, 4, 2, 3, 2, 1>("mfma  256x128 w8 pipe1", A, B, M, N, K, 1, out);
  run<256, 128, 4, 2, 3, 3, 1>("both  256x128 w8 pipe1", A, B, M, N, K, 1, out);
  run<256, 128, 4, 2, 3, 3, 1>("both  256x128 w8 pipe1", A, B, M, N, K, 4, out);
  run<256, 128, 4, 2, 3, 1, 1>("load  256x128 w8 pipe1", A, B, M, N, K, 4, out);
  // 256x128, 4 waves (wave tile 128x64)
  run<256, 128, 2, 2, 3, 2, 1>("mfma  256x128 w4 pipe1", A, B, M, N, K, 1, out);
  run<256, 128, 2, 2, 3, 3, 1>("both  256x128 w4 pipe1", A, B, M, N, K, 4, out);
  // 64x64 4 waves, the current winner
  run<64, 64, 2, 2, 4, 3, 0>("both  64x64 w4 pipe0", A, B, M, N, K, 1, out);
  run<64, 64, 2, 2, 4, 3, 1>("both  64x64 w4 pipe1", A, B, M, N, K, 1, out);
  return 0;
}
