// Microbenchmark: per-CU operand-feed rate from L2 (or the Infinity Cache)
// against the bytes a CU keeps in flight, for the two ways a GEMM can stage
// operands: LDS-DMA (global_load_lds_dwordx4, what mmad_gemm_kernel uses) and
// plain global_load_dwordx4 into VGPRs.  Question it answers: is the ~75 GB/s
// per CU the GEMM main loop reaches a latency x bytes-in-flight limit (then
// more in flight, e.g. register-staged prefetch beside the LDS ring, raises
// it) or a per-CU path limit (then only fewer bytes per FLOP help)?
// One workgroup per CU (grid 256), each wave streams 1 KiB per load
// instruction (16 B per lane, contiguous) with U loads outstanding.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_feed tools/ubench_feed.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef int int4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma16(const void* src, unsigned lds) {
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// register staging: U loads per wave outstanding, consumed (xor) in order
template <int U>
__global__ void feed_reg(const int4v* __restrict__ buf, unsigned mask, int iters, int* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // each wave walks its own 1 KiB blocks: block index = (wave_global * 97 + j) & mask
  unsigned blk = (unsigned)(blockIdx.x * nw + w) * 977u;
  int4v r[U];
  int4v acc = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < U; ++j) r[j] = buf[((blk + j) & mask) * 64 + lane];
  blk += U;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      acc ^= r[j];
      r[j] = buf[((blk + j) & mask) * 64 + lane];
    }
    blk += U;
  }
#pragma unroll
  for (int j = 0; j < U; ++j) acc ^= r[j];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x7fffffff) out[0] = 1;
}

// LDS-DMA: U 1 KiB DMAs per wave outstanding into a per-wave ring of U slots
template <int U>
__global__ void feed_lds(const int4v* __restrict__ buf, unsigned mask, int iters, int* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned blk = (unsigned)(blockIdx.x * nw + w) * 977u;
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)(smem + w * U * 1024));
#pragma unroll
  for (int j = 0; j < U; ++j) dma16(buf + ((blk + j) & mask) * 64 + lane, base + j * 1024);
  blk += U;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      wait_vm<U - 1>();   // slot j landed
      dma16(buf + ((blk + j) & mask) * 64 + lane, base + j * 1024);
    }
    blk += U;
  }
  wait_vm<0>();
  if (lane == 0 && smem[w * U * 1024] == 0x7f && iters < 0) out[0] = 1;
}

template <int U>
static void run(int mode, int nt, const int4v* buf, size_t bytes, int* out, const char* where) {
  const unsigned mask = (unsigned)(bytes / 1024) - 1;
  const int grid = 256, iters = 200;
  const int lds = mode ? (nt / 64) * U * 1024 : 0;
  if (lds > 160 * 1024) return;
  auto launch = [&]() {
    if (mode)
      hipLaunchKernelGGL(feed_lds<U>, dim3(grid), dim3(nt), lds, 0, buf, mask, iters, out);
    else
      hipLaunchKernelGGL(feed_reg<U>, dim3(grid), dim3(nt), 0, 0, buf, mask, iters, out);
  };
  if (mode) CHECK(hipFuncSetAttribute((const void*)feed_lds<U>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  for (int i = 0; i < 3; ++i) launch();
  CHECK(hipGetLastError());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 10;
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double per = ms / 1e3 / reps;
  const double total = (double)grid * (nt / 64) * (iters + 1) * U * 1024.0;
  const double inflight_kb = (nt / 64) * U;   // KiB outstanding per CU
  printf("%-4s %-5s waves/CU %2d  U %2d  in flight %4.0f KiB/CU  %7.2f us  %6.1f GB/s per CU  %5.2f TB/s chip\n",
         where, mode ? "dma" : "reg", nt / 64, U, inflight_kb, per * 1e6, total / per / 1e9 / grid,
         total / per / 1e12);
}

int main() {
  int* out;
  CHECK(hipMalloc(&out, 4));
  const size_t sizes[2] = {2u << 20, 64u << 20};   // L2-resident per XCD / Infinity Cache
  const char* names[2] = {"L2", "MALL"};
  for (int si = 0; si < 2; ++si) {
    int4v* buf;
    CHECK(hipMalloc(&buf, sizes[si]));
    CHECK(hipMemset(buf, 1, sizes[si]));
    for (int mode = 0; mode < 2; ++mode)
      for (int nt : {256, 512, 1024}) {
        run<1>(mode, nt, buf, sizes[si], out, names[si]);
        run<2>(mode, nt, buf, sizes[si], out, names[si]);
        run<4>(mode, nt, buf, sizes[si], out, names[si]);
        run<8>(mode, nt, buf, sizes[si], out, names[si]);
        run<16>(mode, nt, buf, sizes[si], out, names[si]);
        run<32>(mode, nt, buf, sizes[si], out, names[si]);
      }
    CHECK(hipFree(buf));
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
