// GPU-side cost of a launch, back to back on one stream (HIP events around
// 200 launches): empty kernels with small / 400-byte kernargs, with a 64 KiB
// static LDS footprint, reading kernarg fields, and a 416-block grid like the
// GEMMs'.  Run with HIP_FORCE_DEV_KERNARG=0 / 1 to see where kernargs live.
// Build: hipcc -O2 --offload-arch=gfx950 tools/ubench_launch.hip -o tools/ubench_launch
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { float* p[40]; int v[20]; };

__global__ void k_small(int* out) { if (out && threadIdx.x == 1023) out[0] = 1; }
__global__ void k_big(Big b) { if (b.p[0] && threadIdx.x == 1023) b.p[0][0] = (float)b.v[3]; }
__global__ void k_big_read(Big b) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += (float)b.v[i % 20] * (b.p[i] ? 1.f : 2.f);
  if (s == 1.2345e-30f) b.p[1][threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_big_lds(Big b) {
  __shared__ float sm[16384];   // 64 KiB
  sm[threadIdx.x] = (float)b.v[1];
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 255] == 1.2345e-30f) b.p[1][threadIdx.x] = 1.f;
}
__global__ __launch_bounds__(256) void k_big_lds_load(Big b, const float* __restrict__ bias) {
  __shared__ float sm[16384];
  const float v = bias[blockIdx.x * 64 + (threadIdx.x & 63)];
  sm[threadIdx.x] = v;
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 255] == 1.2345e-30f) b.p[1][threadIdx.x] = 1.f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename F>
float per_launch_us(F f, hipStream_t s) {
  for (int i = 0; i < 20; ++i) f();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < 200; ++i) f();
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / 200.f;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float* buf;
  CK(hipMalloc(&buf, 1 << 24));
  Big b{};
  for (int i = 0; i < 40; ++i) b.p[i] = nullptr;
  b.p[1] = buf;
  for (int i = 0; i < 20; ++i) b.v[i] = i;
  const char* ev = getenv("HIP_FORCE_DEV_KERNARG");
  printf("HIP_FORCE_DEV_KERNARG=%s\n", ev ? ev : "(unset)");
  for (int grid : {1, 256, 416, 832}) {
    printf("grid %4d: small %.2f  big %.2f  big_read %.2f  big_lds64k %.2f  big_lds64k+load %.2f us\n", grid,
           per_launch_us([&] { k_small<<<grid, 256, 0, s>>>(nullptr); }, s),
           per_launch_us([&] { k_big<<<grid, 256, 0, s>>>(b); }, s),
           per_launch_us([&] { k_big_read<<<grid, 256, 0, s>>>(b); }, s),
           per_launch_us([&] { k_big_lds<<<grid, 256, 0, s>>>(b); }, s),
           per_launch_us([&] { k_big_lds_load<<<grid, 256, 0, s>>>(b, buf); }, s));
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
