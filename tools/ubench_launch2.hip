// Where the fixed cost of a dependent launch goes (HIP events around 200
// back-to-back launches on one stream, and the same 200 launches captured in
// one hipGraph): a trivial kernel; one global load per thread (cold buffer /
// the buffer the previous launch wrote / a buffer in the same 2 MiB page);
// 64 KiB static LDS with and without that load; a 3.4 MB store (a GEMM
// output's dirty bytes at the next boundary).
// Build: hipcc -O2 --offload-arch=gfx950 tools/ubench_launch2.hip -o tools/ubench_launch2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <functional>

__global__ __launch_bounds__(256) void k_empty(float* out) { if (out && threadIdx.x == 4096) out[0] = 1.f; }
__global__ __launch_bounds__(256) void k_load(const float* __restrict__ in, float* out) {
  const float v = in[(blockIdx.x * 256 + threadIdx.x) & 65535];
  if (v == 1.2345e-30f) out[threadIdx.x] = v;
}
__global__ __launch_bounds__(256) void k_lds(float* out) {
  __shared__ float sm[16384];
  sm[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 255] == 1.2345e-30f) out[threadIdx.x] = 1.f;
}
__global__ __launch_bounds__(256) void k_lds_load(const float* __restrict__ in, float* out) {
  __shared__ float sm[16384];
  sm[threadIdx.x] = in[(blockIdx.x * 256 + threadIdx.x) & 65535];
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 255] == 1.2345e-30f) out[threadIdx.x] = 1.f;
}
__global__ __launch_bounds__(256) void k_store(float* out, int n4) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256)
    ((float4*)out)[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

static float eager_us(const std::function<void()>& f, hipStream_t s) {
  for (int i = 0; i < 20; ++i) f();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < 200; ++i) f();
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / 200.f;
}
static float graph_us(const std::function<void()>& f, hipStream_t s) {
  hipGraph_t g; hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < 200; ++i) f();
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int r = 0; r < 3; ++r) (void)hipGraphLaunch(ge, s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
  return ms * 1000.f / 1000.f;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *a, *b, *big;
  CK(hipMalloc(&a, 1 << 24));
  CK(hipMalloc(&b, 1 << 24));
  CK(hipMalloc(&big, 64 << 20));
  CK(hipMemset(a, 0, 1 << 24));
  const int n4 = (int)(3.4e6 / 16);
  for (int grid : {32, 256, 512}) {
    struct V { const char* name; std::function<void()> f; };
    V vs[] = {
        {"empty", [&] { k_empty<<<grid, 256, 0, s>>>(nullptr); }},
        {"load", [&] { k_load<<<grid, 256, 0, s>>>(a, b); }},
        {"lds64k", [&] { k_lds<<<grid, 256, 0, s>>>(b); }},
        {"lds64k+load", [&] { k_lds_load<<<grid, 256, 0, s>>>(a, b); }},
        {"store3.4MB", [&] { k_store<<<grid, 256, 0, s>>>(big, n4); }},
        {"store3.4MB;load", [&] { k_store<<<grid, 256, 0, s>>>(big, n4); k_load<<<grid, 256, 0, s>>>(big, b); }},
    };
    for (auto& v : vs)
      printf("grid %4d %-18s eager %6.2f us/launch  graph %6.2f us/launch\n", grid, v.name, eager_us(v.f, s),
             graph_us(v.f, s));
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
