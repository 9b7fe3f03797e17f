// Where the fixed cost of a dependent launch goes (HIP events around 200
// back-to-back launches on one stream, and the same 200 launches captured in
// one hipGraph): a trivial kernel; one global load per thread (cold buffer /
// the buffer the previous launch wrote / a buffer in the same 2 MiB page);
// 64 KiB static LDS with and without that load; a 3.4 MB store (a GEMM
// output's dirty bytes at the next boundary).
// Build: hipcc -O2 --offload-arch=gfx950 tools/ubench_launch2.hip -o tools/ubench_launch2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
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

// the host cost of one hipGraphLaunch: a single-stream chain of 40 kernels vs
// the same 40 kernels captured across two streams (a fork / join event pair
// around every second kernel, like the train step's side-stream dW GEMMs)
static void graph_host(hipStream_t s, hipStream_t s2, float* b) {
  hipEvent_t ev[64];
  for (auto& e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (int forked = 0; forked < 2; ++forked) {
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    int k = 0;
    for (int i = 0; i < 40; ++i) {
      if (forked && i % 2 == 1) {
        (void)hipEventRecord(ev[k], s);
        (void)hipStreamWaitEvent(s2, ev[k++], 0);
        k_empty<<<256, 256, 0, s2>>>(b);
        (void)hipEventRecord(ev[k], s2);
        (void)hipStreamWaitEvent(s, ev[k++], 0);
      } else {
        k_empty<<<256, 256, 0, s>>>(b);
      }
    }
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 50; ++r) (void)hipGraphLaunch(ge, s);
    auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    printf("graph of 40 kernels, %s: host %.1f us per hipGraphLaunch, wall %.1f us per replay\n",
           forked ? "20 on a 2nd stream (fork/join events)" : "one stream",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 50,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / 50);
    (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
  }
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
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  graph_host(s, s2, b);
  CK(hipStreamSynchronize(s));
  return 0;
}
