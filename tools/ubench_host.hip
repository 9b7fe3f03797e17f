// Host-side cost of the HIP operations one executor step issues: kernel
// launches (small and 400-byte kernarg structs; <<<>>>, hipExtLaunchKernelGGL,
// hipModuleLaunchKernel with a pre-packed kernarg buffer), hipEventRecord,
// cross-stream hipStreamWaitEvent (event flag variants) and the stream-memory
// pair hipStreamWriteValue32 / hipStreamWaitValue32.  Prints microseconds per
// call.  Build: hipcc -O2 --offload-arch=gfx950 tools/ubench_host.hip -o tools/ubench_host
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstring>

struct Big { float v[100]; int n; };

__global__ void empty_k(int* p) { if (p && threadIdx.x == 1234567) p[0] = 1; }
__global__ void big_k(Big b, int* p) { if (p && threadIdx.x == 1234567) p[0] = b.n; }
__global__ void ptr_k(const Big* b, int* p) { if (p && threadIdx.x == 1234567) p[0] = b->n; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename F>
double per_call_us(int n, F f, hipStream_t s, hipStream_t s2) {
  for (int i = 0; i < 50; ++i) f();
  (void)hipStreamSynchronize(s);
  (void)hipStreamSynchronize(s2);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(s);
  (void)hipStreamSynchronize(s2);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev_nf, ev_dt, ev_def;
  CK(hipEventCreateWithFlags(&ev_nf, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&ev_dt, hipEventDisableTiming));
  CK(hipEventCreate(&ev_def));
  Big b{};
  b.n = 3;
  Big* db = nullptr;
  CK(hipMalloc(&db, sizeof(Big)));
  CK(hipMemcpy(db, &b, sizeof(Big), hipMemcpyHostToDevice));
  unsigned int* flag = nullptr;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  hipFunction_t fbig;
  CK(hipGetFuncBySymbol(&fbig, reinterpret_cast<const void*>(big_k)));
  const int n = 2000;
  auto report = [](const char* what, double us) { printf("%-44s %7.2f us\n", what, us); };
  report("launch empty <<<256x256>>>", per_call_us(n, [&] { empty_k<<<256, 256, 0, s>>>(nullptr); }, s, s2));
  report("launch 400-B struct <<<832x256>>>",
         per_call_us(n, [&] { big_k<<<832, 256, 0, s>>>(b, nullptr); }, s, s2));
  report("launch pointer-to-struct <<<832x256>>>",
         per_call_us(n, [&] { ptr_k<<<832, 256, 0, s>>>(db, nullptr); }, s, s2));
  report("launch + hipGetLastError", per_call_us(n, [&] {
           big_k<<<832, 256, 0, s>>>(b, nullptr);
           (void)hipGetLastError();
         }, s, s2));
  report("hipExtLaunchKernelGGL 400-B", per_call_us(n, [&] {
           hipExtLaunchKernelGGL(big_k, dim3(832), dim3(256), 0, s, nullptr, nullptr, 0, b, nullptr);
         }, s, s2));
  {
    struct { Big b; int* p; } kargs;
    kargs.b = b;
    kargs.p = nullptr;
    size_t sz = sizeof(kargs);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &kargs, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    report("hipModuleLaunchKernel packed 400-B", per_call_us(n, [&] {
             (void)hipModuleLaunchKernel(fbig, 832, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
           }, s, s2));
  }
  report("hipEventRecord (no timing, no fence)", per_call_us(n, [&] { (void)hipEventRecord(ev_nf, s); }, s, s2));
  report("record+wait other stream (no timing/fence)", per_call_us(n, [&] {
           (void)hipEventRecord(ev_nf, s);
           (void)hipStreamWaitEvent(s2, ev_nf, 0);
         }, s, s2));
  report("record+wait other stream (no timing)", per_call_us(n, [&] {
           (void)hipEventRecord(ev_dt, s);
           (void)hipStreamWaitEvent(s2, ev_dt, 0);
         }, s, s2));
  report("record+wait other stream (default)", per_call_us(n, [&] {
           (void)hipEventRecord(ev_def, s);
           (void)hipStreamWaitEvent(s2, ev_def, 0);
         }, s, s2));
  report("record+wait same stream", per_call_us(n, [&] {
           (void)hipEventRecord(ev_nf, s);
           (void)hipStreamWaitEvent(s, ev_nf, 0);
         }, s, s2));
  report("launch s, record, wait s2, launch s2", per_call_us(n, [&] {
           big_k<<<832, 256, 0, s>>>(b, nullptr);
           (void)hipEventRecord(ev_nf, s);
           (void)hipStreamWaitEvent(s2, ev_nf, 0);
           big_k<<<832, 256, 0, s2>>>(b, nullptr);
         }, s, s2));
  unsigned int ctr = 0;
  report("writeValue32 s + waitValue32 s2", per_call_us(n, [&] {
           ++ctr;
           (void)hipStreamWriteValue32(s, flag, ctr, 0);
           (void)hipStreamWaitValue32(s2, flag, ctr, hipStreamWaitValueGte, 0xffffffffu);
         }, s, s2));
  report("launch s, write, wait s2, launch s2", per_call_us(n, [&] {
           ++ctr;
           big_k<<<832, 256, 0, s>>>(b, nullptr);
           (void)hipStreamWriteValue32(s, flag, ctr, 0);
           (void)hipStreamWaitValue32(s2, flag, ctr, hipStreamWaitValueGte, 0xffffffffu);
           big_k<<<832, 256, 0, s2>>>(b, nullptr);
         }, s, s2));
  report("hipStreamWriteValue32 alone", per_call_us(n, [&] {
           ++ctr;
           (void)hipStreamWriteValue32(s, flag, ctr, 0);
         }, s, s2));
  CK(hipStreamSynchronize(s));
  CK(hipStreamSynchronize(s2));
  CK(hipFree(db));
  CK(hipFree(flag));
  return 0;
}
