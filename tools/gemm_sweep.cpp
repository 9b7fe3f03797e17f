// Tile-plan sweep of the production GEMM kernels through the C-ABI (no
// Python in the timing loop).  For every GEMM of the bench AE (D=2048,
// btl=100, 5 layers) at a given batch, time each (cfg, split-K) plan and the
// automatic plan with hipEvents around 20 back-to-back launches.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/gemm_sweep tools/gemm_sweep.cpp \
//          -Licra2021_multimodal_ad_amd -lmmad -Wl,-rpath,$PWD/icra2021_multimodal_ad_amd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "../include/mmad.h"

static int pad(int x) { return (x + 127) / 128 * 128; }

__global__ void init_k(__bf16* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = (__bf16)(((float)(h & 0xffff) / 32768.f - 1.f) * scale);
  }
}

static double time_us(const std::function<int()>& fn, int iters = 20) {
  for (int i = 0; i < 3; ++i)
    if (fn() != 0) { printf("ERR %s\n", mmad_last_error_string()); exit(1); }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) fn();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int only = argc > 2 ? atoi(argv[2]) : -1;   // layer filter
  const int dbg = argc > 3 ? atoi(argv[3]) : 0;     // 1 skip main loop, 2 skip epilogue
  mmad_tune_set(3, dbg);
  printf("batch %d dbg %d\n", B, dbg);
  const int widths[11] = {2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048};
  const int Mp = pad(B);
  __bf16 *x, *w, *y, *dz, *dx;
  float *b, *st, *dw;
  (void)hipMalloc(&x, (size_t)Mp * 2048 * 2);
  (void)hipMalloc(&w, (size_t)2048 * 2048 * 2);
  (void)hipMalloc(&y, (size_t)Mp * 2048 * 2);
  (void)hipMalloc(&dz, (size_t)Mp * 2048 * 2);
  (void)hipMalloc(&dx, (size_t)Mp * 2048 * 2);
  (void)hipMalloc(&b, 2048 * 4);
  (void)hipMalloc(&st, (size_t)(Mp / 32) * 2 * 2048 * 4);
  (void)hipMalloc(&dw, (size_t)2048 * 2048 * 4);
  (void)hipMemset(b, 0, 2048 * 4);
  init_k<<<1024, 256>>>(x, (size_t)Mp * 2048, 1u, 1.f);
  init_k<<<1024, 256>>>(w, (size_t)2048 * 2048, 2u, 0.02f);
  init_k<<<1024, 256>>>(dz, (size_t)Mp * 2048, 3u, 1.f);
  (void)hipDeviceSynchronize();
  const int plans[] = {-1, 0, 1, 2, 3, 4, 5};
  const int BMs[] = {128, 256, 128, 64, 64, 128}, BNs[] = {128, 128, 256, 64, 128, 128};
  double tot_auto = 0, tot_best = 0;
  for (int li = 0; li < 10; ++li) {
    if (only >= 0 && li != only) continue;
    const int K = widths[li], N = widths[li + 1], Kp = pad(K), Np = pad(N);
    for (int kind = 0; kind < 3; ++kind) {
      auto fn = [&]() -> int {
        if (kind == 0)
          return mmad_fc_fwd(MMAD_BF16, B, N, K, Mp, Np, Kp, x, w, b, MMAD_ACT_LEAKYRELU, 0.2f, nullptr,
                             nullptr, y, st, nullptr);
        if (kind == 1) return mmad_fc_bwd_data(MMAD_BF16, B, N, K, Mp, Np, Kp, dz, w, dx, nullptr, nullptr);
        return mmad_fc_bwd_weight(MMAD_BF16, Mp, Np, Kp, dz, x, dw, nullptr);
      };
      const char* kn[3] = {"fwd", "bwd_data", "bwd_w"};
      const double fl = 2.0 * B * K * N;
      printf("L%d %-8s %4d->%4d:", li, kn[kind], K, N);
      double best = 1e30, au = 0;
      int bc = -1;
      for (int p : plans) {
        mmad_tune_set(0, p);
        // skip plans that do not divide the output
        const int om = kind == 2 ? Np : Mp, on = kind == 0 ? Np : Kp;
        if (p >= 0 && (om % BMs[p] || on % BNs[p])) continue;
        const double us = time_us(fn);
        if (p < 0) au = us;
        else if (us < best) { best = us; bc = p; }
        printf(" %s%d=%.1f", p < 0 ? "auto" : "c", p, us);
      }
      printf(" | auto %.1fus %.0fTF best c%d %.1fus %.0fTF\n", au, fl / au / 1e6, bc, best, fl / best / 1e6);
      tot_auto += au;
      tot_best += best;
      mmad_tune_set(0, -1);
    }
  }
  printf("total auto %.1f us, best %.1f us\n", tot_auto, tot_best);
  return 0;
}
