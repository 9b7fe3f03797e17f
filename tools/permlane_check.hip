// Checks mmad_common.h's lane_xor16 / lane_xor32 (v_permlane16/32_swap) against
// __shfl_xor(v, 16 / 32) on every lane of several waves, and sum_lane_groups
// against the shuffle form bit for bit.  Build: hipcc --offload-arch=gfx950
// -I include -I icra2021_multimodal_ad_amd/csrc tools/permlane_check.hip -o tools/permlane_check
#include <cstdio>
#include <hip/hip_runtime.h>
#include "mmad_common.h"

__global__ void k(const float* in, unsigned* bad) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const float v = in[t];
  unsigned b = 0;
  if (__builtin_bit_cast(unsigned, lane_xor16(v)) != __builtin_bit_cast(unsigned, __shfl_xor(v, 16))) b |= 1;
  if (__builtin_bit_cast(unsigned, lane_xor32(v)) != __builtin_bit_cast(unsigned, __shfl_xor(v, 32))) b |= 2;
  float s = v;
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  if (__builtin_bit_cast(unsigned, sum_lane_groups(v)) != __builtin_bit_cast(unsigned, s)) b |= 4;
  bad[t] = b;
}

int main() {
  const int n = 4 * 512;
  float h[n];
  for (int i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000003u) * 1e-3f - 300.f;
  float* d;
  unsigned* b;
  hipMalloc(&d, n * 4);
  hipMalloc(&b, n * 4);
  hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(4), dim3(512), 0, 0, d, b);
  unsigned hb[n];
  hipMemcpy(hb, b, n * 4, hipMemcpyDeviceToHost);
  int nb = 0;
  for (int i = 0; i < n; ++i) nb += hb[i] != 0;
  printf("permlane_check: %d of %d lanes differ (bits: 1 xor16, 2 xor32, 4 sum)\n", nb, n);
  if (nb) printf("first bad lane %d code %u\n", [&] { for (int i = 0; i < n; ++i) if (hb[i]) return i; return -1; }(), hb[0]);
  return nb != 0;
}
