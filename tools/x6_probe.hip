// Precision / speed probe: an fp32 GEMM on the bf16 matrix cores by operand
// splitting, against the exact-f32 MFMA chain the parity path runs.
//   f32 : v_mfma_f32_16x16x4_f32 chain (the exact-fp32 path's inner product)
//   x3  : x = hi + lo (two bf16), acc += hh + hl + lh          (3 MFMAs / 16 k)
//   x6  : x = hi + mid + lo (three bf16), acc += the six terms
//         down to 2^-16 relative, smallest first               (6 MFMAs / 16 k)
// with v_mfma_f32_16x16x16_bf16 (4 bf16 per lane).  One wave per 16x16
// output tile, fragments straight from global memory (a precision probe, not
// a tuned kernel), K = 2048; every output compared with an fp64 host GEMM.
// Reports per variant the max and RMS error relative to sum_k |a_k b_k| (the
// scale a rounding error of the sum is measured against) and the time of a
// MFMA-only loop (fragments in registers) per 16x16x16 block.
// Build: hipcc -O3 --offload-arch=gfx950 tools/x6_probe.hip -o tools/x6_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short ushortx8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ unsigned short bf16_rne(float x) {
  unsigned u = __builtin_bit_cast(unsigned, x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf16_f(unsigned short h) {
  return __builtin_bit_cast(float, (unsigned)h << 16);
}

// x = h + m + l (+ a residual below 2^-24 |x|): each difference is exact in fp32
__device__ __forceinline__ void split3(float x, short& h, short& m, short& l) {
  const unsigned short hb = bf16_rne(x);
  const float r1 = x - bf16_f(hb);
  const unsigned short mb = bf16_rne(r1);
  const float r2 = r1 - bf16_f(mb);
  h = (short)hb;
  m = (short)mb;
  l = (short)bf16_rne(r2);
}

template <int V>
__global__ void gemm_probe(const float* A, const float* B, float* C, int M, int N, int K) {
  // one wave per 16x16 tile; A [M][K] row-major, B [K][N] row-major
  const int lane = threadIdx.x;
  const int tm = blockIdx.x / (N / 16), tn = blockIdx.x % (N / 16);
  const int r = lane % 16, g = lane / 16;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 16) {
    if (V == 0) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float a = A[(size_t)(tm * 16 + r) * K + k0 + 4 * s + g];
        const float b = B[(size_t)(k0 + 4 * s + g) * N + tn * 16 + r];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      }
    } else {
      shortx4 ah, am, al, bh, bm, bl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = A[(size_t)(tm * 16 + r) * K + k0 + 4 * g + i];
        const float b = B[(size_t)(k0 + 4 * g + i) * N + tn * 16 + r];
        short h, m, l;
        split3(a, h, m, l);
        ah[i] = h; am[i] = m; al[i] = l;
        split3(b, h, m, l);
        bh[i] = h; bm[i] = m; bl[i] = l;
      }
      if (V == 1) {
        // two-way split: lo = bf16(x - hi) = bf16(m + l)
        shortx4 alo, blo;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          alo[i] = (short)bf16_rne(bf16_f((unsigned short)am[i]) + bf16_f((unsigned short)al[i]));
          blo[i] = (short)bf16_rne(bf16_f((unsigned short)bm[i]) + bf16_f((unsigned short)bl[i]));
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, blo, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(alo, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, acc, 0, 0, 0);
      } else {
        // smallest terms first: hl + lh + mm (2^-16), hm + mh (2^-8), hh
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(am, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(am, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, acc, 0, 0, 0);
      }
    }
  }
  // C/D: col = lane & 15, row = 4 * (lane >> 4) + i
#pragma unroll
  for (int i = 0; i < 4; ++i) C[(size_t)(tm * 16 + 4 * g + i) * N + tn * 16 + r] = acc[i];
}

// the same with v_mfma_f32_16x16x32_bf16 (8 bf16 per lane: k = 8g..8g+7)
// V = 3: two-way split (3 MFMAs per 16x16x32), V = 4: three-way (6 MFMAs)
template <int V>
__global__ void gemm_probe32(const float* A, const float* B, float* C, int M, int N, int K) {
  const int lane = threadIdx.x;
  const int tm = blockIdx.x / (N / 16), tn = blockIdx.x % (N / 16);
  const int r = lane % 16, g = lane / 16;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 32) {
    ushortx8 ah, am, al, bh, bm, bl;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float a = A[(size_t)(tm * 16 + r) * K + k0 + 8 * g + i];
      const float b = B[(size_t)(k0 + 8 * g + i) * N + tn * 16 + r];
      short h, m, l;
      split3(a, h, m, l);
      ah[i] = h; am[i] = m; al[i] = l;
      split3(b, h, m, l);
      bh[i] = h; bm[i] = m; bl[i] = l;
    }
    auto mf = [&](ushortx8 x, ushortx8 y) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x), __builtin_bit_cast(bf16x8, y),
                                                    acc, 0, 0, 0);
    };
    if (V == 3) {
      ushortx8 alo, blo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        alo[i] = bf16_rne(bf16_f(am[i]) + bf16_f(al[i]));
        blo[i] = bf16_rne(bf16_f(bm[i]) + bf16_f(bl[i]));
      }
      mf(ah, blo);
      mf(alo, bh);
      mf(ah, bh);
    } else {
      mf(ah, bl);
      mf(al, bh);
      mf(am, bm);
      mf(ah, bm);
      mf(am, bh);
      mf(ah, bh);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) C[(size_t)(tm * 16 + 4 * g + i) * N + tn * 16 + r] = acc[i];
}

// a 64x64 wave tile's inner step as the GEMM runs it: 4 A + 4 B fragments of
// one 32-deep K step read from LDS as fp32, then 16 output fragments.
//   V = 0: 8 x v_mfma_f32_16x16x4_f32 per output fragment (exact-f32 path)
//   V = 3 / 4: split the 8 fragments once, then 3 / 6 x 16x16x32 bf16 each
template <int V>
__global__ __launch_bounds__(256) void inner_loop(float* out, int iters) {
  __shared__ float lds[8][64][8];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 8 * 64 * 8; i += 256) (&lds[0][0][0])[i] = (float)(i % 97) * 1e-3f - 0.04f;
  __syncthreads();
  floatx4 acc[4][4] = {};
  for (int it = 0; it < iters; ++it) {
    float f[8][8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int t = 0; t < 8; ++t) f[q][t] = lds[q][lane][(t + it) & 7];
    if (V == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 8; ++s)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f[i][s], f[4 + j][s], acc[i][j], 0, 0, 0);
    } else {
      ushortx8 h[8], m[8], l[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          short a, b, c;
          split3(f[q][t], a, b, c);
          h[q][t] = a; m[q][t] = b; l[q][t] = c;
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          auto mf = [&](ushortx8 x, ushortx8 y) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x),
                                                                __builtin_bit_cast(bf16x8, y), acc[i][j], 0, 0, 0);
          };
          if (V == 3) {
            mf(h[i], m[4 + j]);
            mf(m[i], h[4 + j]);
            mf(h[i], h[4 + j]);
          } else {
            mf(h[i], l[4 + j]);
            mf(l[i], h[4 + j]);
            mf(m[i], m[4 + j]);
            mf(h[i], m[4 + j]);
            mf(m[i], h[4 + j]);
            mf(h[i], h[4 + j]);
          }
        }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA issue cost: the same instruction mix with operands in registers
template <int V>
__global__ void mfma_loop(float* out, int iters) {
  floatx4 acc[4] = {};
  const float x = (float)threadIdx.x * 1e-3f;
  shortx4 a = {(short)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (short)threadIdx.x};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (V == 0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, acc[j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < (V == 1 ? 3 : 6); ++s)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, acc[j], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int M = 256, N = 256, K = 2048;
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> A((size_t)M * K), B((size_t)K * N);
  // activation-like (post-LeakyReLU, mixed scale) and weight-like operands
  for (auto& v : A) { float t = nd(rng); v = t > 0 ? t : 0.2f * t; }
  for (auto& v : B) v = 0.03f * nd(rng);
  std::vector<double> ref((size_t)M * N), mag((size_t)M * N);
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      double s = 0, a = 0;
      for (int k = 0; k < K; ++k) {
        const double p = (double)A[(size_t)i * K + k] * B[(size_t)k * N + j];
        s += p;
        a += fabs(p);
      }
      ref[(size_t)i * N + j] = s;
      mag[(size_t)i * N + j] = a;
    }
  float *dA, *dB, *dC, *dO;
  CK(hipMalloc(&dA, A.size() * 4));
  CK(hipMalloc(&dB, B.size() * 4));
  CK(hipMalloc(&dC, (size_t)M * N * 4));
  CK(hipMalloc(&dO, 1024 * 256 * 4));
  CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> C((size_t)M * N);
  const char* names[3] = {"f32 (16x16x4 f32 chain)", "x3 (2-way split, 3 bf16 MFMA)", "x6 (3-way split, 6 bf16 MFMA)"};
  std::vector<float> c0;
  for (int v = 0; v < 3; ++v) {
    const int tiles = (M / 16) * (N / 16);
    if (v == 0) gemm_probe<0><<<tiles, 64>>>(dA, dB, dC, M, N, K);
    if (v == 1) gemm_probe<1><<<tiles, 64>>>(dA, dB, dC, M, N, K);
    if (v == 2) gemm_probe<2><<<tiles, 64>>>(dA, dB, dC, M, N, K);
    CK(hipGetLastError());
    CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
    if (v == 0) c0 = C;
    double mx = 0, rms = 0, mx_vs_f32 = 0;
    for (size_t i = 0; i < C.size(); ++i) {
      const double e = fabs((double)C[i] - ref[i]) / mag[i];
      mx = e > mx ? e : mx;
      rms += e * e;
      const double d = fabs((double)C[i] - (double)c0[i]) / mag[i];
      mx_vs_f32 = d > mx_vs_f32 ? d : mx_vs_f32;
    }
    rms = sqrt(rms / C.size());
    // MFMA-only timing: 1024 blocks x 4 waves, 4 accumulators per wave
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 2000;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (v == 0) mfma_loop<0><<<1024, 256>>>(dO, iters);
      if (v == 1) mfma_loop<1><<<1024, 256>>>(dO, iters);
      if (v == 2) mfma_loop<2><<<1024, 256>>>(dO, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // fp32-equivalent flops of the loop: 1024 blocks * 4 waves * iters * 4 acc * (16x16x16 MACs * 2)
    const double fl = 1024.0 * 4 * iters * 4 * (16 * 16 * 16 * 2.0);
    printf("%-32s max err %.3e  rms err %.3e  (rel. to sum|ab|; max |diff vs f32 path| %.3e)  "
           "MFMA loop %.2f ms = %.1f fp32-equivalent TFLOP/s\n",
           names[v], mx, rms, mx_vs_f32, ms, fl / (ms * 1e-3) / 1e12);
  }
  const char* n32[2] = {"x3 via 16x16x32", "x6 via 16x16x32"};
  for (int v = 0; v < 2; ++v) {
    const int tiles = (M / 16) * (N / 16);
    if (v == 0) gemm_probe32<3><<<tiles, 64>>>(dA, dB, dC, M, N, K);
    else gemm_probe32<4><<<tiles, 64>>>(dA, dB, dC, M, N, K);
    CK(hipGetLastError());
    CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, rms = 0;
    for (size_t i = 0; i < C.size(); ++i) {
      const double e = fabs((double)C[i] - ref[i]) / mag[i];
      mx = e > mx ? e : mx;
      rms += e * e;
    }
    printf("%-32s max err %.3e  rms err %.3e\n", n32[v], mx, sqrt(rms / C.size()));
  }
  // inner-loop timing: 1024 blocks x 4 waves, 64x64 wave tile, 32-deep K steps
  const char* nl[3] = {"inner f32 (8 x 16x16x4 / frag)", "inner x3 (split + 3 x 16x16x32)", "inner x6 (split + 6 x 16x16x32)"};
  for (int v = 0; v < 3; ++v) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 400;
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (v == 0) inner_loop<0><<<1024, 256>>>(dO, iters);
      if (v == 1) inner_loop<3><<<1024, 256>>>(dO, iters);
      if (v == 2) inner_loop<4><<<1024, 256>>>(dO, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double fl = 1024.0 * 4 * iters * 16 * (16 * 16 * 32 * 2.0);
    printf("%-34s %.2f ms = %.1f fp32-equivalent TFLOP/s\n", nl[v], ms, fl / (ms * 1e-3) / 1e12);
  }
  return 0;
}
