// Column-slab kernels around the MFMA GEMMs: BatchNorm1d train/eval,
// BN+activation backward, bias/loss reductions, input packing, Adam, and the
// variational-information-bottleneck reparameterisation.  All HBM-bound:
// 16-byte accesses per lane, one 64-column x 128-row slab per 256-thread
// block (grid = Np/64 x Mp/128, thousands of blocks at the bench shapes).
#include "mmad_common.h"
#include "mmad_ops.h"
#include "mmad_gemm.h"

#include <hip/hip_ext.h>

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <system_error>
#include <type_traits>

#define SLAB_COLS 64
#define SLAB_ROWS 128

namespace {

template <typename T> struct Vec { static constexpr int N = 16 / sizeof(T); };

// ---------------------------------------------------------------------------
// BN eval affine: scale = gamma/sqrt(rv+eps), shift = beta - rm*scale
__global__ void bn_eval_affine_k(int N, int Np, const float* gamma, const float* beta,
                                 const float* rm, const float* rv, float eps, float* scale,
                                 float* shift) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Np) return;
  if (j < N) {
    float s = gamma[j] * (float)(1.0 / sqrt((double)rv[j] + (double)eps));
    scale[j] = s;
    shift[j] = beta[j] - rm[j] * s;
  } else {
    scale[j] = 0.f;
    shift[j] = 0.f;
  }
}

// Merge the GEMM-epilogue Welford partials of 64 columns -> (mean, var) in LDS
// (the merge in fp64, as torch's CPU BatchNorm accumulates its statistics).
__device__ void merge_welford(int M, int nparts, const float* stats, int Np, int n0, float* s_mean,
                              float* s_var) {
  __shared__ double pm[4][SLAB_COLS], pq[4][SLAB_COLS], pn[4][SLAB_COLS];
  const int tid = threadIdx.x, c = tid & 63, grp = tid >> 6;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int i = grp; i < nparts; i += 4) {
    int cnt = M - i * MMAD_PART_ROWS;
    cnt = cnt < 0 ? 0 : (cnt > MMAD_PART_ROWS ? MMAD_PART_ROWS : cnt);
    if (cnt == 0) continue;
    const double mb = stats[(size_t)i * 2 * Np + n0 + c];
    const double qb = stats[((size_t)i * 2 + 1) * Np + n0 + c];
    const double nb = (double)cnt;
    const double nn = n + nb;
    const double d = mb - mean;
    mean += d * (nb / nn);
    m2 += qb + d * d * (n * nb / nn);
    n = nn;
  }
  pm[grp][c] = mean;
  pq[grp][c] = m2;
  pn[grp][c] = n;
  __syncthreads();
  if (tid < SLAB_COLS) {
    double n1 = 0.0, mu = 0.0, q = 0.0;
    for (int g = 0; g < 4; ++g) {
      const double nb = pn[g][tid];
      if (nb == 0.0) continue;
      const double nn = n1 + nb;
      const double d = pm[g][tid] - mu;
      mu += d * (nb / nn);
      q += pq[g][tid] + d * d * (n1 * nb / nn);
      n1 = nn;
    }
    s_mean[tid] = (float)mu;
    s_var[tid] = n1 > 0.0 ? (float)(q / n1) : 0.f;  // biased variance (normalisation)
  }
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(256) void bn_train_apply_k(int M, int N, int Np, const T* __restrict__ a,
                                                        const float* __restrict__ stats, int nparts,
                                                        const float* gamma, const float* beta,
                                                        float* rmean, float* rvar, float momentum,
                                                        float eps, float* save_mean,
                                                        float* save_rstd, T* __restrict__ y) {
  __shared__ float s_mean[SLAB_COLS], s_var[SLAB_COLS], s_sc[SLAB_COLS], s_sh[SLAB_COLS];
  const int n0 = blockIdx.x * SLAB_COLS, r0 = blockIdx.y * SLAB_ROWS, tid = threadIdx.x;
  merge_welford(M, nparts, stats, Np, n0, s_mean, s_var);
  if (tid < SLAB_COLS) {
    const int col = n0 + tid;
    float sc = 0.f, sh = 0.f;
    if (col < N) {
      const float rstd = (float)(1.0 / sqrt((double)s_var[tid] + (double)eps));
      sc = gamma[col] * rstd;
      sh = beta[col] - s_mean[tid] * sc;
      if (blockIdx.y == 0) {
        save_mean[col] = s_mean[tid];
        save_rstd[col] = rstd;
        const float unb = M > 1 ? s_var[tid] * (float)M / (float)(M - 1) : s_var[tid];
        rmean[col] = (1.f - momentum) * rmean[col] + momentum * s_mean[tid];
        rvar[col] = (1.f - momentum) * rvar[col] + momentum * unb;
      }
    } else if (blockIdx.y == 0) {
      save_mean[col] = 0.f;
      save_rstd[col] = 0.f;
    }
    s_sc[tid] = sc;
    s_sh[tid] = sh;
  }
  __syncthreads();
  constexpr int V = Vec<T>::N;
  constexpr int CPR = SLAB_COLS / V;
  for (int idx = tid; idx < SLAB_ROWS * CPR; idx += 256) {
    const int rl = idx / CPR, ch = idx % CPR;
    const int row = r0 + rl;
    const size_t off = (size_t)row * Np + n0 + ch * V;
    uint4v raw = *(const uint4v*)(a + off);
    T* e = (T*)&raw;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float v = to_f32<T>(e[k]) * s_sc[ch * V + k] + s_sh[ch * V + k];
      e[k] = from_f32<T>(row < M ? v : 0.f);
    }
    *(uint4v*)(y + off) = raw;
  }
}

// Train-mode BN finalize only: batch mean/rstd, per-column affine for the
// consumers' normalise-on-load, running-stat update.  One thread per column:
// every chunk partial is loaded up front (one memory round trip), then merged
// sequentially in chunk order (Chan et al. pairwise Welford update).
__global__ __launch_bounds__(64) void bn_finalize_k(int M, int N, int Np, const float* __restrict__ stats,
                                                    int nparts, const float* gamma, const float* beta,
                                                    float* rmean, float* rvar, float momentum,
                                                    float eps, float* save_mean, float* save_rstd,
                                                    float* scale, float* shift) {
  constexpr int U = 16;
  const int col = blockIdx.x * 64 + threadIdx.x;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int i0 = 0; i0 < nparts; i0 += U) {
    float mb[U], qb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u < nparts ? i0 + u : nparts - 1;
      mb[u] = stats[(size_t)i * 2 * Np + col];
      qb[u] = stats[((size_t)i * 2 + 1) * Np + col];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u;
      int cnt = M - i * MMAD_PART_ROWS;
      cnt = cnt < 0 ? 0 : (cnt > MMAD_PART_ROWS ? MMAD_PART_ROWS : cnt);
      if (i >= nparts || cnt == 0) continue;
      const double nb = (double)cnt, nn = n + nb, d = (double)mb[u] - mean;
      mean += d * (nb / nn);
      m2 += (double)qb[u] + d * d * (n * nb / nn);
      n = nn;
    }
  }
  const float var = n > 0.0 ? (float)(m2 / n) : 0.f;
  if (col < N) {
    const float rstd = (float)(1.0 / sqrt((double)var + (double)eps));
    const float sc = gamma[col] * rstd;
    save_mean[col] = mean;
    save_rstd[col] = rstd;
    scale[col] = sc;
    shift[col] = beta[col] - mean * sc;
    const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    rmean[col] = (1.f - momentum) * rmean[col] + momentum * mean;
    rvar[col] = (1.f - momentum) * rvar[col] + momentum * unb;
  } else {
    save_mean[col] = 0.f;
    save_rstd[col] = 0.f;
    scale[col] = 0.f;
    shift[col] = 0.f;
  }
}

// Finalize + fold.  Block (kb, nb): the 64 producer columns k0..k0+63 (its
// statistics merge is recomputed per n-block: 16 KB of L2 reads) and the
// 64 * FOLD_RPT consumer rows n0.. of W.  Merge order: 4 chunk groups
// (g, g+4, ...) each sequential, then ((g0 + g1) + g2) + g3.
template <typename TW, int FOLD_RPT>
__global__ __launch_bounds__(256) void bn_fold_k(int M, int N, int Np, const float* __restrict__ stats,
                                                 int nparts, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, float* rmean,
                                                 float* rvar, float momentum, float eps,
                                                 float* save_mean, float* save_rstd, float* scale,
                                                 float* shift, const float* __restrict__ W,
                                                 TW* __restrict__ wout, float* __restrict__ cpart,
                                                 int cp_stride) {
  // all of a group's partials in flight at once (128 partial rows = 4096
  // windows in one round trip; the merge order below is unchanged)
  constexpr int U = 32;
  __shared__ double pm[4][64], pq[4][64], pn[4][64];
  __shared__ float s_sc[64], s_sh[64];
  const int k0 = blockIdx.x * 64, n0 = blockIdx.y * 64 * FOLD_RPT, tid = threadIdx.x;
  // W tile loads first (independent of the statistics): rows r + 64 i, 16 columns
  const int r = tid >> 2, cq = (tid & 3) * 16;
  floatx4 wv[FOLD_RPT][4];
#pragma unroll
  for (int i = 0; i < FOLD_RPT; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      wv[i][u] = *(const floatx4*)(W + (size_t)(n0 + r + 64 * i) * Np + k0 + cq + 4 * u);
  {
    // shifted sums about chunk 0's mean K (no division in the chain: the
    // pairwise Welford update it replaced held a dependent fp64 division per
    // chunk, ~4.6 us of a 4096-row fold, tools/fold_probe.py):
    //   S1 = sum n_i (mean_i - K),  S2 = sum [M2_i + n_i (mean_i - K)^2],
    //   mean = K + S1 / n,  M2 = S2 - S1^2 / n
    // (K is within ~std/sqrt(32) of the batch mean, so S1^2 / n stays a few
    // per cent of S2: no cancellation to speak of in fp64)
    const int c = tid & 63, grp = tid >> 6;
    const double K = stats[k0 + c];
    double n = 0.0, s1 = 0.0, s2 = 0.0;
    for (int i0 = grp; i0 < nparts; i0 += 4 * U) {
      float mb[U], qb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + 4 * u, nparts - 1);
        mb[u] = stats[(size_t)i * 2 * Np + k0 + c];
        qb[u] = stats[((size_t)i * 2 + 1) * Np + k0 + c];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + 4 * u;
        int cnt = M - i * MMAD_PART_ROWS;
        cnt = cnt < 0 ? 0 : (cnt > MMAD_PART_ROWS ? MMAD_PART_ROWS : cnt);
        if (i >= nparts || cnt == 0) continue;
        const double nb = (double)cnt, d = (double)mb[u] - K;
        n += nb;
        s1 = fma(nb, d, s1);
        s2 += fma(nb * d, d, (double)qb[u]);
      }
    }
    pm[grp][c] = s1;
    pq[grp][c] = s2;
    pn[grp][c] = n;
  }
  __syncthreads();
  if (tid < 64) {
    const double n1 = ((pn[0][tid] + pn[1][tid]) + pn[2][tid]) + pn[3][tid];
    const double t1 = ((pm[0][tid] + pm[1][tid]) + pm[2][tid]) + pm[3][tid];
    const double t2 = ((pq[0][tid] + pq[1][tid]) + pq[2][tid]) + pq[3][tid];
    const double K = stats[k0 + tid];
    const double mud = n1 > 0.0 ? K + t1 / n1 : 0.0;
    const double q = n1 > 0.0 ? fmax(t2 - t1 * (t1 / n1), 0.0) : 0.0;
    const float mu = (float)mud;
    const float var = n1 > 0.0 ? (float)(q / n1) : 0.f;
    const int col = k0 + tid;
    float sc = 0.f, sh = 0.f;
    if (col < N) {
      const float rstd = (float)(1.0 / sqrt((double)var + (double)eps));
      sc = gamma[col] * rstd;
      sh = beta[col] - mu * sc;
      if (blockIdx.y == 0) {
        save_mean[col] = mu;
        save_rstd[col] = rstd;
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        rmean[col] = (1.f - momentum) * rmean[col] + momentum * mu;
        rvar[col] = (1.f - momentum) * rvar[col] + momentum * unb;
      }
    } else if (blockIdx.y == 0) {
      save_mean[col] = 0.f;
      save_rstd[col] = 0.f;
    }
    if (blockIdx.y == 0) {
      scale[col] = sc;
      shift[col] = sh;
    }
    s_sc[tid] = sc;
    s_sh[tid] = sh;
  }
  __syncthreads();
  // W' = W * scale (row r, 16 columns), c = sum shift * W (sequential, then
  // the 4 quarter-row lanes combined ((q0 + q1) + (q2 + q3)))
#pragma unroll
  for (int i = 0; i < FOLD_RPT; ++i) {
    const int row = n0 + r + 64 * i;
    float cs = 0.f;
    TW o[16];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kl = cq + 4 * u + e;
        o[4 * u + e] = from_f32<TW>(wv[i][u][e] * s_sc[kl]);
        cs += s_sh[kl] * wv[i][u][e];
      }
    TW* dst = wout + (size_t)row * Np + k0 + cq;
#pragma unroll
    for (int v = 0; v < 16 * (int)sizeof(TW) / 16; ++v)
      *((uint4v*)dst + v) = *((const uint4v*)o + v);
    cs += __shfl_xor(cs, 1);
    cs += __shfl_xor(cs, 2);
    if ((tid & 3) == 0) cpart[(size_t)blockIdx.x * cp_stride + row] = cs;
  }
}

// ---------------------------------------------------------------------------
// BN(train) + activation backward.  Pass 1: per-slab partial sums of dy and
// dy*xhat.  Pass 2: finalise dgamma/dbeta, dz, and db partials.
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_k(int M, int Np, const T* __restrict__ dy,
                                                       const T* __restrict__ a,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       double* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  constexpr int CPR = SLAB_COLS / V;
  constexpr int RG = 256 / CPR;  // row groups
  __shared__ double s1[RG][SLAB_COLS], s2[RG][SLAB_COLS];
  const int n0 = blockIdx.x * SLAB_COLS, r0 = blockIdx.y * SLAB_ROWS, tid = threadIdx.x;
  const int ch = tid % CPR, rg = tid / CPR;
  double acc1[V], acc2[V], mu[V], rs[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    acc1[k] = 0.0;
    acc2[k] = 0.0;
    mu[k] = mean[n0 + ch * V + k];
    rs[k] = rstd[n0 + ch * V + k];
  }
  for (int rl = rg; rl < SLAB_ROWS; rl += RG) {
    const int row = r0 + rl;
    if (row >= M) break;
    const size_t off = (size_t)row * Np + n0 + ch * V;
    uint4v rd = *(const uint4v*)(dy + off);
    uint4v ra = *(const uint4v*)(a + off);
    const T* pd = (const T*)&rd;
    const T* pa = (const T*)&ra;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const double d = to_f32<T>(pd[k]);
      acc1[k] += d;
      acc2[k] += d * (((double)to_f32<T>(pa[k]) - mu[k]) * rs[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    s1[rg][ch * V + k] = acc1[k];
    s2[rg][ch * V + k] = acc2[k];
  }
  __syncthreads();
  if (tid < SLAB_COLS) {
    double t1 = 0.0, t2 = 0.0;
    for (int g = 0; g < RG; ++g) { t1 += s1[g][tid]; t2 += s2[g][tid]; }
    part[((size_t)blockIdx.y * 2) * Np + n0 + tid] = t1;
    part[((size_t)blockIdx.y * 2 + 1) * Np + n0 + tid] = t2;
  }
}

// dz = act'(a) * gamma*rstd/M * (M*dy - sum(dy) - xhat*sum(dy*xhat)) over RB
// 64-column x 128-row slabs; sums from the bwd-data GEMM epilogue partials,
// merged once per block.  The first slab's loads (dy, a, the column
// constants, the partials) are issued before any use, so the block's first
// slab costs one memory round trip; each later slab's dy / a are loaded
// under the previous slab's arithmetic.  Per slab the same arithmetic and
// the same db-partial order as RB = 1 (bit-identical for every RB).  LK: the
// activation is LeakyReLU (the AE's), known at compile time -- with a run-time
// act the per-element switch stays inside the unrolled loop, 32 branch chains
// per row group and slab
template <typename T, int PU, int RB, bool LK>
__global__ __launch_bounds__(256) void bn_bwd_apply_k(int act_rt, float slope, int M, int N, int Np,
                                                      int nparts, const T* __restrict__ dy,
                                                      const T* __restrict__ a,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      const float* __restrict__ gamma,
                                                      const double* __restrict__ part,
                                                      T* __restrict__ dz, float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta, float* __restrict__ dbpart) {
  constexpr int V = Vec<T>::N;
  constexpr int CPR = SLAB_COLS / V;      // threads per row
  constexpr int RG = 256 / CPR;           // row groups
  constexpr int RPT = SLAB_ROWS / RG;     // rows per thread and slab
  const int act = LK ? (int)MMAD_ACT_LEAKYRELU : act_rt;
  // PU: partial chunks per group loaded at once (16 from 2048 rows: one round
  // trip for all of a 4096-row batch's 64 chunks; same summation order)
  __shared__ double s_red[RG][SLAB_COLS];
  __shared__ double s_p1[4][SLAB_COLS], s_p2[4][SLAB_COLS];
  const int n0 = blockIdx.x * SLAB_COLS, tid = threadIdx.x;
  const int ch = tid % CPR, rg = tid / CPR;
  // (1) this thread's dy / a rows of the first slab
  uint4v rd[RPT], ra[RPT];
  auto load_slab = [&](int slab) {
    const int r0 = slab * SLAB_ROWS;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const size_t off = (size_t)(r0 + rg + i * RG) * Np + n0 + ch * V;
      rd[i] = *(const uint4v*)(dy + off);
      ra[i] = *(const uint4v*)(a + off);
    }
  };
  load_slab(blockIdx.y * RB);
  // (2) partial sums: 4 groups of 64 columns, group g sums chunks g, g+4, ...
  {
    const int c = tid & 63, grp = tid >> 6;
    double t1 = 0.0, t2 = 0.0;
    for (int i0 = grp; i0 < nparts; i0 += 4 * PU) {
      double p1[PU], p2[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int i = i0 + 4 * u < nparts ? i0 + 4 * u : grp;
        p1[u] = part[((size_t)i * 2) * Np + n0 + c];
        p2[u] = part[((size_t)i * 2 + 1) * Np + n0 + c];
      }
#pragma unroll
      for (int u = 0; u < PU; ++u)
        if (i0 + 4 * u < nparts) { t1 += p1[u]; t2 += p2[u]; }
    }
    s_p1[grp][c] = t1;
    s_p2[grp][c] = t2;
  }
  __syncthreads();
  if (tid < SLAB_COLS) {
    double t1 = ((s_p1[0][tid] + s_p1[1][tid]) + s_p1[2][tid]) + s_p1[3][tid];
    double t2 = ((s_p2[0][tid] + s_p2[1][tid]) + s_p2[2][tid]) + s_p2[3][tid];
    const int col = n0 + tid;
    if (col >= N) { t1 = 0.0; t2 = 0.0; }
    s_p1[0][tid] = t1;
    s_p2[0][tid] = t2;
    if (blockIdx.y == 0) { dbeta[col] = (float)t1; dgamma[col] = (float)t2; }
  }
  __syncthreads();
  // (3) column constants (loaded after the partials: their registers are free by then)
  float mu[V], rs[V], gm[V];
#pragma unroll
  for (int k = 0; k < V; k += 4) {
    const int col = n0 + ch * V + k;
    *(floatx4*)&mu[k] = *(const floatx4*)(mean + col);
    *(floatx4*)&rs[k] = *(const floatx4*)(rstd + col);
    *(floatx4*)&gm[k] = *(const floatx4*)(gamma + col);
  }
  // da = gamma rstd / M (M dy - sum dy - xhat sum dy xhat): the bracket nearly
  // cancels, so on the exact-fp32 path it is evaluated in fp64 (as the
  // reference's CPU BatchNorm backward does its reductions), dz and its column
  // sums too.  The bf16 path (this kernel runs there from 2048 rows, c3 / c4)
  // rounds dz to 8 bits: its bracket in fp32 (M * dy exact, M a power of two
  // at the bench shapes; the column sums rounded once), which halves the
  // kernel's registers and doubles its waves per SIMD -- a 4096-row apply ran
  // at 2.2-2.5 TB/s with the fp64 bracket (tools/apply_probe.py)
  using CT = std::conditional_t<sizeof(T) == 2, float, double>;
  const CT invM = (CT)1 / (CT)M;
  CT cf[V], dbv[V], dgv[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int col = n0 + ch * V + k;
    cf[k] = col < N ? (CT)gm[k] * (CT)rs[k] * invM : (CT)0;
    dbv[k] = (CT)s_p1[0][ch * V + k];
    dgv[k] = (CT)s_p2[0][ch * V + k];
  }
  for (int sb = 0; sb < RB; ++sb) {
    const int slab = blockIdx.y * RB + sb;
    const int r0 = slab * SLAB_ROWS;
    CT accb[V];
#pragma unroll
    for (int k = 0; k < V; ++k) accb[k] = (CT)0;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int row = r0 + rg + i * RG;
      const T* pd = (const T*)&rd[i];
      const T* pa = (const T*)&ra[i];
      T* po = (T*)&rd[i];      // dz over dy in place: element k is read before it is written
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float av = to_f32<T>(pa[k]);
        const CT xh = ((CT)av - (CT)mu[k]) * (CT)rs[k];
        const CT da = cf[k] * ((CT)M * (CT)to_f32<T>(pd[k]) - dbv[k] - xh * dgv[k]);
        float d = (float)(da * (CT)act_grad_from_out(av, act, slope));
        d = row < M ? d : 0.f;
        const T dt = from_f32<T>(d);
        po[k] = dt;
        accb[k] += (CT)to_f32<T>(dt);
      }
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i)
      *(uint4v*)(dz + (size_t)(r0 + rg + i * RG) * Np + n0 + ch * V) = rd[i];
    // the next slab's rows load under this slab's reduction
    if (sb + 1 < RB) load_slab(slab + 1);
#pragma unroll
    for (int k = 0; k < V; ++k) s_red[rg][ch * V + k] = accb[k];
    __syncthreads();
    if (tid < SLAB_COLS) {
      double t = 0.0;
      for (int g = 0; g < RG; ++g) t += s_red[g][tid];
      dbpart[(size_t)slab * Np + n0 + tid] = (float)t;
    }
    if (sb + 1 < RB) __syncthreads();   // s_red reused by the next slab
  }
}

// Activation backward without BatchNorm (an FCLayer with bn=False):
// dz = dy * act'(a) from the activation OUTPUT a, plus the per-slab column
// sums of dz (the bias gradient) -> db partials [Mp/128][Np]
template <typename T>
__global__ __launch_bounds__(256) void act_bwd_k(int act, float slope, int M, int Np,
                                                 const T* __restrict__ dy, const T* __restrict__ a,
                                                 T* __restrict__ dz, float* __restrict__ dbpart) {
  constexpr int V = Vec<T>::N;
  constexpr int CPR = SLAB_COLS / V;
  constexpr int RG = 256 / CPR;
  __shared__ double s_red[RG][SLAB_COLS];
  const int n0 = blockIdx.x * SLAB_COLS, r0 = blockIdx.y * SLAB_ROWS, tid = threadIdx.x;
  const int ch = tid % CPR, rg = tid / CPR;
  double acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.0;
  for (int rl = rg; rl < SLAB_ROWS; rl += RG) {
    const int row = r0 + rl;
    const size_t off = (size_t)row * Np + n0 + ch * V;
    const uint4v rd = *(const uint4v*)(dy + off);
    const uint4v ra = *(const uint4v*)(a + off);
    const T* pd = (const T*)&rd;
    const T* pa = (const T*)&ra;
    uint4v ro;
    T* po = (T*)&ro;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float d = to_f32<T>(pd[k]) * act_grad_from_out(to_f32<T>(pa[k]), act, slope);
      d = row < M ? d : 0.f;
      po[k] = from_f32<T>(d);
      acc[k] += (double)to_f32<T>(po[k]);
    }
    *(uint4v*)(dz + off) = ro;
  }
#pragma unroll
  for (int k = 0; k < V; ++k) s_red[rg][ch * V + k] = acc[k];
  __syncthreads();
  if (tid < SLAB_COLS) {
    double t = 0.0;
    for (int g = 0; g < RG; ++g) t += s_red[g][tid];
    dbpart[(size_t)blockIdx.y * Np + n0 + tid] = (float)t;
  }
}

// column sums of a packed matrix -> partials [Mp/128][Np]
template <typename T>
__global__ __launch_bounds__(256) void matrix_colsum_k(int M, int Np, const T* __restrict__ x,
                                                       float* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  constexpr int CPR = SLAB_COLS / V;
  constexpr int RG = 256 / CPR;
  __shared__ float s_red[RG][SLAB_COLS];
  const int n0 = blockIdx.x * SLAB_COLS, r0 = blockIdx.y * SLAB_ROWS, tid = threadIdx.x;
  const int ch = tid % CPR, rg = tid / CPR;
  float acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.f;
  for (int rl = rg; rl < SLAB_ROWS; rl += RG) {
    const int row = r0 + rl;
    if (row >= M) break;
    uint4v r = *(const uint4v*)(x + (size_t)row * Np + n0 + ch * V);
    const T* p = (const T*)&r;
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] += to_f32<T>(p[k]);
  }
#pragma unroll
  for (int k = 0; k < V; ++k) s_red[rg][ch * V + k] = acc[k];
  __syncthreads();
  if (tid < SLAB_COLS) {
    float t = 0.f;
    for (int g = 0; g < RG; ++g) t += s_red[g][tid];
    part[(size_t)blockIdx.y * Np + n0 + tid] = t;
  }
}

__global__ void colsum_k(int n_parts, int N, int Np, const float* __restrict__ part,
                         int stride, float scale, float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Np) return;
  float t = 0.f;
  if (j < N)
    for (int i = 0; i < n_parts; ++i) t += part[(size_t)i * stride + j];
  out[j] = scale * t;
}

__global__ __launch_bounds__(1024) void sum2d_k(int rows, int cols, const float* __restrict__ x,
                                                int64_t ld, float scale, float* out, int accumulate) {
  __shared__ float red[16];
  float t = 0.f;
  const int64_t n = (int64_t)rows * cols;
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const int64_t r = i / cols, c = i % cols;
    t += x[r * ld + c];
  }
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += red[i];
    out[0] = (accumulate ? out[0] : 0.f) + scale * s;
  }
}

// PU output chunks per thread (chunk u of the block at blockIdx*256*PU +
// u*256 + tid): every chunk's loads are issued before the first conversion,
// PU x V/4 16-B loads in flight per thread
template <typename T, int PU>
__global__ void pack_input_k(int M, int K, int Mp, int Kp, const float* __restrict__ x, int ldx,
                             int vec, T* __restrict__ out, const MmadDyn* __restrict__ dyn) {
  constexpr int V = Vec<T>::N;
  if (dyn) x = dyn->x;
  const int cpr = Kp / V;
  const int64_t total = (int64_t)Mp * cpr;
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * PU + threadIdx.x;
  floatx4 f[PU][V / 4];
  bool full[PU];
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int64_t idx = base + (int64_t)u * blockDim.x;
    const int row = (int)(idx / cpr), c0 = (int)(idx % cpr) * V;
    full[u] = vec && idx < total && row < M && c0 + V <= K;
    if (full[u]) {
      // 16-B aligned rows (checked by the launcher): V/4 dwordx4 loads
      const float* src = x + (size_t)row * ldx + c0;
#pragma unroll
      for (int q = 0; q < V / 4; ++q) f[u][q] = *(const floatx4*)(src + 4 * q);
    }
  }
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int64_t idx = base + (int64_t)u * blockDim.x;
    if (idx >= total) continue;
    const int row = (int)(idx / cpr), c0 = (int)(idx % cpr) * V;
    uint4v r;
    T* p = (T*)&r;
    if (full[u]) {
#pragma unroll
      for (int k = 0; k < V; ++k) p[k] = from_f32<T>(f[u][k / 4][k % 4]);
    } else {
      const float* src = x + (size_t)row * ldx + c0;
#pragma unroll
      for (int k = 0; k < V; ++k) p[k] = from_f32<T>((row < M && c0 + k < K) ? src[k] : 0.f);
    }
    *(uint4v*)(out + (size_t)row * Kp + c0) = r;
  }
}

template <typename T>
__global__ void unpack_k(int M, int N, int Np, const T* __restrict__ y, float* __restrict__ out,
                         int ldo) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)M * N) return;
  const int row = (int)(idx / N), col = (int)(idx % N);
  out[(size_t)row * ldo + col] = to_f32<T>(y[(size_t)row * Np + col]);
}

template <typename T>
__global__ void sse_k(int M, int N, int Np, const T* __restrict__ y, const float* __restrict__ x,
                      int ldx, float* __restrict__ part) {
  __shared__ float red[4];
  float t = 0.f;
  const int64_t n = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int row = (int)(i / N), col = (int)(i % N);
    const float d = to_f32<T>(y[(size_t)row * Np + col]) - x[(size_t)row * ldx + col];
    t += d * d;
  }
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam, single-tensor formula) over a flat buffer
__global__ __launch_bounds__(256) void adam_k(int64_t n, float* __restrict__ p,
                                              const float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, float w1, float w2, float eps,
                                              float step_size, float bc2_sqrt, bf16* shadow,
                                              int64_t n_shadow, const MmadDyn* dyn) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (dyn) {   // graph-captured step: this step's bias-correction terms
    step_size = dyn->ad_step;
    bc2_sqrt = dyn->ad_bc2;
  }
  if (i4 + 4 <= n) {
    floatx4 pp = *(floatx4*)(p + i4), gg = *(const floatx4*)(g + i4);
    floatx4 mm = *(floatx4*)(m + i4), vv = *(floatx4*)(v + i4);
    adam4(pp, mm, vv, gg, w1, w2, eps, step_size, bc2_sqrt);
    *(floatx4*)(p + i4) = pp;
    *(floatx4*)(m + i4) = mm;
    *(floatx4*)(v + i4) = vv;
    if (shadow && i4 + 4 <= n_shadow) {
      bf16x4 s;
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] = (bf16)pp[k];
      *(bf16x4*)(shadow + i4) = s;
    } else if (shadow) {   // a shadow shorter than the buffer, ending inside this quad
      for (int k = 0; k < 4 && i4 + k < n_shadow; ++k) shadow[i4 + k] = (bf16)pp[k];
    }
  } else {
    for (int64_t i = i4; i < n; ++i) {
      float pp = p[i], mm = m[i], vv = v[i];
      adam_elem(pp, mm, vv, g[i], w1, w2, eps, step_size, bc2_sqrt);
      p[i] = pp;
      m[i] = mm;
      v[i] = vv;
      if (shadow && i < n_shadow) shadow[i] = (bf16)pp;
    }
  }
}

__global__ void to_bf16_k(int64_t n, const float* __restrict__ x, bf16* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (bf16)x[i];
}
__global__ void from_bf16_k(int64_t n, const bf16* __restrict__ x, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (float)x[i];
}

// ---------------------------------------------------------------------------
// One launch for all end-of-backward reductions (bias grads, loss): job j,
// block x covers 256 output columns; scalar jobs run in block x == 0 only.
__global__ __launch_bounds__(256) void reduce_jobs_k(MmadReduceJobs jobs) {
  const MmadReduceJob& jb = jobs.j[blockIdx.y];
  const int tid = threadIdx.x;
  if (jb.scalar) {
    if (blockIdx.x != 0) return;
    __shared__ float red[4];
    float t = 0.f;
    for (int i = 0; i < jb.nparts; ++i)
      for (int c = tid; c < jb.N; c += 256) t += jb.src[(size_t)i * jb.stride + c];
    t *= jb.scale;
    float t2 = 0.f;
    for (int c = tid; c < jb.n2; c += 256) t2 += jb.src2[c];
    t += jb.scale2 * t2;
    t = wave_sum(t);
    if ((tid & 63) == 0) red[tid >> 6] = t;
    __syncthreads();
    if (tid == 0) (jobs.dyn ? jobs.dyn->loss : jb.dst)[0] = red[0] + red[1] + red[2] + red[3];
    return;
  }
  const int j = blockIdx.x * 256 + tid;
  if (j >= jb.Np) return;
  float t = 0.f;
  if (j < jb.N) {
    // sequential partial order (the fused dW epilogue's and the flat Adam's),
    // with 32 partial loads in flight per round trip (the data-parallel step
    // reduces every layer's bias partials here: 128 dependent loads per column
    // at 4096 rows took 70 us on the step's critical tail)
    constexpr int U = 32;
    int i = 0;
    for (; i + U <= jb.nparts; i += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = jb.src[(size_t)(i + u) * jb.stride + j];
#pragma unroll
      for (int u = 0; u < U; ++u) t += v[u];
    }
    for (; i < jb.nparts; ++i) t += jb.src[(size_t)i * jb.stride + j];
  }
  jb.dst[j] = jb.scale * t;
}

// Adam over two flat segments (a layer's weights and its bias/gamma/beta)
__global__ __launch_bounds__(256) void adam2_k(MmadAdamSeg s0, MmadAdamSeg s1, float w1, float w2,
                                               float eps, float step_size, float bc2_sqrt) {
  int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const MmadAdamSeg* sg = &s0;
  if (i4 >= s0.n) { i4 -= s0.n; sg = &s1; }
  if (i4 >= sg->n) return;
  float* p = sg->p + i4;
  float* g = sg->g + i4;
  float* m = sg->m + i4;
  float* v = sg->v + i4;
  floatx4 gg;
  if (sg->bsrc && i4 < sg->bNp) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = (int)i4 + k;
      float t = 0.f;
      if (e < sg->bN)
        for (int i = 0; i < sg->bparts; ++i) t += sg->bsrc[(size_t)i * sg->bstride + e];
      gg[k] = t;
    }
    *(floatx4*)g = gg;
  } else {
    gg = *(const floatx4*)g;
  }
  floatx4 pp = *(floatx4*)p, mm = *(floatx4*)m, vv = *(floatx4*)v;
  adam4(pp, mm, vv, gg, w1, w2, eps, step_size, bc2_sqrt);
  *(floatx4*)p = pp;
  *(floatx4*)m = mm;
  *(floatx4*)v = vv;
  if (sg->shadow) {
    bf16x4 sh;
#pragma unroll
    for (int k = 0; k < 4; ++k) sh[k] = (bf16)pp[k];
    *(bf16x4*)((bf16*)sg->shadow + i4) = sh;
  }
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG -> N(0,1) via Box-Muller
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c[0] = hi1 ^ c[1] ^ k0;
  c[1] = lo1;
  c[2] = hi0 ^ c[3] ^ k1;
  c[3] = lo0;
}
__device__ __forceinline__ float philox_normal(uint64_t seed, uint64_t offset, uint64_t idx) {
  uint32_t c[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)offset, (uint32_t)(offset >> 32)};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const float u1 = ((c[0] >> 8) + 1) * (1.0f / 16777217.0f);  // (0,1]
  const float u2 = (c[1] >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853071795864f * u2);
}

template <typename T>
__global__ __launch_bounds__(256) void vib_fwd_k(int B, int btl, int k, const T* __restrict__ enc,
                                                 int ld_enc, const float* __restrict__ eps,
                                                 float* __restrict__ eps_out, uint64_t seed,
                                                 uint64_t offset, int det, T* __restrict__ z,
                                                 int ld_z, int Mpz, float* kl_part,
                                                 const MmadDyn* __restrict__ dyn) {
  // one thread per element of the packed z buffer [Mpz][ld_z]; rows < B also
  // contribute the KL term of their (mu, logvar) pair.
  __shared__ float red[4];
  if (dyn) {
    eps = dyn->eps;
    seed = dyn->seed;
    offset = dyn->offset;
  }
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)Mpz * ld_z;
  float kl = 0.f;
  if (idx < total) {
    const int row = (int)(idx / ld_z), c = (int)(idx % ld_z);
    float out = 0.f;
    if (c < btl && row < k * B) {
      const int kk = row / B, b = row % B;
      const float mu = to_f32<T>(enc[(size_t)b * ld_enc + c]);
      const float lv = to_f32<T>(enc[(size_t)b * ld_enc + btl + c]);
      if (det) {
        out = mu;
      } else {
        const size_t ei = ((size_t)kk * B + b) * btl + c;
        const float e = eps ? eps[ei] : philox_normal(seed, offset, ei);
        if (eps_out) eps_out[ei] = e;
        out = e * __expf(0.5f * lv) + mu;
      }
      if (kk == 0 && kl_part) kl = -0.5f * (1.f + lv - mu * mu - __expf(lv));
    }
    z[idx] = from_f32<T>(out);
  }
  if (kl_part) {
    kl = wave_sum(kl);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = kl;
    __syncthreads();
    if (threadIdx.x == 0) kl_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void vib_bwd_k(int B, int btl, int k, const T* __restrict__ enc,
                                                 int ld_enc, const float* __restrict__ eps,
                                                 const T* __restrict__ dz, int ld_dz, float beta,
                                                 T* __restrict__ denc, int ld_denc, int Mpe) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)Mpe * ld_denc) return;
  const int b = (int)(idx / ld_denc), c = (int)(idx % ld_denc);
  float out = 0.f;
  if (b < B && c < 2 * btl) {
    const int cc = c < btl ? c : c - btl;
    const float mu = to_f32<T>(enc[(size_t)b * ld_enc + cc]);
    const float lv = to_f32<T>(enc[(size_t)b * ld_enc + btl + cc]);
    if (c < btl) {
      float s = 0.f;
      for (int kk = 0; kk < k; ++kk) s += to_f32<T>(dz[((size_t)kk * B + b) * ld_dz + cc]);
      out = s + beta * mu;
    } else {
      const float sig = __expf(0.5f * lv);
      float s = 0.f;
      for (int kk = 0; kk < k; ++kk)
        s += to_f32<T>(dz[((size_t)kk * B + b) * ld_dz + cc]) * eps[((size_t)kk * B + b) * btl + cc];
      out = 0.5f * sig * s + 0.5f * beta * (__expf(lv) - 1.f);
    }
  }
  denc[idx] = from_f32<T>(out);
}

}  // namespace

// ===========================================================================
// host launchers
// ===========================================================================
static inline int nblk(int64_t n, int b) { return (int)((n + b - 1) / b); }

int mmad_bn_eval_affine(int N, int Np, const float* gamma, const float* beta, const float* rm,
                        const float* rv, float eps, float* scale, float* shift, void* stream) {
  MMAD_CHECK_ARG(N >= 0 && Np >= N, "bn_eval_affine: bad sizes");
  if (Np == 0) return MMAD_OK;
  bn_eval_affine_k<<<nblk(Np, 256), 256, 0, (hipStream_t)stream>>>(N, Np, gamma, beta, rm, rv, eps,
                                                                    scale, shift);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_bn_train_apply(int dtype, int M, int N, int Mp, int Np, const void* a, const float* stats,
                        const float* gamma, const float* beta, float* running_mean,
                        float* running_var, float momentum, float eps, float* save_mean,
                        float* save_rstd, void* y, void* stream) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && M >= 1 && M <= Mp && N <= Np,
                 "bn_train_apply: bad sizes M=%d Mp=%d N=%d Np=%d", M, Mp, N, Np);
  dim3 grd(Np / SLAB_COLS, Mp / SLAB_ROWS);
  const int nparts = Mp / MMAD_PART_ROWS;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    bn_train_apply_k<bf16><<<grd, 256, 0, s>>>(M, N, Np, (const bf16*)a, stats, nparts, gamma, beta,
                                               running_mean, running_var, momentum, eps, save_mean,
                                               save_rstd, (bf16*)y);
  else
    bn_train_apply_k<float><<<grd, 256, 0, s>>>(M, N, Np, (const float*)a, stats, nparts, gamma,
                                                beta, running_mean, running_var, momentum, eps,
                                                save_mean, save_rstd, (float*)y);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_bn_finalize(int M, int N, int Mp, int Np, const float* stats, const float* gamma,
                     const float* beta, float* running_mean, float* running_var, float momentum,
                     float eps, float* save_mean, float* save_rstd, float* scale, float* shift,
                     void* stream) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && M >= 1 && M <= Mp && N <= Np,
                 "bn_finalize: bad sizes");
  bn_finalize_k<<<Np / 64, 64, 0, (hipStream_t)stream>>>(
      M, N, Np, stats, Mp / MMAD_PART_ROWS, gamma, beta, running_mean, running_var, momentum, eps,
      save_mean, save_rstd, scale, shift);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_bn_finalize_fold(int dtype, int M, int N, int Mp, int Np, const float* stats,
                          const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float momentum, float eps, float* save_mean,
                          float* save_rstd, float* scale, float* shift, const float* W, int Nc_p,
                          void* wout, float* cpart, void* stream) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && Nc_p % 64 == 0 && M >= 1 && M <= Mp && N <= Np,
                 "bn_finalize_fold: bad sizes");
  MMAD_CHECK_ARG(Nc_p % 128 == 0, "bn_finalize_fold: consumer rows not a multiple of 128");
  // consumer rows per block: 64 * rpt (the Welford merge is recomputed per
  // block, so fewer, taller blocks read fewer partials)
  const int rpt = 2;   // 64-row consumer groups per block (4 measured no faster, r02bj_*)
  dim3 grd(Np / 64, Nc_p / (64 * rpt));
  hipStream_t s = (hipStream_t)stream;
#define MMAD_FOLD(TW_, R_)                                                                        \
  bn_fold_k<TW_, R_><<<grd, 256, 0, s>>>(M, N, Np, stats, Mp / MMAD_PART_ROWS, gamma, beta,       \
                                         running_mean, running_var, momentum, eps, save_mean,    \
                                         save_rstd, scale, shift, W, (TW_*)wout, cpart, Nc_p);
  if (dtype == MMAD_BF16) {
    if (rpt == 4) { MMAD_FOLD(bf16, 4) } else { MMAD_FOLD(bf16, 2) }
  } else {
    if (rpt == 4) { MMAD_FOLD(float, 4) } else { MMAD_FOLD(float, 2) }
  }
#undef MMAD_FOLD
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_reduce_jobs(const MmadReduceJobs& jobs, int n_jobs, int max_np, void* stream) {
  MMAD_CHECK_ARG(n_jobs >= 1 && n_jobs <= MMAD_MAX_REDUCE_JOBS, "reduce_jobs: bad job count");
  dim3 grd((max_np + 255) / 256, n_jobs);
  reduce_jobs_k<<<grd, 256, 0, (hipStream_t)stream>>>(jobs);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_adam2(const MmadAdamSeg& s0, const MmadAdamSeg& s1, float w1, float w2, float eps,
               float step_size, float bc2_sqrt, void* stream) {
  MMAD_CHECK_ARG(s0.n % 4 == 0 && s1.n % 4 == 0, "adam2: segment lengths must be multiples of 4");
  const int64_t n4 = (s0.n + s1.n) / 4;
  if (n4 == 0) return MMAD_OK;
  adam2_k<<<nblk(n4, 256), 256, 0, (hipStream_t)stream>>>(s0, s1, w1, w2, eps, step_size,
                                                          bc2_sqrt);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_bn_act_bwd_apply(int dtype, int act, float slope, int M, int N, int Mp, int Np,
                          const void* dy, const void* a, const float* save_mean,
                          const float* save_rstd, const float* gamma, const double* part,
                          int nparts, void* dz, float* dgamma, float* dbeta, float* db_partials,
                          void* stream) {
  return mmad_bn_act_bwd_apply_ev(dtype, act, slope, M, N, Mp, Np, dy, a, save_mean, save_rstd, gamma,
                                  part, nparts, dz, dgamma, dbeta, db_partials, stream, nullptr);
}

int mmad_bn_act_bwd_apply_ev(int dtype, int act, float slope, int M, int N, int Mp, int Np,
                             const void* dy, const void* a, const float* save_mean,
                             const float* save_rstd, const float* gamma, const double* part,
                             int nparts, void* dz, float* dgamma, float* dbeta, float* db_partials,
                             void* stream, void* done) {
  // 128-row slabs per block (knob 13: 1, 2 or 4; any other value = 1; halved
  // until it divides the row slabs): the column partials are merged once per
  // block instead of once per 128-row slab
  int rb = mmad_knob(13);
  if (rb != 1 && rb != 2 && rb != 4) rb = 1;
  while (rb > 1 && (Mp / SLAB_ROWS) % rb) rb >>= 1;
  dim3 grd(Np / SLAB_COLS, Mp / (SLAB_ROWS * rb));
  hipStream_t s = (hipStream_t)stream;
  const bool wide = nparts > 4 * 8;   // 16 partial chunks per round trip (8 no faster, r02bj_*)
  const bool lk = act == MMAD_ACT_LEAKYRELU;
  hipEvent_t dev = (hipEvent_t)done;
#define MMAD_BNB_T(T, PU_, RB_, LK_)                                                                   \
  if (dev)                                                                                             \
    hipExtLaunchKernelGGL(bn_bwd_apply_k<T, PU_, RB_, LK_>, grd, dim3(256), 0u, s, nullptr, dev, 0u, act, \
                          slope, M, N, Np, nparts, (const T*)dy, (const T*)a, save_mean, save_rstd,    \
                          gamma, part, (T*)dz, dgamma, dbeta, db_partials);                           \
  else                                                                                                 \
    bn_bwd_apply_k<T, PU_, RB_, LK_><<<grd, 256, 0, s>>>(act, slope, M, N, Np, nparts, (const T*)dy,   \
                                                         (const T*)a, save_mean, save_rstd, gamma,     \
                                                         part, (T*)dz, dgamma, dbeta, db_partials);
#define MMAD_BNB(PU_, RB_)                   \
  if (dtype == MMAD_BF16) {                  \
    if (lk) {                                \
      MMAD_BNB_T(bf16, PU_, RB_, true)       \
    } else {                                 \
      MMAD_BNB_T(bf16, PU_, RB_, false)      \
    }                                        \
  } else if (lk) {                           \
    MMAD_BNB_T(float, PU_, RB_, true)        \
  } else {                                   \
    MMAD_BNB_T(float, PU_, RB_, false)       \
  }
#define MMAD_BNB_RB(PU_)      \
  if (rb == 4) {              \
    MMAD_BNB(PU_, 4)          \
  } else if (rb == 2) {       \
    MMAD_BNB(PU_, 2)          \
  } else {                    \
    MMAD_BNB(PU_, 1)          \
  }
  if (wide) {
    MMAD_BNB_RB(16)
  } else {
    MMAD_BNB_RB(8)
  }
#undef MMAD_BNB_RB
#undef MMAD_BNB
#undef MMAD_BNB_T
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

size_t mmad_bn_act_bwd_ws(int Mp, int Np) { return (size_t)(Mp / SLAB_ROWS) * 2 * Np * sizeof(double); }

int mmad_bn_act_bwd(int dtype, int act, float slope, int M, int N, int Mp, int Np, const void* dy,
                    const void* a, const float* save_mean, const float* save_rstd,
                    const float* gamma, void* dz, float* dgamma, float* dbeta, float* db_partials,
                    void* ws, void* stream) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && M >= 1 && M <= Mp && N <= Np,
                 "bn_act_bwd: bad sizes");
  dim3 grd(Np / SLAB_COLS, Mp / SLAB_ROWS);
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)ws;
  const int nparts = Mp / SLAB_ROWS;
  if (dtype == MMAD_BF16) {
    bn_bwd_reduce_k<bf16><<<grd, 256, 0, s>>>(M, Np, (const bf16*)dy, (const bf16*)a, save_mean,
                                              save_rstd, part);
    bn_bwd_apply_k<bf16, 8, 1, false><<<grd, 256, 0, s>>>(act, slope, M, N, Np, nparts, (const bf16*)dy,
                                             (const bf16*)a, save_mean, save_rstd, gamma, part,
                                             (bf16*)dz, dgamma, dbeta, db_partials);
  } else {
    bn_bwd_reduce_k<float><<<grd, 256, 0, s>>>(M, Np, (const float*)dy, (const float*)a, save_mean,
                                               save_rstd, part);
    bn_bwd_apply_k<float, 8, 1, false><<<grd, 256, 0, s>>>(act, slope, M, N, Np, nparts, (const float*)dy,
                                              (const float*)a, save_mean, save_rstd, gamma, part,
                                              (float*)dz, dgamma, dbeta, db_partials);
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_matrix_colsum_partials(int dtype, int M, int Mp, int Np, const void* x, float* part,
                                void* stream) {
  dim3 grd(Np / SLAB_COLS, Mp / SLAB_ROWS);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    matrix_colsum_k<bf16><<<grd, 256, 0, s>>>(M, Np, (const bf16*)x, part);
  else
    matrix_colsum_k<float><<<grd, 256, 0, s>>>(M, Np, (const float*)x, part);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_colsum(int n_parts, int N, int Np, const float* partials, int part_stride, float scale,
                float* out, void* stream) {
  MMAD_CHECK_ARG(n_parts >= 0 && N <= Np, "colsum: bad sizes");
  if (Np == 0) return MMAD_OK;
  colsum_k<<<nblk(Np, 256), 256, 0, (hipStream_t)stream>>>(n_parts, N, Np, partials, part_stride,
                                                            scale, out);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_sum2d(int rows, int cols, const float* x, int64_t ld, float scale, float* out,
               int accumulate, void* stream) {
  MMAD_CHECK_ARG(rows >= 0 && cols >= 0, "sum2d: bad sizes");
  sum2d_k<<<1, 1024, 0, (hipStream_t)stream>>>(rows, cols, x, ld, scale, out, accumulate);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_sum(int64_t n, const float* x, float scale, float* out, int accumulate, void* stream) {
  MMAD_CHECK_ARG(n >= 0 && n < (1LL << 31), "sum: bad n");
  return mmad_sum2d(1, (int)n, x, n, scale, out, accumulate, stream);
}

int mmad_pack_input_dyn(int dtype, int M, int K, int Mp, int Kp, const float* x, int ld_x,
                        void* out, const MmadDyn* dyn, void* stream) {
  MMAD_CHECK_ARG(M <= Mp && K <= Kp && Kp % 8 == 0 && ld_x >= K, "pack_input: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  // with dyn the source is read at run time: x is the current call's value
  // (same alignment class is required of every later replay, see mmad_ae)
  const int vec = ((uintptr_t)x % 16 == 0 && ld_x % 4 == 0) ? 1 : 0;
  if (dtype == MMAD_BF16) {
    const int64_t n = (int64_t)Mp * (Kp / 8);
    pack_input_k<bf16, 4><<<nblk(n, 256 * 4), 256, 0, s>>>(M, K, Mp, Kp, x, ld_x, vec, (bf16*)out, dyn);
  } else {
    const int64_t n = (int64_t)Mp * (Kp / 4);
    pack_input_k<float, 4><<<nblk(n, 256 * 4), 256, 0, s>>>(M, K, Mp, Kp, x, ld_x, vec, (float*)out, dyn);
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_pack_input(int dtype, int M, int K, int Mp, int Kp, const float* x, int ld_x, void* out,
                    void* stream) {
  return mmad_pack_input_dyn(dtype, M, K, Mp, Kp, x, ld_x, out, nullptr, stream);
}

int mmad_unpack_output(int dtype, int M, int N, int Np, const void* y, float* out, int ld_out,
                       void* stream) {
  MMAD_CHECK_ARG(N <= Np && ld_out >= N, "unpack_output: bad sizes");
  const int64_t n = (int64_t)M * N;
  if (n == 0) return MMAD_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    unpack_k<bf16><<<nblk(n, 256), 256, 0, s>>>(M, N, Np, (const bf16*)y, out, ld_out);
  else
    unpack_k<float><<<nblk(n, 256), 256, 0, s>>>(M, N, Np, (const float*)y, out, ld_out);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_sse_partials(int dtype, int M, int N, int Np, const void* y, const float* x, int ldx,
                      float* part, int nparts, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    sse_k<bf16><<<nparts, 256, 0, s>>>(M, N, Np, (const bf16*)y, x, ldx, part);
  else
    sse_k<float><<<nparts, 256, 0, s>>>(M, N, Np, (const float*)y, x, ldx, part);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

double mmad_decimal_of(float f) {
  // the shortest decimal that rounds to f, as a double: the Python float a
  // caller's optimizer holds (0.9, 0.999, 1e-3) when it reached us as float.
  // std::to_chars / from_chars: shortest round-trip form, independent of the
  // process locale (snprintf / strtod read LC_NUMERIC's decimal point).  A
  // hyper-parameter that was not a short decimal (a scheduler's lr) comes
  // back as the shortest decimal of its float, i.e. within the float's
  // rounding of the caller's double -- the float ABI carries no more.
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof buf, f);
  if (r.ec != std::errc()) return (double)f;
  double d = 0.0;
  const auto q = std::from_chars(buf, r.ptr, d);
  return q.ec == std::errc() && q.ptr == r.ptr ? d : (double)f;
}

MmadAdamConsts mmad_adam_consts(float lr, float beta1, float beta2, float eps, int step) {
  // torch.optim.Adam (_single_tensor_adam): 1 - beta, lr / (1 - beta1^t) and
  // sqrt(1 - beta2^t) in double from the optimizer's double hyper-parameters,
  // each cast to float where torch casts it (the scalar operand of a float op)
  const double b1 = mmad_decimal_of(beta1), b2 = mmad_decimal_of(beta2), l = mmad_decimal_of(lr);
  const double bc1 = 1.0 - pow(b1, step), bc2 = 1.0 - pow(b2, step);
  MmadAdamConsts c;
  c.w1 = (float)(1.0 - b1);
  c.w2 = (float)(1.0 - b2);
  c.eps = eps;
  c.step_size = (float)(l / bc1);
  c.bc2_sqrt = (float)pow(bc2, 0.5);
  return c;
}

int mmad_adam_w(int64_t n, float* p, const float* g, float* m, float* v, float w1, float w2,
                float eps, float step_size, float bc2_sqrt, void* shadow, int64_t n_shadow,
                void* stream) {
  return mmad_adam_dyn(n, p, g, m, v, w1, w2, eps, step_size, bc2_sqrt, shadow, n_shadow, nullptr,
                       stream);
}

int mmad_adam(int64_t n, float* p, const float* g, float* m, float* v, float beta1, float beta2,
              float eps, float step_size, float bc2_sqrt, void* shadow, int64_t n_shadow,
              void* stream) {
  // public entry: the caller's betas; the update constants as torch forms them
  const MmadAdamConsts c = mmad_adam_consts(1e-3f, beta1, beta2, eps, 1);
  return mmad_adam_w(n, p, g, m, v, c.w1, c.w2, eps, step_size, bc2_sqrt, shadow, n_shadow, stream);
}

int mmad_adam_dyn(int64_t n, float* p, const float* g, float* m, float* v, float w1, float w2,
                  float eps, float step_size, float bc2_sqrt, void* shadow, int64_t n_shadow,
                  const MmadDyn* dyn, void* stream) {
  MMAD_CHECK_ARG(n >= 0 && n_shadow >= 0 && n_shadow <= n, "adam: bad sizes");
  if (n == 0) return MMAD_OK;
  MMAD_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                 "adam: buffers must be 16-byte aligned");
  adam_k<<<nblk((n + 3) / 4, 256), 256, 0, (hipStream_t)stream>>>(
      n, p, g, m, v, w1, w2, eps, step_size, bc2_sqrt, (bf16*)shadow, n_shadow, dyn);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_to_bf16(int64_t n, const float* x, void* y, void* stream) {
  if (n == 0) return MMAD_OK;
  to_bf16_k<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, x, (bf16*)y);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_from_bf16(int64_t n, const void* x, float* y, void* stream) {
  if (n == 0) return MMAD_OK;
  from_bf16_k<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(n, (const bf16*)x, y);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_vib_reparam_fwd(int dtype, int B, int btl, int k, const void* enc_out, int ld_enc,
                         const float* eps, float* eps_out, uint64_t seed, uint64_t offset,
                         int deterministic, void* z, int ld_z, float* kl_partial, void* stream) {
  return mmad_vib_reparam_fwd_dyn(dtype, B, btl, k, enc_out, ld_enc, eps, eps_out, seed, offset,
                                  deterministic, z, ld_z, kl_partial, nullptr, stream);
}

int mmad_vib_reparam_fwd_dyn(int dtype, int B, int btl, int k, const void* enc_out, int ld_enc,
                             const float* eps, float* eps_out, uint64_t seed, uint64_t offset,
                             int deterministic, void* z, int ld_z, float* kl_partial,
                             const MmadDyn* dyn, void* stream) {
  MMAD_CHECK_ARG(B >= 1 && btl >= 1 && k >= 1 && ld_enc >= 2 * btl && ld_z >= btl,
                 "vib_reparam_fwd: bad sizes");
  const int Mpz = mmad_roundup(k * B, MMAD_PAD);
  const int64_t n = (int64_t)Mpz * ld_z;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    vib_fwd_k<bf16><<<nblk(n, 256), 256, 0, s>>>(B, btl, k, (const bf16*)enc_out, ld_enc, eps,
                                                 eps_out, seed, offset, deterministic, (bf16*)z,
                                                 ld_z, Mpz, kl_partial, dyn);
  else
    vib_fwd_k<float><<<nblk(n, 256), 256, 0, s>>>(B, btl, k, (const float*)enc_out, ld_enc, eps,
                                                  eps_out, seed, offset, deterministic, (float*)z,
                                                  ld_z, Mpz, kl_partial, dyn);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int64_t mmad_vib_kl_parts(int B, int k, int ld_z) {
  const int Mpz = mmad_roundup(k * B, MMAD_PAD);
  return ((int64_t)Mpz * ld_z + 255) / 256;
}

int mmad_vib_reparam_bwd(int dtype, int B, int btl, int k, const void* enc_out, int ld_enc,
                         const float* eps, const void* dz, int ld_dz, float beta_kl,
                         void* d_enc_out, int ld_denc, float* colsum, void* stream) {
  MMAD_CHECK_ARG(B >= 1 && btl >= 1 && k >= 1 && ld_denc >= 2 * btl, "vib_reparam_bwd: bad sizes");
  const int Mpe = mmad_roundup(B, MMAD_PAD);
  const int64_t n = (int64_t)Mpe * ld_denc;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    vib_bwd_k<bf16><<<nblk(n, 256), 256, 0, s>>>(B, btl, k, (const bf16*)enc_out, ld_enc, eps,
                                                 (const bf16*)dz, ld_dz, beta_kl,
                                                 (bf16*)d_enc_out, ld_denc, Mpe);
  else
    vib_bwd_k<float><<<nblk(n, 256), 256, 0, s>>>(B, btl, k, (const float*)enc_out, ld_enc, eps,
                                                  (const float*)dz, ld_dz, beta_kl,
                                                  (float*)d_enc_out, ld_denc, Mpe);
  MMAD_LAUNCH_CHECK();
  if (colsum) return mmad_matrix_colsum_partials(dtype, B, Mpe, ld_denc, d_enc_out, colsum, stream);
  return MMAD_OK;
}

int mmad_act_bwd(int dtype, int act, float slope, int M, int Mp, int Np, const void* dy,
                 const void* a, void* dz, float* db_partials, void* stream) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && M >= 0 && M <= Mp && dy && a && dz && db_partials,
                 "act_bwd: bad arguments");
  dim3 grd(Np / SLAB_COLS, Mp / SLAB_ROWS);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMAD_BF16)
    act_bwd_k<bf16><<<grd, 256, 0, s>>>(act, slope, M, Np, (const bf16*)dy, (const bf16*)a, (bf16*)dz,
                                        db_partials);
  else
    act_bwd_k<float><<<grd, 256, 0, s>>>(act, slope, M, Np, (const float*)dy, (const float*)a,
                                         (float*)dz, db_partials);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

// ---------------------------------------------------------------------------
// Standalone Activation (modules/activation.py:20-45), fp32: element-wise
// forms one thread per 4 values; softmax / logsoftmax one wave per row
// (max, sum of exp by wave shuffles; rows of any width).
namespace {
__device__ __forceinline__ float act_elem(int act, float v, float slope) {
  switch (act) {
    case MMAD_ACT_LEAKYRELU: return v > 0.f ? v : v * slope;
    case MMAD_ACT_RELU: return v > 0.f ? v : 0.f;
    case MMAD_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    case MMAD_ACT_TANH: return tanhf(v);
    case MMAD_ACT_LOGSIGMOID: return fminf(v, 0.f) - log1pf(expf(-fabsf(v)));
    default: return v;
  }
}
__device__ __forceinline__ float act_elem_grad(int act, float y, float dy, float slope) {
  switch (act) {
    case MMAD_ACT_LEAKYRELU: return y > 0.f ? dy : dy * slope;
    case MMAD_ACT_RELU: return y > 0.f ? dy : 0.f;
    case MMAD_ACT_SIGMOID: return dy * y * (1.f - y);
    case MMAD_ACT_TANH: return dy * (1.f - y * y);
    case MMAD_ACT_LOGSIGMOID: return dy * (1.f - expf(y));   // d/dx log sigma(x) = 1 - sigma(x)
    default: return dy;
  }
}
__global__ __launch_bounds__(256) void act_elem_fwd_k(int act, float slope, int M, int N, const float* x,
                                                      int64_t ldx, float* y, int64_t ldy) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = i / N, c = i % N;
  if (r >= M) return;
  y[r * ldy + c] = act_elem(act, x[r * ldx + c], slope);
}
__global__ __launch_bounds__(256) void act_elem_bwd_k(int act, float slope, int M, int N, const float* y,
                                                      int64_t ldy, const float* dy, int64_t lddy,
                                                      float* dx, int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = i / N, c = i % N;
  if (r >= M) return;
  dx[r * lddx + c] = act_elem_grad(act, y[r * ldy + c], dy[r * lddy + c], slope);
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
// one 64-lane wave per row, 4 rows per block
__global__ __launch_bounds__(256) void act_row_fwd_k(int logsm, int M, int N, const float* x, int64_t ldx,
                                                     float* y, int64_t ldy) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (int64_t)row * ldx;
  float mx = -INFINITY;
  for (int c = lane; c < N; c += 64) mx = fmaxf(mx, xr[c]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s += expf(xr[c] - mx);
  s = wave_sum(s);
  const float ls = logf(s);
  float* yr = y + (int64_t)row * ldy;
  for (int c = lane; c < N; c += 64) {
    const float z = xr[c] - mx;
    yr[c] = logsm ? z - ls : expf(z) / s;
  }
}
__global__ __launch_bounds__(256) void act_row_bwd_k(int logsm, int M, int N, const float* y, int64_t ldy,
                                                     const float* dy, int64_t lddy, float* dx,
                                                     int64_t lddx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* yr = y + (int64_t)row * ldy;
  const float* gr = dy + (int64_t)row * lddy;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s += logsm ? gr[c] : gr[c] * yr[c];
  s = wave_sum(s);
  float* dr = dx + (int64_t)row * lddx;
  for (int c = lane; c < N; c += 64)
    dr[c] = logsm ? gr[c] - expf(yr[c]) * s : yr[c] * (gr[c] - s);
}
}  // namespace

int mmad_activation_fwd(int act, float slope, int M, int N, const float* x, int64_t ldx, float* y,
                        int64_t ldy, void* stream) {
  MMAD_CHECK_ARG(act >= MMAD_ACT_NONE && act <= MMAD_ACT_LOGSOFTMAX, "activation_fwd: bad act %d", act);
  MMAD_CHECK_ARG(M >= 0 && N >= 0 && ldx >= N && ldy >= N && (M == 0 || N == 0 || (x && y)),
                 "activation_fwd: bad arguments");
  if (M == 0 || N == 0) return MMAD_OK;
  hipStream_t s = (hipStream_t)stream;
  if (act == MMAD_ACT_SOFTMAX || act == MMAD_ACT_LOGSOFTMAX) {
    act_row_fwd_k<<<(M + 3) / 4, 256, 0, s>>>(act == MMAD_ACT_LOGSOFTMAX, M, N, x, ldx, y, ldy);
  } else {
    const int64_t n = (int64_t)M * N;
    act_elem_fwd_k<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(act, slope, M, N, x, ldx, y, ldy);
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_activation_bwd(int act, float slope, int M, int N, const float* y, int64_t ldy,
                        const float* dy, int64_t lddy, float* dx, int64_t lddx, void* stream) {
  MMAD_CHECK_ARG(act >= MMAD_ACT_NONE && act <= MMAD_ACT_LOGSOFTMAX, "activation_bwd: bad act %d", act);
  MMAD_CHECK_ARG(M >= 0 && N >= 0 && ldy >= N && lddy >= N && lddx >= N &&
                     (M == 0 || N == 0 || (y && dy && dx)),
                 "activation_bwd: bad arguments");
  if (M == 0 || N == 0) return MMAD_OK;
  hipStream_t s = (hipStream_t)stream;
  if (act == MMAD_ACT_SOFTMAX || act == MMAD_ACT_LOGSOFTMAX) {
    act_row_bwd_k<<<(M + 3) / 4, 256, 0, s>>>(act == MMAD_ACT_LOGSOFTMAX, M, N, y, ldy, dy, lddy, dx, lddx);
  } else {
    const int64_t n = (int64_t)M * N;
    act_elem_bwd_k<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(act, slope, M, N, y, ldy, dy, lddy, dx, lddx);
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

// ---------------------------------------------------------------------------
// Standalone reconstruction loss, modules/loss.py:47-52 (Loss('mse',
// reduction)): sum (or mean) of (y_hat - y)^2 and its gradient.  (Inside the
// autoencoder the sum-MSE is fused into the last decoder GEMM's epilogue;
// this is the plugin-surface Loss called on its own.)  Deterministic: a fixed
// grid of MSE_PARTS blocks, each a fixed strided order, then one block sums
// the partials in order.
namespace {
constexpr int MSE_PARTS = 256;
__global__ __launch_bounds__(256) void mse_partials_k(int64_t n, const float* __restrict__ a,
                                                      const float* __restrict__ b, float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  const bool vec = (((uintptr_t)a | (uintptr_t)b) % 16) == 0;
  const int64_t n4 = vec ? n / 4 : 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)MSE_PARTS * 256) {
    const floatx4 x = ((const floatx4*)a)[i], y = ((const floatx4*)b)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = x[e] - y[e];
      acc = fmaf(d, d, acc);
    }
  }
  for (int64_t i = 4 * n4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)MSE_PARTS * 256) {
    const float d = a[i] - b[i];
    acc = fmaf(d, d, acc);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ __launch_bounds__(256) void mse_grad_k(int64_t n, const float* __restrict__ a,
                                                  const float* __restrict__ b, const float* __restrict__ g,
                                                  float scale, float* __restrict__ da, float* __restrict__ db) {
  const float s = scale * (g ? g[0] : 1.f);
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float d = s * (a[i] - b[i]);
    if (da) da[i] = d;
    if (db) db[i] = -d;
  }
}
}  // namespace

int mmad_mse_loss_ws_floats(void) { return MSE_PARTS; }

int mmad_mse_loss(int64_t n, const float* y_hat, const float* y, int mean, float* loss_out, float* work,
                  void* stream) {
  MMAD_CHECK_ARG(n >= 1 && y_hat && y && loss_out && work, "mse_loss: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  mse_partials_k<<<MSE_PARTS, 256, 0, s>>>(n, y_hat, y, work);
  MMAD_LAUNCH_CHECK();
  return mmad_sum(MSE_PARTS, work, mean ? (float)(1.0 / (double)n) : 1.f, loss_out, 0, stream);
}

int mmad_mse_grad(int64_t n, const float* y_hat, const float* y, const float* g, int mean, float* d_yhat,
                  float* d_y, void* stream) {
  MMAD_CHECK_ARG(n >= 1 && y_hat && y && (d_yhat || d_y), "mse_grad: bad arguments");
  const float scale = mean ? (float)(2.0 / (double)n) : 2.f;
  const int64_t blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
  mse_grad_k<<<(int)blocks, 256, 0, (hipStream_t)stream>>>(n, y_hat, y, g, scale, d_yhat, d_y);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}
