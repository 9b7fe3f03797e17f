// NAP fit on the device (utils/metric.py:183-238 fits it on the train diffs):
//   Rotater.fit     utils/normalize.py:52-70   mu_r = mean(x), V = right
//                                              singular vectors of x - mu_r
//   Standardizer.fit utils/normalize.py:25-34 on the rotated train diffs
//                                              rot = (x - mu_r) V (fp32 matmul,
//                                              Rotater.run :72-103):
//                                              mu_s = mean(rot), var = ddof-1
//                                              variance of rot (np.cov, fp64)
//
// Schedule (all on the caller's stream, caller-owned workspace):
//   1. column means of x, fp64 partials per row chunk, reduced in chunk order
//      -> mu_r (fp32, as the reference's x.float().mean(0))
//   2. Gram G = xc^T xc in fp64 (xc = fp32(x - mu_r) formed on the fly while
//      staging tiles in LDS), upper-triangular 64x64 tile set, mirrored
//   3. eigendecomposition of G (rocSOLVER dsyevd, the one library call; the
//      right singular vectors of xc are G's eigenvectors), descending order
//      -> V [W][R], R = min(N, W)
//   4. rot = xc V in fp32 (LDS-tiled FMA), column sum / sum of squares in
//      fp64 per row chunk, reduced in chunk order -> mu_s, var
// Every reduction has a fixed order: the fit is deterministic.
//
// rocSOLVER / rocBLAS are resolved at run time from the copies already in the
// process (torch's librocsolver.so.0 / librocblas.so.5), falling back to
// dlopen by soname: one instance per process, no link-time dependency.
#include <dlfcn.h>
#include <mutex>

#include "mmad_common.h"

namespace {

constexpr int MEAN_COLS = 256;     // columns per block of the mean pass
constexpr int MEAN_ROWS = 2048;    // rows per partial
constexpr int GT = 64;             // Gram / rotation output tile
constexpr int GK = 32;             // rows (Gram) / features (rotation) per LDS stage
constexpr int ROT_ROWS = 1024;     // rows per rotation-statistics partial

__global__ __launch_bounds__(256) void nap_colsum_k(int64_t N, int W, const float* __restrict__ x,
                                                    int64_t ldx, double* __restrict__ part) {
  const int c = blockIdx.x * MEAN_COLS + threadIdx.x;
  if (c >= W) return;
  const int64_t r0 = (int64_t)blockIdx.y * MEAN_ROWS;
  const int64_t r1 = r0 + MEAN_ROWS < N ? r0 + MEAN_ROWS : N;
  double s = 0.0;
  for (int64_t r = r0; r < r1; ++r) s += (double)x[r * ldx + c];
  part[(int64_t)blockIdx.y * W + c] = s;
}

__global__ __launch_bounds__(256) void nap_mean_k(int64_t N, int W, int nparts,
                                                  const double* __restrict__ part,
                                                  float* __restrict__ mu) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= W) return;
  double s = 0.0;
  for (int p = 0; p < nparts; ++p) s += part[(int64_t)p * W + c];
  mu[c] = (float)(s / (double)N);
}

// G[i][j] = sum_n xc[n][i] xc[n][j], tiles (ti <= tj) of 64x64, 256 threads,
// 4x4 outputs per thread (rows ty + 16a, cols tx + 16b: conflict-free LDS reads)
__global__ __launch_bounds__(256) void nap_gram_k(int64_t N, int W, const float* __restrict__ x,
                                                  int64_t ldx, const float* __restrict__ mu,
                                                  int T, double* __restrict__ G) {
  // linear upper-triangular tile index -> (ti, tj), ti <= tj
  int t = blockIdx.x, ti = 0;
  while (t >= T - ti) { t -= T - ti; ++ti; }
  const int tj = ti + t;
  const int i0 = ti * GT, j0 = tj * GT;
  __shared__ double As[GK][GT];
  __shared__ double Bs[GK][GT];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  double acc[4][4] = {};
  const int lc = tid & 63, lr = tid >> 6;   // loader: column lc, rows lr + 4q
  const int ci = i0 + lc, cj = j0 + lc;
  const float mi = ci < W ? mu[ci] : 0.f, mj = cj < W ? mu[cj] : 0.f;
  for (int64_t n0 = 0; n0 < N; n0 += GK) {
#pragma unroll
    for (int q = 0; q < GK / 4; ++q) {
      const int r = lr + 4 * q;
      const int64_t n = n0 + r;
      float a = 0.f, b = 0.f;
      if (n < N) {
        if (ci < W) a = x[n * ldx + ci] - mi;   // fp32 centring, as the reference's x - mu
        if (cj < W) b = x[n * ldx + cj] - mj;
      }
      As[r][lc] = (double)a;
      Bs[r][lc] = (double)b;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < GK; ++k) {
      double av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { av[u] = As[k][ty + 16 * u]; bv[u] = Bs[k][tx + 16 * u]; }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[u][w] = fma(av[u], bv[w], acc[u][w]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int i = i0 + ty + 16 * u, j = j0 + tx + 16 * w;
      if (i < W && j < W) {
        G[(int64_t)i * W + j] = acc[u][w];
        G[(int64_t)j * W + i] = acc[u][w];
      }
    }
}

// dsyevd leaves eigenvectors in the columns of the (column-major) matrix in
// ascending eigenvalue order: V[i][r] = A[i + (W-1-r) W], r < R
__global__ __launch_bounds__(256) void nap_evec_k(int W, int R, const double* __restrict__ A,
                                                  float* __restrict__ v) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)W * R) return;
  const int i = (int)(e / R), r = (int)(e % R);
  v[e] = (float)A[(int64_t)(W - 1 - r) * W + i];
}

// rot = xc V (fp32, Rotater.run's matmul): per block a 64-column slice of rot
// over a ROT_ROWS row chunk, as 64x64 sub-tiles; per column the fp64 sums of
// rot and rot^2 over the chunk -> part[chunk][2][R]
__global__ __launch_bounds__(256) void nap_rotstats_k(int64_t N, int W, int R,
                                                      const float* __restrict__ x, int64_t ldx,
                                                      const float* __restrict__ mu,
                                                      const float* __restrict__ v,
                                                      double* __restrict__ part) {
  __shared__ float Xs[GT][GK + 1];
  __shared__ float Vs[GK][GT];
  __shared__ double red[2][16][GT];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int c0 = blockIdx.x * GT;
  const int64_t rbeg = (int64_t)blockIdx.y * ROT_ROWS;
  const int64_t rend = rbeg + ROT_ROWS < N ? rbeg + ROT_ROWS : N;
  double s1[4] = {}, s2[4] = {};
  for (int64_t m0 = rbeg; m0 < rend; m0 += GT) {
    float acc[4][4] = {};
    for (int k0 = 0; k0 < W; k0 += GK) {
      // X tile [64 rows][32 features]: thread -> feature tid & 31, rows (tid >> 5) + 8q
#pragma unroll
      for (int q = 0; q < GT / 8; ++q) {
        const int r = (tid >> 5) + 8 * q, k = tid & 31;
        const int64_t n = m0 + r;
        const int f = k0 + k;
        Xs[r][k] = (n < rend && f < W) ? x[n * ldx + f] - mu[f] : 0.f;
      }
      // V tile [32 features][64 columns]
#pragma unroll
      for (int q = 0; q < GK / 4; ++q) {
        const int k = (tid >> 6) + 4 * q, c = tid & 63;
        const int f = k0 + k;
        Vs[k][c] = (f < W && c0 + c < R) ? v[(int64_t)f * R + c0 + c] : 0.f;
      }
      __syncthreads();
#pragma unroll 8
      for (int k = 0; k < GK; ++k) {
        float av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { av[u] = Xs[ty + 16 * u][k]; bv[u] = Vs[k][tx + 16 * u]; }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int w = 0; w < 4; ++w) acc[u][w] = fmaf(av[u], bv[w], acc[u][w]);
      }
      __syncthreads();
    }
    // rows past the chunk end hold 0 (zero X rows): they add nothing
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const double r = (double)acc[u][w];
        s1[w] += r;
        s2[w] += r * r;
      }
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    red[0][ty][tx + 16 * w] = s1[w];
    red[1][ty][tx + 16 * w] = s2[w];
  }
  __syncthreads();
  if (tid < 2 * GT) {
    const int which = tid / GT, c = tid % GT;
    double s = 0.0;
    for (int y = 0; y < 16; ++y) s += red[which][y][c];
    if (c0 + c < R) part[((int64_t)blockIdx.y * 2 + which) * R + c0 + c] = s;
  }
}

__global__ __launch_bounds__(256) void nap_stats_k(int64_t N, int R, int nparts,
                                                   const double* __restrict__ part,
                                                   float* __restrict__ mu_s,
                                                   float* __restrict__ var) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= R) return;
  double s1 = 0.0, s2 = 0.0;
  for (int p = 0; p < nparts; ++p) {
    s1 += part[((int64_t)p * 2 + 0) * R + c];
    s2 += part[((int64_t)p * 2 + 1) * R + c];
  }
  const double mean = s1 / (double)N;
  mu_s[c] = (float)mean;
  const double ss = s2 - s1 * mean;                  // sum (rot - mean)^2
  var[c] = (float)((ss > 0.0 ? ss : 0.0) / (double)(N - 1));
}

// ---- rocSOLVER (run-time resolved) ---------------------------------------
typedef void* rb_handle;
struct SolverApi {
  int (*create_handle)(rb_handle*);
  int (*destroy_handle)(rb_handle);
  int (*set_stream)(rb_handle, hipStream_t);
  int (*dsyevd)(rb_handle, int evect, int uplo, int n, double* A, int lda, double* D, double* E,
                int* info);
  bool ok;
};
constexpr int RB_EVECT_ORIGINAL = 211;   // rocblas_evect_original
constexpr int RB_FILL_UPPER = 121;       // rocblas_fill_upper

void* find_lib(const char* sym, const char* soname) {
  if (dlsym(RTLD_DEFAULT, sym)) return RTLD_DEFAULT;
  return dlopen(soname, RTLD_NOW | RTLD_GLOBAL);
}

const SolverApi& solver() {
  static SolverApi api{};
  static std::once_flag once;
  std::call_once(once, [] {
    void* hb = find_lib("rocblas_create_handle", "librocblas.so.5");
    void* hs = find_lib("rocsolver_dsyevd", "librocsolver.so.0");
    if (!hb || !hs) return;
    api.create_handle = (decltype(api.create_handle))dlsym(hb, "rocblas_create_handle");
    api.destroy_handle = (decltype(api.destroy_handle))dlsym(hb, "rocblas_destroy_handle");
    api.set_stream = (decltype(api.set_stream))dlsym(hb, "rocblas_set_stream");
    api.dsyevd = (decltype(api.dsyevd))dlsym(hs, "rocsolver_dsyevd");
    api.ok = api.create_handle && api.destroy_handle && api.set_stream && api.dsyevd;
  });
  return api;
}

struct FitWS {
  double* G;       // [W][W]
  double* D;       // [W] eigenvalues
  double* E;       // [W] dsyevd scratch
  double* mpart;   // [ceil(N / MEAN_ROWS)][W]
  double* rpart;   // [ceil(N / ROT_ROWS)][2][R]
  int* info;
  size_t total;
};

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

FitWS carve_fit(int64_t N, int W, char* base) {
  const int64_t R = N < W ? N : W;
  FitWS w{};
  size_t o = 0;
  auto take = [&](size_t bytes) { char* p = base ? base + o : nullptr; o += al256(bytes); return p; };
  w.G = (double*)take((size_t)W * W * 8);
  w.D = (double*)take((size_t)W * 8);
  w.E = (double*)take((size_t)W * 8);
  w.mpart = (double*)take((size_t)((N + MEAN_ROWS - 1) / MEAN_ROWS) * W * 8);
  w.rpart = (double*)take((size_t)((N + ROT_ROWS - 1) / ROT_ROWS) * 2 * R * 8);
  w.info = (int*)take(sizeof(int));
  w.total = o;
  return w;
}

}  // namespace

size_t mmad_nap_fit_ws_bytes(int64_t N, int W) {
  if (N < 2 || W < 1) return 0;
  return carve_fit(N, W, nullptr).total;
}

int mmad_nap_fit(int64_t N, int W, const float* x, int64_t ldx, float* mu_r, float* v, float* mu_s,
                 float* var, void* ws, size_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(N >= 2 && W >= 1 && W <= 46340 && ldx >= W && x && mu_r && v && mu_s && var && ws,
                 "nap_fit: bad arguments (N=%lld W=%d ldx=%lld)", (long long)N, W, (long long)ldx);
  MMAD_CHECK_ARG(N / MEAN_ROWS < 65535 && N / ROT_ROWS < 65535, "nap_fit: N=%lld too large",
                 (long long)N);
  const FitWS w = carve_fit(N, W, (char*)ws);
  MMAD_CHECK_ARG(ws_bytes >= w.total, "nap_fit: workspace %zu < %zu bytes", ws_bytes, w.total);
  MMAD_CHECK_ARG(((uintptr_t)ws) % 256 == 0, "nap_fit: workspace must be 256-byte aligned");
  const SolverApi& api = solver();
  if (!api.ok) {
    mmad_set_error("nap_fit: rocSOLVER / rocBLAS not found in the process (librocsolver.so.0)");
    return MMAD_EHIP;
  }
  hipStream_t s = (hipStream_t)stream;
  const int R = (int)(N < W ? N : W);
  const int mparts = (int)((N + MEAN_ROWS - 1) / MEAN_ROWS);
  nap_colsum_k<<<dim3((W + MEAN_COLS - 1) / MEAN_COLS, mparts), 256, 0, s>>>(N, W, x, ldx, w.mpart);
  MMAD_LAUNCH_CHECK();
  nap_mean_k<<<(W + 255) / 256, 256, 0, s>>>(N, W, mparts, w.mpart, mu_r);
  MMAD_LAUNCH_CHECK();
  const int T = (W + GT - 1) / GT;
  nap_gram_k<<<T * (T + 1) / 2, 256, 0, s>>>(N, W, x, ldx, mu_r, T, w.G);
  MMAD_LAUNCH_CHECK();
  rb_handle h = nullptr;
  if (api.create_handle(&h) != 0) {
    mmad_set_error("nap_fit: rocblas_create_handle failed");
    return MMAD_EHIP;
  }
  int st = api.set_stream(h, s);
  if (st == 0) st = api.dsyevd(h, RB_EVECT_ORIGINAL, RB_FILL_UPPER, W, w.G, W, w.D, w.E, w.info);
  int info = 0;
  const hipError_t ce = hipMemcpyAsync(&info, w.info, sizeof(int), hipMemcpyDeviceToHost, s);
  const hipError_t se = ce == hipSuccess ? hipStreamSynchronize(s) : ce;
  api.destroy_handle(h);
  if (st != 0) {
    mmad_set_error("nap_fit: rocsolver_dsyevd returned status %d", st);
    return MMAD_EHIP;
  }
  MMAD_HIP_CHECK(se);
  if (info != 0) {
    mmad_set_error("nap_fit: eigensolver did not converge (info=%d)", info);
    return MMAD_EHIP;
  }
  const int64_t nv = (int64_t)W * R;
  nap_evec_k<<<(unsigned)((nv + 255) / 256), 256, 0, s>>>(W, R, w.G, v);
  MMAD_LAUNCH_CHECK();
  const int rparts = (int)((N + ROT_ROWS - 1) / ROT_ROWS);
  nap_rotstats_k<<<dim3((R + GT - 1) / GT, rparts), 256, 0, s>>>(N, W, R, x, ldx, mu_r, v, w.rpart);
  MMAD_LAUNCH_CHECK();
  nap_stats_k<<<(R + 255) / 256, 256, 0, s>>>(N, R, rparts, w.rpart, mu_s, var);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}
