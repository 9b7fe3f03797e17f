// Anomaly-score metrics on the device (utils/metric.py of the reference, which
// runs them through sklearn / numpy on the host):
//   AUROC = metrics.auc(metrics.roc_curve(label, score))        :29-44
//   AUPR  = metrics.auc(recall, precision) of
//           metrics.precision_recall_curve(label, score)       :97-116
//   F1 at the valid 90 % quantile (test > thr)                  :118-130
//   precision / recall of the confusion matrix (test >= thr)    :83-95
//
// Rank metrics: one descending radix sort of (order-preserving key, label)
// pairs (rocPRIM) + an inclusive scan of the sorted labels; then every element
// finds its tie run [lo, hi) by binary search on the sorted keys, so
//   AUROC U = sum over positives of (#neg in later runs + 0.5 #neg in its run)
//   AUPR     = sum over run ends j of (R_j - R_{j-1}) (P_j + P_{j-1}) / 2
// with (R_{-1}, P_{-1}) = (0, 1): the trapezoid sklearn.metrics.auc takes
// over precision_recall_curve's points (one per distinct threshold, no
// dropped points, the (recall 0, precision 1) end point appended).  Both sums
// are fp64, reduced per block and then in block order (deterministic).
// Ties count one half exactly as roc_curve's collapsed thresholds do.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "mmad_common.h"

namespace {

__device__ __forceinline__ uint32_t order_key(float f) {
  uint32_t u = f == 0.f ? 0u : __float_as_uint(f);     // -0.0 ties with +0.0
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);   // ascending float order
}

__global__ void keys_k(int64_t n, const float* __restrict__ score, const uint8_t* __restrict__ label,
                       uint32_t* __restrict__ key, uint8_t* __restrict__ lab) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = order_key(score[i]);
  lab[i] = label[i] ? 1 : 0;
}

// first index in [0, n) whose (descending) key is <= k  /  < k
__device__ __forceinline__ int64_t first_le(const uint32_t* key, int64_t n, uint32_t k) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key[mid] > k) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t first_lt(const uint32_t* key, int64_t n, uint32_t k) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key[mid] >= k) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) t += red[q];
  __syncthreads();
  return t;
}

// per block: partial U (AUROC numerator) and partial AUPR area
__global__ __launch_bounds__(256) void rank_contrib_k(int64_t n, const uint32_t* __restrict__ key,
                                                      const uint8_t* __restrict__ lab,
                                                      const uint32_t* __restrict__ cum,
                                                      double* __restrict__ part) {
  __shared__ double red[4];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const double P = n > 0 ? (double)cum[n - 1] : 0.0;
  double u = 0.0, a = 0.0;
  if (i < n) {
    const uint32_t k = key[i];
    const int64_t lo = first_le(key, n, k), hi = first_lt(key, n, k);
    const double pos_before = lo > 0 ? (double)cum[lo - 1] : 0.0;
    const double pos_run = (double)cum[hi - 1] - pos_before;
    if (lab[i]) {
      const double neg_after = (double)(n - hi) - (P - (double)cum[hi - 1]);
      const double neg_run = (double)(hi - lo) - pos_run;
      u = neg_after + 0.5 * neg_run;
    }
    if (i == hi - 1) {
      const double tp = (double)cum[i], cnt = (double)(i + 1);
      const double prec = tp / cnt;                       // cnt > 0
      const double rec = P > 0.0 ? tp / P : 1.0;
      double prec_p = 1.0, rec_p = 0.0;
      if (lo > 0) {
        prec_p = pos_before / (double)lo;
        rec_p = P > 0.0 ? pos_before / P : 1.0;
      }
      a = (rec - rec_p) * (prec + prec_p) * 0.5;
    }
  }
  const double su = block_sum_d(u, red);
  const double sa = block_sum_d(a, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = su;
    part[2 * blockIdx.x + 1] = sa;
  }
}

// out: auroc, aupr, n_pos, n_neg (fp64)
__global__ __launch_bounds__(256) void rank_final_k(int64_t n, int nblk, const double* __restrict__ part,
                                                    const uint32_t* __restrict__ cum,
                                                    double* __restrict__ out) {
  __shared__ double red[4];
  double u = 0.0, a = 0.0;
  // fixed order: thread t sums blocks t, t+256, ... then the block sum
  for (int b = threadIdx.x; b < nblk; b += 256) {
    u += part[2 * b];
    a += part[2 * b + 1];
  }
  const double su = block_sum_d(u, red);
  const double sa = block_sum_d(a, red);
  if (threadIdx.x == 0) {
    const double P = n > 0 ? (double)cum[n - 1] : 0.0, N = (double)n - P;
    out[0] = (P > 0.0 && N > 0.0) ? su / (P * N) : __builtin_nan("");
    out[1] = sa;
    out[2] = P;
    out[3] = N;
  }
}

// threshold = quantile(sorted ascending valid, q) with numpy's 'linear' rule
// (virtual index q (n-1)); counts for F1 (test > thr) and the confusion
// matrix (test >= thr).  out: thr, f1, p, r, precision, recall, tp, fp, fn, tn
__global__ __launch_bounds__(256) void threshold_k(int64_t nv, const float* __restrict__ vs_sorted, double q,
                                                   int64_t nt, const float* __restrict__ test,
                                                   const uint8_t* __restrict__ label,
                                                   double* __restrict__ out) {
  __shared__ double red[4];
  __shared__ float s_thr;
  if (threadIdx.x == 0) {
    const double vi = q * (double)(nv - 1);
    int64_t lo = (int64_t)floor(vi);
    if (lo < 0) lo = 0;
    if (lo > nv - 1) lo = nv - 1;
    const int64_t hi = lo + 1 < nv ? lo + 1 : nv - 1;
    const double g = vi - (double)lo;
    const double a = vs_sorted[lo], b = vs_sorted[hi];
    // numpy _lerp: a + (b - a) * g, switched to b - (b - a) * (1 - g) for g >= 0.5
    const double thr = g >= 0.5 ? b - (b - a) * (1.0 - g) : a + (b - a) * g;
    s_thr = (float)thr;
    out[0] = (double)(float)thr;
  }
  __syncthreads();
  const float thr = s_thr;
  double gt_pos = 0, gt = 0, ge_pos = 0, ge = 0, pos = 0;
  for (int64_t i = threadIdx.x; i < nt; i += 256) {
    const float s = test[i];
    const bool l = label[i] != 0;
    gt += s > thr;
    gt_pos += (s > thr) && l;
    ge += s >= thr;
    ge_pos += (s >= thr) && l;
    pos += l;
  }
  gt = block_sum_d(gt, red);
  gt_pos = block_sum_d(gt_pos, red);
  ge = block_sum_d(ge, red);
  ge_pos = block_sum_d(ge_pos, red);
  pos = block_sum_d(pos, red);
  if (threadIdx.x == 0) {
    const double nan = __builtin_nan("");
    const double p = gt > 0 ? gt_pos / gt : nan, r = pos > 0 ? gt_pos / pos : nan;
    out[1] = p * r * 2.0 / (p + r);
    out[2] = p;
    out[3] = r;
    const double tp = ge_pos, fp = ge - ge_pos, fn = pos - ge_pos, tn = (double)nt - ge - fn;
    out[4] = tp + fp > 0 ? tp / (tp + fp) : nan;
    out[5] = tp + fn > 0 ? tp / (tp + fn) : nan;
    out[6] = tp;
    out[7] = fp;
    out[8] = fn;
    out[9] = tn;
  }
}

struct RankWS {
  uint32_t *key_in, *key_out, *cum;
  uint8_t *lab_in, *lab_out;
  double* part;
  void* tmp;
  size_t tmp_bytes;
  size_t total;
};

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

hipError_t carve_rank(int64_t n, char* base, RankWS& w) {
  size_t off = 0;
  auto take = [&](size_t b) -> char* {
    char* p = base ? base + off : nullptr;
    off += align256(b);
    return p;
  };
  w.key_in = (uint32_t*)take(n * 4);
  w.key_out = (uint32_t*)take(n * 4);
  w.cum = (uint32_t*)take(n * 4);
  w.lab_in = (uint8_t*)take(n);
  w.lab_out = (uint8_t*)take(n);
  w.part = (double*)take((size_t)2 * ((n + 255) / 256 + 1) * 8);
  size_t sort_b = 0, scan_b = 0;
  hipError_t e = rocprim::radix_sort_pairs_desc(nullptr, sort_b, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                (uint8_t*)nullptr, (uint8_t*)nullptr, (size_t)n);
  if (e != hipSuccess) return e;
  e = rocprim::inclusive_scan(nullptr, scan_b, (const uint8_t*)nullptr, (uint32_t*)nullptr, (size_t)n,
                              rocprim::plus<uint32_t>());
  if (e != hipSuccess) return e;
  w.tmp_bytes = sort_b > scan_b ? sort_b : scan_b;
  w.tmp = take(w.tmp_bytes);
  w.total = off;
  return hipSuccess;
}

}  // namespace

size_t mmad_rank_metrics_ws_bytes(int64_t n) {
  if (n < 1) n = 1;
  RankWS w;
  if (carve_rank(n, nullptr, w) != hipSuccess) return 0;
  return w.total;
}

int mmad_rank_metrics(int64_t n, const float* score, const uint8_t* label, double* out, void* ws,
                      size_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(n >= 1 && n < (1LL << 31) && score && label && out && ws,
                 "rank_metrics: bad arguments (n=%lld)", (long long)n);
  RankWS w;
  MMAD_HIP_CHECK(carve_rank(n, (char*)ws, w));
  MMAD_CHECK_ARG(ws_bytes >= w.total, "rank_metrics: workspace %zu < %zu bytes", ws_bytes, w.total);
  MMAD_CHECK_ARG(((uintptr_t)ws) % 256 == 0, "rank_metrics: workspace must be 256-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)((n + 255) / 256);
  keys_k<<<nb, 256, 0, s>>>(n, score, label, w.key_in, w.lab_in);
  MMAD_LAUNCH_CHECK();
  size_t tb = w.tmp_bytes;
  MMAD_HIP_CHECK(rocprim::radix_sort_pairs_desc(w.tmp, tb, w.key_in, w.key_out, w.lab_in, w.lab_out,
                                                (size_t)n, 0, 32, s));
  tb = w.tmp_bytes;
  MMAD_HIP_CHECK(rocprim::inclusive_scan(w.tmp, tb, (const uint8_t*)w.lab_out, w.cum, (size_t)n,
                                         rocprim::plus<uint32_t>(), s));
  rank_contrib_k<<<nb, 256, 0, s>>>(n, w.key_out, w.lab_out, w.cum, w.part);
  MMAD_LAUNCH_CHECK();
  rank_final_k<<<1, 256, 0, s>>>(n, nb, w.part, w.cum, out);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

size_t mmad_threshold_metrics_ws_bytes(int64_t n_valid) {
  if (n_valid < 1) n_valid = 1;
  size_t sort_b = 0;
  if (rocprim::radix_sort_keys(nullptr, sort_b, (float*)nullptr, (float*)nullptr, (size_t)n_valid) !=
      hipSuccess)
    return 0;
  return align256((size_t)n_valid * 4) + align256(sort_b);
}

int mmad_threshold_metrics(int64_t n_valid, const float* valid, int64_t n_test, const float* test,
                           const uint8_t* label, double q, double* out, void* ws, size_t ws_bytes,
                           void* stream) {
  MMAD_CHECK_ARG(n_valid >= 1 && n_valid < (1LL << 31) && n_test >= 1 && valid && test && label &&
                     out && ws && q >= 0.0 && q <= 1.0,
                 "threshold_metrics: bad arguments");
  const size_t need = mmad_threshold_metrics_ws_bytes(n_valid);
  MMAD_CHECK_ARG(need > 0 && ws_bytes >= need, "threshold_metrics: workspace %zu < %zu bytes", ws_bytes,
                 need);
  hipStream_t s = (hipStream_t)stream;
  float* sorted = (float*)ws;
  void* tmp = (char*)ws + align256((size_t)n_valid * 4);
  size_t tb = need - align256((size_t)n_valid * 4);
  MMAD_HIP_CHECK(rocprim::radix_sort_keys(tmp, tb, valid, sorted, (size_t)n_valid, 0, 32, s));
  threshold_k<<<1, 256, 0, s>>>(n_valid, sorted, q, n_test, test, label, out);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}
