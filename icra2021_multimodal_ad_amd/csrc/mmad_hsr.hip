// HSR_Net multimodal fusion producer (utils/data_loaders.py:152-229), batched.
//
// The reference runs the fusion net one window at a time in a Python loop and
// grows its output with torch.cat (O(N^2) copies, :183-228).  Here one
// 256-thread workgroup produces one window's whole fused row: the RGB and
// depth conv stacks (2x2/s2 -> 3x3/p1 -> 2x2/s2, ReLU after each) run through
// two LDS planes, the F/T scalar is broadcast and the mic MFCCs go through the
// two 1-D convs the reference borrows from its LiDAR branch (conv1l, conv2l;
// :217-220).  fp32 throughout (the reference's dtype); the weights are
// wave-uniform reads (scalar cache), activations live in LDS, and each output
// channel plane is one coalesced 64- or 256-float store into the window's row.
#include "mmad_common.h"
#include "mmad_ops.h"

namespace {
// packed weight layout (mmad_hsr_weight_count floats), torch shapes [co][ci][k..]
constexpr int W1R = 0;           // conv1r.weight [16][3][2][2]
constexpr int B1R = W1R + 192;
constexpr int W2R = B1R + 16;    // conv2r.weight [16][16][3][3]
constexpr int B2R = W2R + 2304;
constexpr int W3R = B2R + 16;    // conv3r.weight [16][16][2][2]
constexpr int B3R = W3R + 1024;
constexpr int W1D = B3R + 16;    // conv1d.weight [8][1][2][2]
constexpr int B1D = W1D + 32;
constexpr int W2D = B1D + 8;     // conv2d.weight [8][8][3][3]
constexpr int B2D = W2D + 576;
constexpr int W3D = B2D + 8;     // conv3d.weight [8][8][2][2]
constexpr int B3D = W3D + 256;
constexpr int W1L = B3D + 8;     // conv1l.weight [8][1][18] (k 18, stride 9, pad 9)
constexpr int B1L = W1L + 144;
constexpr int W2L = B1L + 8;     // conv2l.weight [16][8][2] (k 2, stride 2)
constexpr int B2L = W2L + 256;
constexpr int NWEIGHTS = B2L + 16;

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// One image stack: C0 input planes of 32x32 -> C channels: 2x2/s2 (16x16),
// 3x3/p1 (16x16), 2x2/s2 (8x8).  Thread tid owns position (y, x) of the
// 16x16 planes, then 64 output positions x (C*64/256) channels of the last conv.
template <int C0, int C>
__device__ __forceinline__ void image_stack(const float* __restrict__ img, const float* __restrict__ w,
                                            int w1, int b1, int w2, int b2, int w3, int b3,
                                            float* sA, float* sB, float* __restrict__ orow, int tid) {
  const int y = tid >> 4, x = tid & 15;
  {
    float in[C0 * 4];
#pragma unroll
    for (int ic = 0; ic < C0; ++ic)
#pragma unroll
      for (int ky = 0; ky < 2; ++ky)
#pragma unroll
        for (int kx = 0; kx < 2; ++kx)
          in[ic * 4 + ky * 2 + kx] = img[ic * 1024 + (2 * y + ky) * 32 + 2 * x + kx];
#pragma unroll
    for (int oc = 0; oc < C; ++oc) {
      float acc = w[b1 + oc];
#pragma unroll
      for (int i = 0; i < C0 * 4; ++i) acc = fmaf(in[i], w[w1 + oc * C0 * 4 + i], acc);
      sA[oc * 256 + tid] = relu(acc);
    }
  }
  __syncthreads();
  {
    float acc[C];
#pragma unroll
    for (int oc = 0; oc < C; ++oc) acc[oc] = w[b2 + oc];
    for (int ic = 0; ic < C; ++ic) {
      float nb[9];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int yy = y + ky - 1, xx = x + kx - 1;
          nb[ky * 3 + kx] = (yy >= 0 && yy < 16 && xx >= 0 && xx < 16) ? sA[ic * 256 + yy * 16 + xx] : 0.f;
        }
#pragma unroll
      for (int oc = 0; oc < C; ++oc)
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[oc] = fmaf(nb[k], w[w2 + (oc * C + ic) * 9 + k], acc[oc]);
    }
#pragma unroll
    for (int oc = 0; oc < C; ++oc) sB[oc * 256 + tid] = relu(acc[oc]);
  }
  __syncthreads();
  {
    constexpr int OPT = C / 4;            // output channels per thread
    const int p = tid & 63, og = tid >> 6;
    const int py = p >> 3, px = p & 7;
    float acc[OPT];
#pragma unroll
    for (int o = 0; o < OPT; ++o) acc[o] = w[b3 + og * OPT + o];
    for (int ic = 0; ic < C; ++ic) {
      float in[4];
#pragma unroll
      for (int ky = 0; ky < 2; ++ky)
#pragma unroll
        for (int kx = 0; kx < 2; ++kx) in[ky * 2 + kx] = sB[ic * 256 + (2 * py + ky) * 16 + 2 * px + kx];
#pragma unroll
      for (int o = 0; o < OPT; ++o)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          acc[o] = fmaf(in[k], w[w3 + ((og * OPT + o) * C + ic) * 4 + k], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < OPT; ++o) orow[(og * OPT + o) * 64 + p] = relu(acc[o]);
  }
  __syncthreads();   // sA / sB reused by the next stack
}

// one workgroup per window; offsets < 0 = modality absent
__global__ __launch_bounds__(256) void hsr_fuse_k(const float* __restrict__ r, const float* __restrict__ d,
                                                  const float* __restrict__ t, const float* __restrict__ m,
                                                  const float* __restrict__ w, float* __restrict__ out,
                                                  int ld_out, int off_r, int off_d, int off_t, int off_m) {
  __shared__ float sA[16 * 256], sB[16 * 256], sM[16];
  const int tid = threadIdx.x;
  const size_t win = blockIdx.x;
  float* orow = out + win * (size_t)ld_out;
  if (off_r >= 0)
    image_stack<3, 16>(r + win * 3072, w, W1R, B1R, W2R, B2R, W3R, B3R, sA, sB, orow + off_r, tid);
  if (off_d >= 0)
    image_stack<1, 8>(d + win * 1024, w, W1D, B1D, W2D, B2D, W3D, B3D, sA, sB, orow + off_d, tid);
  if (off_t >= 0 && tid < 64) orow[off_t + tid] = t[win];   // t[i].repeat(1,1,8,8)
  if (off_m >= 0) {
    // conv1l over 13 MFCCs: 8 channels x 2 positions (input index 9*pos + k - 9)
    const float* mw = m + win * 13;
    if (tid < 16) {
      const int oc = tid >> 1, pos = tid & 1;
      float acc = w[B1L + oc];
#pragma unroll
      for (int k = 0; k < 18; ++k) {
        const int idx = 9 * pos + k - 9;
        const float v = (idx >= 0 && idx < 13) ? mw[idx] : 0.f;
        acc = fmaf(v, w[W1L + oc * 18 + k], acc);
      }
      sM[oc * 2 + pos] = relu(acc);
    }
    __syncthreads();
    // conv2l: 16 channels x 1 position; view(-1,2,8,1).repeat(1,1,1,8):
    // channel oc fills columns oc*8 .. oc*8+7 of the mic block
    if (tid < 128) {
      const int oc = tid >> 3;
      float acc = w[B2L + oc];
#pragma unroll
      for (int ic = 0; ic < 8; ++ic)
#pragma unroll
        for (int k = 0; k < 2; ++k) acc = fmaf(sM[ic * 2 + k], w[W2L + (oc * 8 + ic) * 2 + k], acc);
      orow[off_m + tid] = relu(acc);
    }
  }
}
}  // namespace

int mmad_hsr_weight_count(void) { return NWEIGHTS; }

int mmad_hsr_fuse(int n, const float* r, const float* d, const float* t, const float* m,
                  const float* weights, int unimodal, float* out, int ld_out, void* stream) {
  MMAD_CHECK_ARG(n >= 0, "hsr_fuse: n must be >= 0 (n=%d)", n);
  MMAD_CHECK_ARG(weights && out, "hsr_fuse: null weights / out");
  int off_r = -1, off_d = -1, off_t = -1, off_m = -1, width;
  if (unimodal) {
    // the reference keeps the last modality it computed (:190-221); the
    // product computes only that one
    if (m) { off_m = 0; width = 128; }
    else if (t) { off_t = 0; width = 64; }
    else if (d) { off_d = 0; width = 512; }
    else if (r) { off_r = 0; width = 1024; }
    else { mmad_set_error("hsr_fuse: unimodal needs one modality"); return MMAD_EINVAL; }
  } else {
    MMAD_CHECK_ARG(r && d && t && m, "hsr_fuse: the fused row needs r, d, t and m (data_loaders.py:224)");
    off_r = 0; off_d = 1024; off_t = 1536; off_m = 1600; width = 1728;
  }
  MMAD_CHECK_ARG(ld_out >= width, "hsr_fuse: ld_out %d < row width %d", ld_out, width);
  if (n == 0) return MMAD_OK;
  hsr_fuse_k<<<n, 256, 0, (hipStream_t)stream>>>(r, d, t, m, weights, out, ld_out, off_r, off_d, off_t, off_m);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

// ---- sensor-stream normalisation (TabularDataset, utils/data_loaders.py) ---
// norm_vec_np (:447-456): per column (v - min) / (max - min) over the n
// windows, NaN -> 0 (a constant column); the reference computes it in fp64
// (its uint8 / uint16 image arrays subtract exactly, the quotient is a
// float64 division), then casts to fp32 (:367-394).  Images additionally
// take the reference's view + F.interpolate(size=32) (nearest, 24 -> 32 rows:
// src row = floor(y * 24 / 32), columns unchanged): out [n][C][32][32] from
// the HWC-flattened [24][32][C] row reinterpreted as [C][24][32] (:368-378).
namespace {

constexpr int NORM_ROWS = 1024;    // rows per min/max partial

template <typename V> __device__ __forceinline__ double ldv(const void* v, int64_t i) {
  return (double)((const V*)v)[i];
}
__device__ __forceinline__ double load_any(const void* v, int vtype, int64_t i) {
  switch (vtype) {
    case MMAD_SRC_U8: return ldv<uint8_t>(v, i);
    case MMAD_SRC_U16: return ldv<uint16_t>(v, i);
    case MMAD_SRC_I32: return ldv<int32_t>(v, i);
    case MMAD_SRC_F32: return ldv<float>(v, i);
    default: return ldv<double>(v, i);
  }
}

__global__ __launch_bounds__(256) void colminmax_k(int64_t n, int F, const void* __restrict__ v,
                                                   int vtype, double* __restrict__ part) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= F) return;
  const int64_t r0 = (int64_t)blockIdx.y * NORM_ROWS;
  const int64_t r1 = r0 + NORM_ROWS < n ? r0 + NORM_ROWS : n;
  double lo = load_any(v, vtype, r0 * F + f), hi = lo;
  for (int64_t r = r0 + 1; r < r1; ++r) {
    const double x = load_any(v, vtype, r * F + f);
    lo = x < lo ? x : lo;
    hi = x > hi ? x : hi;
  }
  part[((int64_t)blockIdx.y * 2 + 0) * F + f] = lo;
  part[((int64_t)blockIdx.y * 2 + 1) * F + f] = hi;
}

__global__ __launch_bounds__(256) void colrange_k(int F, int nparts, double* __restrict__ part) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= F) return;
  double lo = part[f], hi = part[F + f];
  for (int p = 1; p < nparts; ++p) {
    const double a = part[((int64_t)p * 2 + 0) * F + f], b = part[((int64_t)p * 2 + 1) * F + f];
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  part[f] = lo;
  part[F + f] = hi;
}

// one thread per OUTPUT element
__global__ __launch_bounds__(256) void minmax_apply_k(int64_t n, int F, const void* __restrict__ v,
                                                      int vtype, const double* __restrict__ range,
                                                      int layout, int64_t out_row,
                                                      float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * out_row) return;
  const int64_t row = e / out_row;
  const int o = (int)(e - row * out_row);
  int f = o;
  if (layout == MMAD_NORM_IMG24) {
    const int c = o >> 10, y = (o >> 5) & 31, x = o & 31;
    f = c * 768 + ((y * 24) >> 5) * 32 + x;
  }
  const double lo = range[f], span = range[F + f] - lo;
  const double q = (load_any(v, vtype, row * F + f) - lo) / span;
  out[e] = q == q ? (float)q : 0.f;   // 0/0 (constant column) -> 0
}

}  // namespace

size_t mmad_minmax_norm_ws_bytes(int64_t n, int F) {
  if (n < 1 || F < 1) return 0;
  return (size_t)((n + NORM_ROWS - 1) / NORM_ROWS) * 2 * F * sizeof(double);
}

int mmad_minmax_norm(int64_t n, int F, const void* v, int vtype, int layout, float* out, void* ws,
                     size_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(n >= 1 && F >= 1 && v && out && ws, "minmax_norm: bad arguments (n=%lld F=%d)",
                 (long long)n, F);
  MMAD_CHECK_ARG(vtype >= MMAD_SRC_F64 && vtype <= MMAD_SRC_F32, "minmax_norm: unknown source type %d",
                 vtype);
  MMAD_CHECK_ARG(layout == MMAD_NORM_FLAT || (layout == MMAD_NORM_IMG24 && F % 768 == 0),
                 "minmax_norm: layout %d does not fit F=%d", layout, F);
  MMAD_CHECK_ARG(ws_bytes >= mmad_minmax_norm_ws_bytes(n, F), "minmax_norm: workspace too small");
  MMAD_CHECK_ARG(n / NORM_ROWS < 65535, "minmax_norm: n=%lld too large", (long long)n);
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)ws;
  const int nparts = (int)((n + NORM_ROWS - 1) / NORM_ROWS);
  colminmax_k<<<dim3((F + 255) / 256, nparts), 256, 0, s>>>(n, F, v, vtype, part);
  MMAD_LAUNCH_CHECK();
  colrange_k<<<(F + 255) / 256, 256, 0, s>>>(F, nparts, part);
  MMAD_LAUNCH_CHECK();
  const int64_t out_row = layout == MMAD_NORM_IMG24 ? (int64_t)(F / 768) * 1024 : F;
  const int64_t total = n * out_row;
  minmax_apply_k<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(n, F, v, vtype, part, layout, out_row,
                                                                  out);
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}
