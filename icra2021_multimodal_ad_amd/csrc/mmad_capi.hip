// C-ABI entry points: layer operators and the whole-autoencoder executor.
//
// The executor replaces the reference's per-op Python dispatch of
// AutoEncoder.step / validate / forward (models/auto_encoder.py:36-91) and
// get_diffs (reconstruction_aggregation.py:6-37): one host call enqueues the
// whole fwd+bwd (or scoring) sequence on one HIP stream, no host syncs, no
// allocation (caller-provided workspace).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mmad_common.h"
#include "mmad_gemm.h"
#include "mmad_ops.h"

static thread_local char g_err[512] = "";

void mmad_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

const char* mmad_last_error_string(void) { return g_err; }
int mmad_abi_version(void) { return MMAD_ABI_VERSION; }
int mmad_pad_granule(void) { return MMAD_PAD; }

int mmad_tile_override() {
  static int v = [] {
    const char* e = getenv("MMAD_GEMM_TILE");
    return e ? atoi(e) : -1;
  }();
  return v;
}

#define RET_IF(x)              \
  do {                         \
    int r_ = (x);              \
    if (r_ != MMAD_OK) return r_; \
  } while (0)

static int check_dims(const char* who, int M, int N, int K, int Mp, int Np, int Kp) {
  MMAD_CHECK_ARG(Mp % MMAD_PAD == 0 && Np % MMAD_PAD == 0 && Kp % MMAD_PAD == 0,
                 "%s: padded dims must be multiples of %d (Mp=%d Np=%d Kp=%d)", who, MMAD_PAD, Mp,
                 Np, Kp);
  MMAD_CHECK_ARG(M >= 1 && N >= 1 && K >= 1 && M <= Mp && N <= Np && K <= Kp,
                 "%s: valid dims out of range (M=%d N=%d K=%d Mp=%d Np=%d Kp=%d)", who, M, N, K,
                 Mp, Np, Kp);
  return MMAD_OK;
}
static int check_dtype(int dtype) {
  MMAD_CHECK_ARG(dtype == MMAD_F32 || dtype == MMAD_BF16, "bad dtype %d", dtype);
  return MMAD_OK;
}

// ---------------------------------------------------------------------------
// layer operators
// ---------------------------------------------------------------------------
int mmad_fc_fwd(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                const void* w, const float* bias, int act, float slope, const float* bn_scale,
                const float* bn_shift, void* y, float* stats, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_fwd", M, N, K, Mp, Np, Kp));
  MMAD_CHECK_ARG(x && w && y, "fc_fwd: null operand");
  MMAD_CHECK_ARG((bn_scale == nullptr) == (bn_shift == nullptr), "fc_fwd: bn_scale/shift pair");
  GemmEpi ep{};
  ep.M = M; ep.N = N; ep.out = y; ep.ldo = Np; ep.bias = bias; ep.act = act; ep.slope = slope;
  ep.bn_scale = bn_scale; ep.bn_shift = bn_shift; ep.part = stats; ep.ldpart = Np;
  return mmad_gemm_dispatch(dtype, GEMM_EPI_FWD, x, Kp, w, Kp, Mp, Np, Kp, ep, (hipStream_t)stream);
}

static int fc_fwd_mse_impl(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                           const void* w, const float* bias, const float* target, int ld_target,
                           int tmod, float grad_scale, void* dz, float* partials, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_fwd_mse", M, N, K, Mp, Np, Kp));
  MMAD_CHECK_ARG(x && w && dz && target && ld_target >= N, "fc_fwd_mse: bad operands");
  GemmEpi ep{};
  ep.M = M; ep.N = N; ep.out = dz; ep.ldo = Np; ep.bias = bias; ep.part = partials;
  ep.ldpart = Np; ep.target = target; ep.ldt = ld_target; ep.tmod = tmod; ep.gscale = grad_scale;
  return mmad_gemm_dispatch(dtype, GEMM_EPI_MSE, x, Kp, w, Kp, Mp, Np, Kp, ep, (hipStream_t)stream);
}

int mmad_fc_fwd_mse(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                    const void* w, const float* bias, const float* target, int ld_target,
                    float grad_scale, void* dz, float* partials, void* stream) {
  return fc_fwd_mse_impl(dtype, M, N, K, Mp, Np, Kp, x, w, bias, target, ld_target, M, grad_scale,
                         dz, partials, stream);
}

int mmad_fc_fwd_score(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                      const void* w, const float* bias, int act, float slope,
                      const float* bn_scale, const float* bn_shift, void* y, const void* ref,
                      float* rowsq, float* diff, int ld_diff, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_fwd_score", M, N, K, Mp, Np, Kp));
  MMAD_CHECK_ARG(x && w && y && ref && rowsq, "fc_fwd_score: null operand");
  MMAD_CHECK_ARG(!diff || ld_diff >= N, "fc_fwd_score: ld_diff < N");
  GemmEpi ep{};
  ep.M = M; ep.N = N; ep.out = y; ep.ldo = Np; ep.bias = bias; ep.act = act; ep.slope = slope;
  ep.bn_scale = bn_scale; ep.bn_shift = bn_shift; ep.ref = ref; ep.ldref = Np; ep.rowsq = rowsq;
  ep.ldrow = Mp; ep.diff = diff; ep.lddiff = ld_diff;
  return mmad_gemm_dispatch(dtype, GEMM_EPI_SCORE, x, Kp, w, Kp, Mp, Np, Kp, ep,
                            (hipStream_t)stream);
}

int mmad_fc_bwd_data(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* dz,
                     const void* w, void* dx, float* colsum, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_bwd_data", M, N, K, Mp, Np, Kp));
  MMAD_CHECK_ARG(dz && w && dx, "fc_bwd_data: null operand");
  GemmEpi ep{};
  ep.M = M; ep.N = K; ep.out = dx; ep.ldo = Kp; ep.part = colsum; ep.ldpart = Kp;
  // dx[Mp][Kp] = dz[Mp][Np] . W[Np][Kp]: contraction over Np, W read MN-major
  return mmad_gemm_dispatch(dtype, GEMM_EPI_BWD_DATA, dz, Np, w, Kp, Mp, Kp, Np, ep,
                            (hipStream_t)stream);
}

int mmad_fc_bwd_weight(int dtype, int Mp, int Np, int Kp, const void* dz, const void* x,
                       float* dw, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_bwd_weight", Mp, Np, Kp, Mp, Np, Kp));
  MMAD_CHECK_ARG(dz && x && dw, "fc_bwd_weight: null operand");
  GemmEpi ep{};
  ep.M = Np; ep.N = Kp; ep.out = dw; ep.ldo = Kp;
  // dW[Np][Kp] = dz^T . x, contraction over the batch; both read MN-major
  return mmad_gemm_dispatch(dtype, GEMM_EPI_BWD_WEIGHT, dz, Np, x, Kp, Np, Kp, Mp, ep,
                            (hipStream_t)stream);
}

// ---------------------------------------------------------------------------
// whole-autoencoder executor
// ---------------------------------------------------------------------------
struct AeLayer {
  int K, N, Kp, Np;
  int act, bn, enc;
  int64_t w_off, b_off, g_off, be_off, bn_off;
};

struct mmad_ae {
  int dtype, n_enc, n_dec, vib, btl;
  float slope, bn_eps, bn_mom;
  std::vector<AeLayer> L;
  int64_t n_params, n_weight, n_bn;
  float *params = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr, *running = nullptr;
  void* shadow = nullptr;
};

struct LayerWS {
  void *out, *y, *dy, *dz;
  float *stats, *mean, *rstd, *bnws, *dbpart, *scale, *shift, *rowsq;
};
struct AeWS {
  int B, k, Mpe, Mpd;
  void *xin, *zbuf, *dzin;
  float *eps, *klpart, *misc;
  int64_t kl_parts;
  std::vector<LayerWS> l;
  int64_t bytes;
};

static size_t esz(int dtype) { return dtype == MMAD_BF16 ? 2 : 4; }

// Carve the workspace (base may be null to size it).  Every buffer is
// 256-byte aligned.
static void carve(const mmad_ae* h, int B, int k, char* base, AeWS& w) {
  int64_t off = 0;
  auto take = [&](int64_t bytes) -> char* {
    off = (off + 255) / 256 * 256;
    char* p = base ? base + off : nullptr;
    off += bytes;
    return p;
  };
  const size_t es = esz(h->dtype);
  w.B = B;
  w.k = k;
  w.Mpe = mmad_roundup(B, MMAD_PAD);
  w.Mpd = mmad_roundup(B * k, MMAD_PAD);
  const int nL = (int)h->L.size();
  w.xin = take((int64_t)w.Mpe * h->L[0].Kp * es);
  w.zbuf = w.dzin = nullptr;
  w.eps = w.klpart = nullptr;
  w.kl_parts = 0;
  if (h->vib) {
    const AeLayer& d0 = h->L[h->n_enc];
    w.zbuf = take((int64_t)w.Mpd * d0.Kp * es);
    w.dzin = take((int64_t)w.Mpd * d0.Kp * es);
    w.eps = (float*)take((int64_t)k * B * h->btl * 4);
    w.kl_parts = mmad_vib_kl_parts(B, k, d0.Kp);
    w.klpart = (float*)take(w.kl_parts * 4);
  }
  w.misc = (float*)take(1024 * 4);
  w.l.resize(nL);
  for (int i = 0; i < nL; ++i) {
    const AeLayer& a = h->L[i];
    const int Mp = a.enc ? w.Mpe : w.Mpd;
    const int64_t mat = (int64_t)Mp * a.Np * es;
    LayerWS& s = w.l[i];
    s.out = take(mat);
    s.y = a.bn ? take(mat) : nullptr;
    s.dy = take(mat);
    s.dz = a.bn ? take(mat) : nullptr;
    s.stats = (float*)take((int64_t)(Mp / MMAD_PART_ROWS) * 2 * a.Np * 4);
    s.mean = (float*)take(a.Np * 4);
    s.rstd = (float*)take(a.Np * 4);
    s.bnws = (float*)take((int64_t)mmad_bn_act_bwd_ws(Mp, a.Np));
    s.dbpart = (float*)take((int64_t)(Mp / 128) * a.Np * 4);
    s.scale = (float*)take(a.Np * 4);
    s.shift = (float*)take(a.Np * 4);
    s.rowsq = (float*)take((int64_t)(a.Np / 128) * Mp * 4);
  }
  w.bytes = (off + 255) / 256 * 256;
}

int mmad_ae_create(mmad_ae** out, int dtype, int n_enc, const int* enc_widths, int n_dec,
                   const int* dec_widths, int vib, float slope, float bn_eps, float bn_momentum) {
  MMAD_CHECK_ARG(out != nullptr, "ae_create: null out");
  *out = nullptr;
  RET_IF(check_dtype(dtype));
  MMAD_CHECK_ARG(n_enc >= 1 && n_dec >= 1 && enc_widths && dec_widths, "ae_create: bad layers");
  for (int i = 0; i <= n_enc; ++i) MMAD_CHECK_ARG(enc_widths[i] >= 1, "ae_create: bad enc width");
  for (int i = 0; i <= n_dec; ++i) MMAD_CHECK_ARG(dec_widths[i] >= 1, "ae_create: bad dec width");
  MMAD_CHECK_ARG(dec_widths[n_dec] == enc_widths[0], "ae_create: decoder must reconstruct input");
  if (vib)
    MMAD_CHECK_ARG(enc_widths[n_enc] == 2 * dec_widths[0],
                   "ae_create: VIB encoder output must be 2*btl");
  else
    MMAD_CHECK_ARG(enc_widths[n_enc] == dec_widths[0], "ae_create: bottleneck mismatch");
  mmad_ae* h = new mmad_ae();
  h->dtype = dtype;
  h->n_enc = n_enc;
  h->n_dec = n_dec;
  h->vib = vib;
  h->btl = dec_widths[0];
  h->slope = slope;
  h->bn_eps = bn_eps;
  h->bn_mom = bn_momentum;
  for (int side = 0; side < 2; ++side) {
    const int n = side == 0 ? n_enc : n_dec;
    const int* wd = side == 0 ? enc_widths : dec_widths;
    for (int i = 0; i < n; ++i) {
      AeLayer a{};
      a.K = wd[i];
      a.N = wd[i + 1];
      a.Kp = mmad_roundup(a.K, MMAD_PAD);
      a.Np = mmad_roundup(a.N, MMAD_PAD);
      a.bn = i < n - 1;
      a.act = a.bn ? MMAD_ACT_LEAKYRELU : MMAD_ACT_NONE;
      a.enc = side == 0;
      h->L.push_back(a);
    }
  }
  int64_t off = 0;
  for (auto& a : h->L) { a.w_off = off; off += (int64_t)a.Np * a.Kp; }
  h->n_weight = off;
  int64_t bn = 0;
  for (auto& a : h->L) {
    a.b_off = off; off += a.Np;
    a.g_off = a.be_off = a.bn_off = -1;
    if (a.bn) {
      a.g_off = off; off += a.Np;
      a.be_off = off; off += a.Np;
      a.bn_off = bn; bn += a.Np;
    }
  }
  h->n_params = off;
  h->n_bn = bn;
  *out = h;
  return MMAD_OK;
}

void mmad_ae_destroy(mmad_ae* h) { delete h; }

int mmad_ae_layout(const mmad_ae* h, int64_t* info, int64_t* totals) {
  MMAD_CHECK_ARG(h && info && totals, "ae_layout: null arg");
  for (size_t i = 0; i < h->L.size(); ++i) {
    const AeLayer& a = h->L[i];
    int64_t* r = info + 7 * i;
    r[0] = a.w_off; r[1] = a.b_off; r[2] = a.g_off; r[3] = a.be_off;
    r[4] = a.Kp; r[5] = a.Np; r[6] = a.bn_off;
  }
  totals[0] = h->n_params;
  totals[1] = h->n_weight;
  totals[2] = h->n_bn;
  totals[3] = (int64_t)h->L.size();
  return MMAD_OK;
}

int64_t mmad_ae_workspace_bytes(const mmad_ae* h, int B, int k) {
  if (!h || B < 1 || k < 1) return -1;
  AeWS w;
  carve(h, B, k, nullptr, w);
  return w.bytes;
}

int mmad_ae_bind(mmad_ae* h, float* params, float* grads, float* adam_m, float* adam_v,
                 void* shadow, float* running) {
  MMAD_CHECK_ARG(h && params, "ae_bind: null params");
  MMAD_CHECK_ARG(h->dtype != MMAD_BF16 || shadow, "ae_bind: bf16 needs a shadow buffer");
  h->params = params;
  h->grads = grads;
  h->m = adam_m;
  h->v = adam_v;
  h->shadow = shadow;
  h->running = running;
  return MMAD_OK;
}

int mmad_ae_sync_shadow(mmad_ae* h, void* stream) {
  MMAD_CHECK_ARG(h && h->params, "ae_sync_shadow: unbound");
  if (h->dtype != MMAD_BF16) return MMAD_OK;
  return mmad_to_bf16(h->n_weight, h->params, h->shadow, stream);
}

static const void* weights(const mmad_ae* h, const AeLayer& a) {
  if (h->dtype == MMAD_BF16) return (const char*)h->shadow + a.w_off * 2;
  return h->params + a.w_off;
}

static const void* input_of(const mmad_ae* h, const AeWS& w, int l) {
  if (l == 0) return w.xin;
  if (h->vib && l == h->n_enc) return w.zbuf;
  const AeLayer& p = h->L[l - 1];
  return p.bn ? w.l[l - 1].y : w.l[l - 1].out;
}

static int prepare_ws(const mmad_ae* h, int B, int k, void* ws, int64_t ws_bytes, AeWS& w) {
  MMAD_CHECK_ARG(B >= 1 && k >= 1, "bad batch B=%d k=%d", B, k);
  MMAD_CHECK_ARG(h->vib || k == 1, "k>1 needs the VIB head");
  carve(h, B, k, (char*)ws, w);
  MMAD_CHECK_ARG(ws && ws_bytes >= w.bytes, "workspace too small (%lld < %lld bytes)",
                 (long long)ws_bytes, (long long)w.bytes);
  MMAD_CHECK_ARG(((uintptr_t)ws) % 256 == 0, "workspace must be 256-byte aligned");
  return MMAD_OK;
}

static inline int rows_of(const mmad_ae* h, const AeWS& w, const AeLayer& a) {
  return a.enc ? w.B : w.B * w.k;
}
static inline int prows_of(const AeWS& w, const AeLayer& a) { return a.enc ? w.Mpe : w.Mpd; }

static float* running_mean(const mmad_ae* h, const AeLayer& a) { return h->running + a.bn_off; }
static float* running_var(const mmad_ae* h, const AeLayer& a) {
  return h->running + h->n_bn + a.bn_off;
}

// forward pass through every layer; mode 0 = train (batch-stat BN, MSE-fused
// last layer), 1 = eval (running-stat affine), 2 = train-BN forward only
static int run_forward(mmad_ae* h, AeWS& w, const float* x, int ld_x, int mode, const float* eps,
                       uint64_t seed, uint64_t offset, void* stream) {
  const int dt = h->dtype;
  const int nL = (int)h->L.size();
  const int B = w.B, k = w.k;
  RET_IF(mmad_pack_input(dt, B, h->L[0].K, w.Mpe, h->L[0].Kp, x, ld_x, w.xin, stream));
  for (int l = 0; l < nL; ++l) {
    const AeLayer& a = h->L[l];
    LayerWS& s = w.l[l];
    const int M = rows_of(h, w, a), Mp = prows_of(w, a);
    const void* in = input_of(h, w, l);
    const void* wt = weights(h, a);
    const float* b = h->params + a.b_off;
    if (mode == 0 && l == nL - 1) {
      RET_IF(fc_fwd_mse_impl(dt, M, a.N, a.K, Mp, a.Np, a.Kp, in, wt, b, x, ld_x, B,
                             2.0f / (float)k, s.out, s.stats, stream));
    } else if (a.bn && mode != 1) {
      RET_IF(mmad_fc_fwd(dt, M, a.N, a.K, Mp, a.Np, a.Kp, in, wt, b, a.act, h->slope, nullptr,
                         nullptr, s.out, s.stats, stream));
      RET_IF(mmad_bn_train_apply(dt, M, a.N, Mp, a.Np, s.out, s.stats, h->params + a.g_off,
                                 h->params + a.be_off, running_mean(h, a), running_var(h, a),
                                 h->bn_mom, h->bn_eps, s.mean, s.rstd, s.y, stream));
    } else if (a.bn) {
      RET_IF(mmad_bn_eval_affine(a.N, a.Np, h->params + a.g_off, h->params + a.be_off,
                                 running_mean(h, a), running_var(h, a), h->bn_eps, s.scale,
                                 s.shift, stream));
      RET_IF(mmad_fc_fwd(dt, M, a.N, a.K, Mp, a.Np, a.Kp, in, wt, b, a.act, h->slope, s.scale,
                         s.shift, s.y, nullptr, stream));
    } else {
      RET_IF(mmad_fc_fwd(dt, M, a.N, a.K, Mp, a.Np, a.Kp, in, wt, b, a.act, h->slope, nullptr,
                         nullptr, s.out, nullptr, stream));
    }
    if (h->vib && l == h->n_enc - 1) {
      const AeLayer& d0 = h->L[h->n_enc];
      RET_IF(mmad_vib_reparam_fwd(dt, B, h->btl, k, s.out, a.Np, eps, w.eps, seed, offset,
                                  mode == 1 ? 1 : 0, w.zbuf, d0.Kp,
                                  mode == 0 ? w.klpart : nullptr, stream));
    }
  }
  return MMAD_OK;
}

// backward through every layer.  from_mse: the last layer's dz and bias
// partials come from the MSE-fused forward epilogue; otherwise the caller has
// packed dL/dx_hat into the last layer's dy buffer.
static int run_backward(mmad_ae* h, AeWS& w, int from_mse, float beta_kl, void* stream) {
  const int dt = h->dtype;
  const int nL = (int)h->L.size();
  for (int l = nL - 1; l >= 0; --l) {
    const AeLayer& a = h->L[l];
    LayerWS& s = w.l[l];
    const int Mp = prows_of(w, a);
    const void* dz = (l == nL - 1) ? (from_mse ? s.out : s.dy) : (a.bn ? s.dz : s.dy);
    const void* in = input_of(h, w, l);
    RET_IF(mmad_fc_bwd_weight(dt, Mp, a.Np, a.Kp, dz, in, h->grads + a.w_off, stream));
    float* gb = h->grads + a.b_off;
    if (l == nL - 1 && from_mse) {
      RET_IF(mmad_colsum(Mp / MMAD_PART_ROWS, a.N, a.Np, s.stats, 2 * a.Np, 1.f, gb, stream));
    } else if (l == nL - 1 || a.bn || (h->vib && l == h->n_enc - 1)) {
      RET_IF(mmad_colsum(Mp / 128, a.N, a.Np, s.dbpart, a.Np, 1.f, gb, stream));
    } else {
      RET_IF(mmad_colsum(Mp / MMAD_PART_ROWS, a.N, a.Np, s.stats, 2 * a.Np, 1.f, gb, stream));
    }
    if (l == 0) break;
    const AeLayer& p = h->L[l - 1];
    LayerWS& ps = w.l[l - 1];
    const int M = rows_of(h, w, a);
    const int Mpp = prows_of(w, p);
    if (h->vib && l == h->n_enc) {
      RET_IF(mmad_fc_bwd_data(dt, M, a.N, a.K, Mp, a.Np, a.Kp, dz, weights(h, a), w.dzin, nullptr,
                              stream));
      RET_IF(mmad_vib_reparam_bwd(dt, w.B, h->btl, w.k, ps.out, p.Np, w.eps, w.dzin, a.Kp, beta_kl,
                                  ps.dy, p.Np, ps.dbpart, stream));
    } else if (p.bn) {
      RET_IF(mmad_fc_bwd_data(dt, M, a.N, a.K, Mp, a.Np, a.Kp, dz, weights(h, a), ps.dy, nullptr,
                              stream));
      RET_IF(mmad_bn_act_bwd(dt, p.act, h->slope, rows_of(h, w, p), p.N, Mpp, p.Np, ps.dy, ps.out,
                             ps.mean, ps.rstd, h->params + p.g_off, ps.dz, h->grads + p.g_off,
                             h->grads + p.be_off, ps.dbpart, ps.bnws, stream));
    } else {
      RET_IF(mmad_fc_bwd_data(dt, M, a.N, a.K, Mp, a.Np, a.Kp, dz, weights(h, a), ps.dy, ps.stats,
                              stream));
    }
  }
  return MMAD_OK;
}

int mmad_ae_train_fwd_bwd(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                          uint64_t seed, uint64_t offset, float beta_kl, float* loss_out,
                          void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->running, "ae_train: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && loss_out, "ae_train: bad input");
  AeWS w;
  RET_IF(prepare_ws(h, B, k, ws, ws_bytes, w));
  RET_IF(run_forward(h, w, x, ld_x, 0, eps, seed, offset, stream));
  RET_IF(run_backward(h, w, 1, beta_kl, stream));
  // loss = sum d^2 / k (+ beta * KL)
  const int nL = (int)h->L.size();
  const AeLayer& last = h->L[nL - 1];
  RET_IF(mmad_sum2d(w.Mpd / MMAD_PART_ROWS, last.N, w.l[nL - 1].stats + last.Np, 2 * last.Np,
                    1.f / (float)w.k, loss_out, 0, stream));
  if (h->vib) RET_IF(mmad_sum(w.kl_parts, w.klpart, beta_kl, loss_out, 1, stream));
  return MMAD_OK;
}

int mmad_ae_backward(mmad_ae* h, const float* dxhat, int ld, int B, void* ws, int64_t ws_bytes,
                     void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads, "ae_backward: unbound handle");
  MMAD_CHECK_ARG(!h->vib, "ae_backward: the VIB model trains through mmad_ae_train_fwd_bwd");
  AeWS w;
  RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w));
  const int nL = (int)h->L.size();
  const AeLayer& last = h->L[nL - 1];
  LayerWS& s = w.l[nL - 1];
  MMAD_CHECK_ARG(dxhat && ld >= last.N, "ae_backward: bad dxhat");
  RET_IF(mmad_pack_input(h->dtype, B, last.N, w.Mpd, last.Np, dxhat, ld, s.dy, stream));
  RET_IF(mmad_matrix_colsum_partials(h->dtype, B, w.Mpd, last.Np, s.dy, s.dbpart, stream));
  return run_backward(h, w, 0, 0.f, stream);
}

int mmad_ae_adam(mmad_ae* h, float lr, float beta1, float beta2, float eps, int step,
                 void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->m && h->v, "ae_adam: unbound handle");
  MMAD_CHECK_ARG(step >= 1, "ae_adam: step must be >= 1");
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  return mmad_adam(h->n_params, h->params, h->grads, h->m, h->v, beta1, beta2, eps,
                   (float)(lr / bc1), (float)sqrt(bc2), h->dtype == MMAD_BF16 ? h->shadow : nullptr,
                   h->dtype == MMAD_BF16 ? h->n_weight : 0, stream);
}

int mmad_ae_forward(mmad_ae* h, const float* x, int ld_x, int B, int train_bn, float* x_hat,
                    int ld_out, float* loss_out, void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->running, "ae_forward: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K, "ae_forward: bad input");
  AeWS w;
  RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w));
  RET_IF(run_forward(h, w, x, ld_x, train_bn ? 2 : 1, nullptr, 0x5eed, 0, stream));
  const AeLayer& last = h->L.back();
  const void* xh = w.l.back().out;
  if (x_hat) RET_IF(mmad_unpack_output(h->dtype, B, last.N, last.Np, xh, x_hat, ld_out, stream));
  if (loss_out) {
    RET_IF(mmad_sse_partials(h->dtype, B, last.N, last.Np, xh, x, ld_x, w.misc, 256, stream));
    RET_IF(mmad_sum(256, w.misc, 1.f, loss_out, 0, stream));
  }
  return MMAD_OK;
}

int mmad_ae_score(mmad_ae* h, const float* x, int ld_x, int B, float* layer_sq, float* diffs,
                  void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->running, "ae_score: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && layer_sq, "ae_score: bad args");
  AeWS w;
  RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w));
  const int dt = h->dtype;
  const int nL = (int)h->L.size();
  // pass 1: full eval forward except the last layer, which scores d0 = x_hat - x
  RET_IF(mmad_pack_input(dt, B, h->L[0].K, w.Mpe, h->L[0].Kp, x, ld_x, w.xin, stream));
  int ld_diff = h->L[0].K;
  for (int e = 0; e < h->n_enc; ++e) ld_diff += h->L[e].N;
  for (int l = 0; l < nL; ++l) {
    const AeLayer& a = h->L[l];
    LayerWS& s = w.l[l];
    const int M = rows_of(h, w, a), Mp = prows_of(w, a);
    const void* in = input_of(h, w, l);
    const float* sc = nullptr;
    const float* sh = nullptr;
    if (a.bn) {
      RET_IF(mmad_bn_eval_affine(a.N, a.Np, h->params + a.g_off, h->params + a.be_off,
                                 running_mean(h, a), running_var(h, a), h->bn_eps, s.scale,
                                 s.shift, stream));
      sc = s.scale;
      sh = s.shift;
    }
    void* out = a.bn ? s.y : s.out;
    if (l == nL - 1) {
      RET_IF(mmad_fc_fwd_score(dt, M, a.N, a.K, Mp, a.Np, a.Kp, in, weights(h, a),
                               h->params + a.b_off, a.act, h->slope, sc, sh, out, w.xin, s.rowsq,
                               diffs, ld_diff, stream));
    } else {
      RET_IF(mmad_fc_fwd(dt, M, a.N, a.K, Mp, a.Np, a.Kp, in, weights(h, a), h->params + a.b_off,
                         a.act, h->slope, sc, sh, out, nullptr, stream));
    }
    if (h->vib && l == h->n_enc - 1) {
      RET_IF(mmad_vib_reparam_fwd(dt, B, h->btl, 1, s.out, a.Np, nullptr, nullptr, 0, 0, 1, w.zbuf,
                                  h->L[h->n_enc].Kp, nullptr, stream));
    }
  }
  // pass 2: x_hat through the encoder, diff against pass-1 activations
  const void* cur = w.l[nL - 1].out;
  int coff = h->L[0].K;
  for (int e = 0; e < h->n_enc; ++e) {
    const AeLayer& a = h->L[e];
    LayerWS& s = w.l[e];
    const void* ref = a.bn ? s.y : s.out;
    RET_IF(mmad_fc_fwd_score(dt, B, a.N, a.K, w.Mpe, a.Np, a.Kp, cur, weights(h, a),
                             h->params + a.b_off, a.act, h->slope, a.bn ? s.scale : nullptr,
                             a.bn ? s.shift : nullptr, s.dy, ref, s.rowsq,
                             diffs ? diffs + coff : nullptr, ld_diff, stream));
    coff += a.N;
    cur = s.dy;
  }
  // per-window sums: layer_sq[0] from the decoder's last layer, [1+e] from pass 2
  const AeLayer& last = h->L[nL - 1];
  RET_IF(mmad_colsum(last.Np / 128, B, B, w.l[nL - 1].rowsq, w.Mpd, 1.f, layer_sq, stream));
  for (int e = 0; e < h->n_enc; ++e) {
    const AeLayer& a = h->L[e];
    RET_IF(mmad_colsum(a.Np / 128, B, B, w.l[e].rowsq, w.Mpe, 1.f, layer_sq + (size_t)(e + 1) * B,
                       stream));
  }
  return MMAD_OK;
}
