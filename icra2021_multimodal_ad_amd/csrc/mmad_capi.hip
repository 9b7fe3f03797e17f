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

// Tuning knobs: ONE table, set only through mmad_tune_set (the library reads
// no environment variables, so every rank of a job runs the same schedule
// unless its code says otherwise).  GEMM knobs (0-11) are read per dispatch;
// the executor's schedule knobs (14-31, 33-35) are copied into a handle when it is
// created (mmad_ae_create), so a handle keeps one schedule for its lifetime.
namespace {
int g_knob[MMAD_KNOB_COUNT] = {
    -1,    // 0  GEMM tile override (-1 = autotuned)
    -1,    // 1  XCD tile-group height (-1 = rule)
    1,     // 2  per-shape autotune on first dispatch
    0,     // 3  diagnostics bits (tools/gemm_phase; tests)
    0,     // 4  split-K override (0 = shape rule)
    -2,    // 5  tile of the Adam-fused dW GEMMs (-2 = shape rule, -1 = autotuned)
    -1,    // 6  tile of the bwd-data GEMMs
    -1,    // 7  tile of the forward GEMMs
    0,     // 8  tile of the main-stream Adam-fused dW GEMMs (-2 = rule, -1 = knob 5)
    0,     // 9  split-K override of the dW GEMMs
    0,     // 10 dW split rule: target 64x64-tile blocks (0 = no split)
    8,     // 11 dW split rule: minimum K stages per slice
    0,     // 12 persistent grid for forward-type GEMMs (0 off; else when the tiles exceed one round)
    2,     // 13 BN-backward apply: 128-row slabs per block (1, 2, 4)
    1024,  // 14 DP: per-layer dW fork from this many padded rows (0 = one fork per bucket)
    0,     // 15 side stream behind a CU mask holding this many CUs for the main stream (0 = off)
    -1,    // 16 train-mode BN schedule (-1 = dtype default: bf16 fused, fp32 apply; 0 apply, 1 fold, 2 fused)
    -1,    // 17 backward BN schedule (-1 = the forward's; 2 = fused into the bwd-data GEMMs)
    2048,  // 18 fused BN up to this many padded rows (fold above)
    2,     // 19 dW GEMMs of the last layers run on the main stream
    4096,  // 20 ping-pong weight shadows from this many padded rows
    1,     // 21 main-stream dW GEMMs when ping-ponging
    2,     // 22 record the bwd-data event every n-th side-stream layer
    1,     // 23 reduce the loss on the side stream after the forward
    1,     // 24 DP: exchange the small bucket after the bwd-data GEMM of this layer
    0,     // 25 also materialise dW in the fused step (grads buffer)
    0,     // 26 side stream at the highest priority (schedule sweeps)
    0,     // 27 executor events with the system-scope fence
    1,     // 28 DP: sharded weight buckets (reduce-scatter, Adam on 1/N, all-gather)
    0,     // 29 schedule study: hold every side-stream dW + Adam until the bwd-data chain is enqueued
    8,     // 30 DP: minimum exchange bucket (MiB of fp32 gradient; consecutive layers merge)
    1,     // 31 bwd-data hand-off events completed by the GEMM launch (hipExtLaunchKernel)
    1024,  // 32 fp32 dW split rule from 2048 rows: target 64x64-tile blocks (0 = no split)
    0,     // 33 ping-pong: the top n layers' side dW forks after their bwd-data + apply
    1,     // 34 ping-pong: side dW fork events completed by the launch producing dz
    0,     // 35 ping-pong: side dW forks in pairs from this layer down (0 = every layer)
};
}  // namespace
int mmad_knob(int k) { return g_knob[k]; }
int mmad_tile_override() { return g_knob[0]; }
int mmad_group_override() { return g_knob[1]; }
int mmad_autotune_enabled() { return g_knob[2]; }
int mmad_dbg_override() { return g_knob[3]; }
int mmad_persist_override() { return g_knob[12]; }
int mmad_splitk_override() { return g_knob[4]; }
int mmad_splitk_dw_override() { return g_knob[9]; }
// dW split-K target blocks (0 = no split): 512 paid before the dW loop stopped
// draining its LDS ring every K stage; since then no split measures faster
// (VIB B=4096 0.991-0.996 vs 1.013 ms/step with the split tail off; r02ae_*)
int mmad_splitk_dw_blocks() { return g_knob[10]; }
int mmad_splitk_dw_min_stages() { return g_knob[11]; }
int mmad_splitk_dw_f32_blocks() { return g_knob[32]; }
// tile for the dW GEMMs with the fused Adam epilogue (the autotuner times
// them without Adam, which under-weights the epilogue's HBM traffic: it picks
// 128x128 for the large layers, 208 blocks for 256 CUs).  Default (-2) = a
// shape rule: 128x128 (cfg 0) when the GEMM is deep (K = batch >= 2048) and
// large (>= 1.5 M parameters), 64x64 (cfg 3) otherwise -- B=1024: 64x64
// everywhere (0.522 vs 0.529 ms/step, tools/tile_adam_sweep.py); B=4096:
// 67 vs 87 us at 1658x2048, 63 vs 78 at 1268x1658, 64x64 better below
// (profiles/r02j_splitk_dw4096_vib.log).
int mmad_tile_adam_override() { return g_knob[5]; }
int mmad_tile_adam_for(int Mp, int Np, int K) {
  if (g_knob[5] != -2) return g_knob[5];
  return (K >= 2048 && (long)Mp * Np >= 1500000L) ? 0 : 3;
}
// tile of the Adam-fused dW GEMMs that run on the main stream at the end of
// the backward (nothing else on the GPU then; -1 = same as knob 5, -2 = a
// rule: 128x128 where that grid covers >= 200 of the 256 CUs).  Default 0:
// 128x128 for both (c2 layer 0, 208 tiles: 27.1 vs 32.6 us under rocprofv3;
// layer 1, 130 tiles: 28.3 vs 25.7 -- yet the step is fastest with both on
// 128x128: 0.4314 / 0.4321-0.4326 / 0.4351 vs 0.4335-0.4339 / 0.4372 ms with
// the knob-5 tiles and 0.4372-0.4378 with the rule on three boxes,
// profiles/r05h_main_tail_dw_tile_ab.txt, r05t_main_tail_dw_tile_ab.txt; at
// 4096 rows knob 5's rule already picks 128x128 for these layers).
int mmad_tile_adam_main_override() { return g_knob[8]; }
int mmad_tile_adam_main_for(int Mp, int Np, int K) {
  if (g_knob[8] != -2) return g_knob[8];
  return (Mp / 128) * (Np / 128) >= 200 ? 0 : mmad_tile_adam_for(Mp, Np, K);
}
// per-epilogue tile overrides (-1 = autotuned): bwd-data GEMMs, forward GEMMs
int mmad_tile_epi_override(int epi) {
  if (epi == GEMM_EPI_BWD_DATA) return g_knob[6];
  if (epi == GEMM_EPI_FWD || epi == GEMM_EPI_MSE) return g_knob[7];
  return -1;
}

static bool knob_valid(int knob) {
  return knob >= 0 && knob < MMAD_KNOB_COUNT;
}
int mmad_tune_set(int knob, int value) {
  if (!knob_valid(knob)) {
    mmad_set_error("tune_set: unknown knob %d", knob);
    return MMAD_EINVAL;
  }
  g_knob[knob] = value;
  return MMAD_OK;
}
int mmad_tune_get(int knob, int* value) {
  if (!knob_valid(knob) || !value) {
    mmad_set_error("tune_get: unknown knob %d", knob);
    return MMAD_EINVAL;
  }
  *value = g_knob[knob];
  return MMAD_OK;
}

int mmad_gemm_splitk_for(int Mp, int Np, int K, int dtype, int epi) {
  if (Mp <= 0 || Np <= 0 || K <= 0 || epi < 0 || epi > 4) return 1;
  return mmad_gemm_splitk(Mp, Np, K, dtype, epi);
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
// split-K workspace of the calling thread's layer-operator GEMMs (optional)
static thread_local char* g_sk_ws = nullptr;

size_t mmad_gemm_ws_bytes(void) {
  size_t slab = 0, ctl = 0;
  mmad_gemm_splitk_bytes(0, 0, &slab, &ctl);
  return slab + ctl;
}

int mmad_gemm_set_workspace(void* ws, size_t bytes) {
  MMAD_CHECK_ARG(!ws || bytes >= mmad_gemm_ws_bytes(), "gemm_set_workspace: %zu < %zu bytes",
                 bytes, mmad_gemm_ws_bytes());
  MMAD_CHECK_ARG(((uintptr_t)ws) % 256 == 0, "gemm_set_workspace: not 256-byte aligned");
  g_sk_ws = (char*)ws;
  return MMAD_OK;
}

int mmad_gemm_status(void* stream) {
  if (!g_sk_ws) return MMAD_OK;
  size_t slab = 0, ctl = 0;
  mmad_gemm_splitk_bytes(0, 0, &slab, &ctl);
  return mmad_gemm_read_status((unsigned*)(g_sk_ws + slab), (hipStream_t)stream, "gemm_status");
}

static int layer_gemm(int dtype, int epi, const void* A, int lda, const void* B, int ldb, int Mp,
                      int Np, int K, GemmEpi ep, void* stream) {
  if (g_sk_ws) {
    size_t slab = 0, ctl = 0;
    mmad_gemm_splitk_bytes(0, 0, &slab, &ctl);
    ep.sk_slab = (float*)g_sk_ws;
    ep.sk_ctl = (unsigned*)(g_sk_ws + slab);
  }
  return mmad_gemm_dispatch(dtype, epi, A, lda, B, ldb, Mp, Np, K, ep, (hipStream_t)stream);
}
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
  return layer_gemm(dtype, GEMM_EPI_FWD, x, Kp, w, Kp, Mp, Np, Kp, ep, stream);
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
  return layer_gemm(dtype, GEMM_EPI_MSE, x, Kp, w, Kp, Mp, Np, Kp, ep, stream);
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
  return layer_gemm(dtype, GEMM_EPI_SCORE, x, Kp, w, Kp, Mp, Np, Kp, ep, stream);
}

int mmad_nap_score(int dtype, int M, int K, int R, int Mp, int Kp, int Rp, const void* x,
                   const void* vt, const float* bias, const float* w, float* rowsq, float* score,
                   void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("nap_score", M, R, K, Mp, Rp, Kp));
  MMAD_CHECK_ARG(x && vt && bias && w && rowsq && score, "nap_score: null operand");
  GemmEpi ep{};
  ep.M = M; ep.N = R; ep.out = nullptr; ep.ldo = Rp; ep.bias = bias; ep.act = MMAD_ACT_NONE;
  ep.ref = nullptr; ep.ldref = Rp; ep.rowsq = rowsq; ep.ldrow = Mp; ep.colw = w;
  RET_IF(layer_gemm(dtype, GEMM_EPI_SCORE, x, Kp, vt, Kp, Mp, Rp, Kp, ep, stream));
  return mmad_colsum(Rp / 128, M, Mp, rowsq, Mp, 1.f / (float)R, score, stream);
}

int mmad_fc_bwd_data(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* dz,
                     const void* w, void* dx, float* colsum, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_bwd_data", M, N, K, Mp, Np, Kp));
  MMAD_CHECK_ARG(dz && w && dx, "fc_bwd_data: null operand");
  GemmEpi ep{};
  ep.M = M; ep.N = K; ep.out = dx; ep.ldo = Kp; ep.part = colsum; ep.ldpart = Kp;
  // dx[Mp][Kp] = dz[Mp][Np] . W[Np][Kp]: contraction over Np, W read MN-major
  return layer_gemm(dtype, GEMM_EPI_BWD_DATA, dz, Np, w, Kp, Mp, Kp, Np, ep, stream);
}

int mmad_fc_bwd_weight(int dtype, int Mp, int Np, int Kp, const void* dz, const void* x,
                       float* dw, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_bwd_weight", Mp, Np, Kp, Mp, Np, Kp));
  MMAD_CHECK_ARG(dz && x && dw, "fc_bwd_weight: null operand");
  GemmEpi ep{};
  ep.M = Np; ep.N = Kp; ep.out = dw; ep.ldo = Kp;
  // dW[Np][Kp] = dz^T . x, contraction over the batch; both read MN-major
  return layer_gemm(dtype, GEMM_EPI_BWD_WEIGHT, dz, Np, x, Kp, Np, Kp, Mp, ep, stream);
}

int mmad_fc_bwd_weight_adam(int dtype, int Mp, int Np, int Kp, const void* dz, const void* x,
                            float* p, float* m, float* v, void* shadow, float* dw, float beta1,
                            float beta2, float eps, float step_size, float bc2_sqrt, void* stream) {
  RET_IF(check_dtype(dtype));
  RET_IF(check_dims("fc_bwd_weight_adam", Mp, Np, Kp, Mp, Np, Kp));
  MMAD_CHECK_ARG(dz && x && p && m && v, "fc_bwd_weight_adam: null operand");
  MMAD_CHECK_ARG(!shadow || dtype == MMAD_BF16, "fc_bwd_weight_adam: the shadow is bf16");
  GemmEpi ep{};
  ep.M = Np; ep.N = Kp; ep.out = dw; ep.ldo = Kp;
  ep.ad_p = p; ep.ad_m = m; ep.ad_v = v; ep.ad_shadow = shadow;
  const MmadAdamConsts c = mmad_adam_consts(1e-3f, beta1, beta2, eps, 1);   // w1 / w2 only
  ep.ad_w1 = c.w1; ep.ad_w2 = c.w2; ep.ad_eps = eps; ep.ad_step = step_size; ep.ad_bc2 = bc2_sqrt;
  ep.dw_nostore = dw ? 0 : 1;
  return layer_gemm(dtype, GEMM_EPI_BWD_WEIGHT, dz, Np, x, Kp, Np, Kp, Mp, ep, stream);
}
