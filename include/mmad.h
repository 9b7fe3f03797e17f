/*
 * mmad.h -- C-ABI of the MI355X-native autoencoder train-and-score hot path.
 *
 * The reference (Yoo-Youngjae/ICRA2021_multimodal_ad) has no FFI: its hot path
 * is stock torch modules behind a Python plugin surface.  Each entry point
 * below names the reference interface it replaces (file:line, relative to the
 * reference repo root).  The Python mirror of that surface
 * (icra2021_multimodal_ad_amd/) binds these with ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Device pointers unless stated.  All
 *    tensors are caller-owned; nothing here allocates device memory.
 *  - Packed layouts: every feature and batch dimension is padded to a
 *    multiple of mmad_pad_granule() (128) with zeros; a [rows][cols] matrix
 *    has leading dimension = padded cols.  "M/N/K" are the valid sizes,
 *    "Mp/Np/Kp" the padded ones.
 *  - dtype selects the activation/weight storage type of the GEMM operands
 *    (MMAD_F32: exact-fp32 parity path on f32 MFMA; MMAD_BF16: bf16 storage,
 *    fp32 accumulation).  Gradients, optimizer state, BN statistics and all
 *    reductions are fp32.
 *  - Every call returns 0 (MMAD_OK) or a negative status; the message is in
 *    mmad_last_error_string() (thread-local).  No exceptions cross the ABI.
 *  - stream is a hipStream_t passed as void* (0 = legacy default stream).
 */
#ifndef MMAD_H_
#define MMAD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMAD_ABI_VERSION 1

enum { MMAD_OK = 0, MMAD_EINVAL = -1, MMAD_EUNSUPPORTED = -2, MMAD_EHIP = -3, MMAD_ERCCL = -4 };
enum { MMAD_F32 = 0, MMAD_BF16 = 1 };
/* modules/activation.py:20-45 (names 'leakyrelu', 'relu', 'sigmoid', 'tanh', None) */
enum { MMAD_ACT_NONE = 0, MMAD_ACT_LEAKYRELU = 1, MMAD_ACT_RELU = 2, MMAD_ACT_SIGMOID = 3,
       MMAD_ACT_TANH = 4, MMAD_ACT_LOGSIGMOID = 5, MMAD_ACT_SOFTMAX = 6, MMAD_ACT_LOGSOFTMAX = 7 };

const char* mmad_last_error_string(void);
int mmad_abi_version(void);
int mmad_pad_granule(void);
/* Tuning knobs (no reference counterpart).  One process-wide table, set only
 * through mmad_tune_set (the library reads no environment variables).  GEMM
 * knobs are read per dispatch; the executor's schedule knobs (14-31, 33-35) are
 * copied into a handle by mmad_ae_create, so set them before creating it.
 *   0  GEMM tile override (-1 autotuned; 0 = 128x128/512 thr, 1 = 256x128,
 *      2 = 128x256, 3 = 64x64/256 thr, 4 = 64x128, 5 = 128x128/256 thr,
 *      6 = 256x256/512 thr (bf16 forward / MSE / score GEMMs without fused BN
 *      or split-K); a tile that does not fit a shape falls back to the tuned one)
 *   1  XCD tile-group height override (-1 rule)
 *   2  per-shape autotune on first dispatch (1, default) or static heuristic (0)
 *   3  diagnostics bits (tools/gemm_phase; 4 = force the split-K combine's
 *      timeout path, tests only)
 *   4  split-K factor override for GEMMs given split-K workspace (0 = shape
 *      rule, 1/2/4/8/16); 9 = the same for the dW GEMMs only; 10 / 11 = the dW
 *      split rule's target number of 64x64-tile blocks (0 = no split, default)
 *      and minimum K stages per slice (8)
 *   5  tile of the Adam-fused dW GEMMs (-2 shape rule, -1 autotuned); 8 = of
 *      those on the main stream at the end of the backward (default 0 =
 *      128x128; -2 = 128x128 where its grid covers >= 200 CUs, else knob 5;
 *      -1 = knob 5);
 *      6 / 7 = tile of the bwd-data / forward GEMMs (-1 autotuned)
 *   12 persistent grid for the forward-type GEMMs without a fused BN or a
 *      split (0 off; any other value: persistent whenever the tiles exceed
 *      one resident round -- with fewer tiles the ordinary grid is the same
 *      launch)
 *   13 BN-backward apply kernel: 128-row slabs per block (1, 2 or 4; any other
 *      value = 1; halved until it divides the row slabs; the column partials
 *      are merged once per block; default 2)
 *   14 data parallel: from this many padded rows, each side-stream dW GEMM
 *      starts at its own dz instead of with its bucket's lowest layer (1024;
 *      0 = one fork per bucket)
 *   15 schedule study: the side stream created behind a CU mask that leaves
 *      this many CUs to the main stream alone (0 = off; the masked stream is
 *      blocking, so call the step on a created non-blocking stream)
 *   16 train-mode BN schedule (-1 dtype default: bf16 fused, fp32 apply;
 *      0 apply kernels, 1 fold into the consumer, 2 fused into the GEMMs)
 *   17 backward BN schedule (-1 = the forward's, 2 = fused into bwd-data)
 *   18 fused BN up to this many padded rows per call (2048; fold above)
 *   19 dW GEMMs of the last layers on the main stream (2)
 *   20 ping-pong weight shadows from this many padded rows (4096); 21 = main-
 *      stream dW GEMMs then (1)
 *   22 record the bwd-data event every n-th side-stream layer (2)
 *   23 reduce the loss on the side stream right after the forward (1)
 *   24 data parallel: exchange the small bucket after this layer's bwd-data (1)
 *   25 also materialise dW in the fused step (0)
 *   26 side stream at the highest priority instead of the lowest (0)
 *   27 executor events with the system-scope fence (0)
 *   28 data parallel: sharded weight buckets (reduce-scatter, Adam on 1/N,
 *      all-gather; 1) or all-reduce + full Adam (0)
 *   29 schedule study: every side-stream dW + Adam GEMM held until the main
 *      stream has enqueued the whole bwd-data chain (0)
 *   30 data parallel: minimum exchange bucket in MiB of fp32 gradient;
 *      consecutive layers (backward order) share a bucket until it holds this
 *      much (8; 0 = one bucket per layer)
 *   31 the bwd-data GEMM's hand-off event to the side stream completed by the
 *      launch itself (hipExtLaunchKernel stop event, 1) or recorded behind it
 *      (0: a marker packet that holds the main stream's next dispatch)
 *   32 exact-fp32 dW GEMMs contracting over >= 2048 rows: split K until the
 *      launch has about this many 64x64-tile blocks, >= 16 K stages per
 *      slice (1024; 0 = never split an fp32 GEMM)
 *   33 ping-pong steps: the side-stream dW + Adam GEMMs of the top this many
 *      layers start once the main stream has also finished the layer's
 *      bwd-data GEMM and BN-backward apply, instead of at its dz (0)
 *   34 ping-pong steps: each side-stream dW's fork event completed by the
 *      launch that produces the layer's dz (BN-backward apply or bwd-data
 *      GEMM, hipExtLaunchKernel stop event) instead of a marker packet on the
 *      main stream; the top layer forks through the loss reduction's wait on
 *      the MSE launch (1; 0 = markers)
 *   35 ping-pong steps: from this layer down the side-stream dW GEMMs fork in
 *      pairs -- every other layer's dz gets no fork event and its dW is issued
 *      with the next lower layer's (0 = every layer forks) */
#define MMAD_KNOB_COUNT 36
int mmad_tune_set(int knob, int value);
int mmad_tune_get(int knob, int* value);
/* The split-K factor the dispatcher picks for a padded GEMM shape (Mp x Np
 * output, K deep) with epilogue `epi` (0 fwd, 1 MSE, 2 bwd-data, 3 dW,
 * 4 score) under the current knobs: 1, 2, 4, 8 or 16 (query only). */
int mmad_gemm_splitk_for(int Mp, int Np, int K, int dtype, int epi);

/* ------------------------------------------------------------------------
 * Layer operators
 * ---------------------------------------------------------------------- */

/* Split-K workspace for the calling thread's layer-operator GEMMs below
 * (optional; no reference counterpart).  Shapes with few output tiles then
 * split their K loop over 2 or 4 workgroups (a fixed factor per shape) that
 * combine in-launch.  ws: device memory of >= mmad_gemm_ws_bytes() bytes,
 * 256-byte aligned, ZEROED before first use (every launch leaves its control
 * words zero); it must not be shared by GEMMs running concurrently on
 * different streams.  ws = NULL turns it off. */
size_t mmad_gemm_ws_bytes(void);
int mmad_gemm_set_workspace(void* ws, size_t bytes);
/* Synchronises `stream` and reports (then clears) a split-K combine that timed
 * out in the calling thread's layer-operator workspace since the last check:
 * MMAD_EHIP and the error string if one did (its output tiles were not
 * written), MMAD_OK otherwise (also without a workspace). */
int mmad_gemm_status(void* stream);

/* FCLayer.forward, layers/fc_layer.py:37-48 (nn.Linear -> Activation -> BN).
 * y[Mp][Np] = bn_affine(act(x[Mp][Kp] . w[Np][Kp]^T + bias[Np])).
 * bn_scale/bn_shift (nullable): eval-mode BatchNorm1d as a per-column affine
 * (see mmad_bn_eval_affine).  stats (nullable, fp32 [Mp/32][2][Np]): per
 * 32-row chunk Welford (mean, M2) of the post-activation values, consumed by
 * mmad_bn_train_apply for train-mode BN.  Rows >= M and cols >= N are written 0. */
int mmad_fc_fwd(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                const void* w, const float* bias, int act, float slope, const float* bn_scale,
                const float* bn_shift, void* y, float* stats, void* stream);

/* Last decoder layer fused with Loss('mse', reduction='sum') forward+backward
 * (modules/loss.py:31-32,47-52; model_builder.py:42):
 * d = x.w^T + bias - target; dz = grad_scale*d (dtype, [Mp][Np]);
 * partials fp32 [Mp/32][2][Np] = (sum_rows dz, sum_rows d^2). */
int mmad_fc_fwd_mse(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                    const void* w, const float* bias, const float* target, int ld_target,
                    float grad_scale, void* dz, float* partials, void* stream);

/* Eval-mode FCLayer.forward fused with the per-window squared-diff reduction
 * of reconstruction_aggregation.py:22-28: y as mmad_fc_fwd (eval affine), and
 * rowsq[Np/128][Mp] = per-128-column partial sums of (y - ref)^2; diff
 * (nullable, fp32, ld_diff) receives y - ref for the valid region. */
int mmad_fc_fwd_score(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* x,
                      const void* w, const float* bias, int act, float slope,
                      const float* bn_scale, const float* bn_shift, void* y, const void* ref,
                      float* rowsq, float* diff, int ld_diff, void* stream);

/* BatchNorm1d eval affine (layers/fc_layer.py:33): scale = gamma/sqrt(rv+eps),
 * shift = beta - rm*scale, for N columns (padded columns -> 0). */
int mmad_bn_eval_affine(int N, int Np, const float* gamma, const float* beta, const float* rm,
                        const float* rv, float eps, float* scale, float* shift, void* stream);

/* BatchNorm1d train-mode forward (layers/fc_layer.py:39-45; torch
 * native_batch_norm): merges the Welford partials of mmad_fc_fwd, normalises
 * a -> y with batch statistics (biased var), updates running stats
 * (momentum, unbiased var), saves mean / rstd for backward. */
int mmad_bn_train_apply(int dtype, int M, int N, int Mp, int Np, const void* a,
                        const float* stats, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, float momentum, float eps,
                        float* save_mean, float* save_rstd, void* y, void* stream);

/* NAP run (utils/metric.py:183-238; Rotater.run utils/normalize.py:72-103 and
 * Standardizer.run :36-45 folded into one GEMM + epilogue):
 *   score[m] = (1/R) sum_{j<R} w[j] * (sum_k x[m][k] vt[j][k] + bias[j])^2
 * with vt = V^T of the rotation, bias = -(mu_r V + mu_s), w = 1/var (0 on
 * padding).  x: packed concatenated diffs [Mp][Kp] (dtype), vt [Rp][Kp]
 * (dtype); rowsq: fp32 workspace [Rp/128][Mp]; score fp32 [M]. */
int mmad_nap_score(int dtype, int M, int K, int R, int Mp, int Kp, int Rp, const void* x,
                   const void* vt, const float* bias, const float* w, float* rowsq, float* score,
                   void* stream);

/* NAP fit (Rotater.fit utils/normalize.py:52-70, then Standardizer.fit
 * :25-34 on the rotated train diffs; utils/metric.py:183-238 fits both on the
 * train diffs).  x: train diffs, device fp32 [N][ldx] (concatenated layers).
 * Outputs (device fp32): mu_r [W] = mean(x), v [W][R] (R = min(N, W)) = the
 * right singular vectors of x - mu_r in descending singular-value order (the
 * eigenvectors of the fp64 Gram, rocSOLVER dsyevd; column signs are the
 * solver's, as the reference's are its SVD's -- NAP scores do not depend on
 * them), mu_s [R] / var [R] = mean and ddof-1 variance of rot = (x - mu_r) v
 * (fp32 product, fp64 statistics as np.cov).  N >= 2.  Deterministic.
 * Synchronises `stream` once (eigensolver convergence flag). */
size_t mmad_nap_fit_ws_bytes(int64_t N, int W);
int mmad_nap_fit(int64_t N, int W, const float* x, int64_t ldx, float* mu_r, float* v, float* mu_s,
                 float* var, void* ws, size_t ws_bytes, void* stream);

/* Backward of Linear (autograd of layers/fc_layer.py:38):
 * dx[Mp][Kp] = dz[Mp][Np] . w[Np][Kp]; colsum (nullable, [Mp/32][2][Kp]
 * slot 0) = per-chunk column sums of dx (bias grad of a no-BN producer). */
int mmad_fc_bwd_data(int dtype, int M, int N, int K, int Mp, int Np, int Kp, const void* dz,
                     const void* w, void* dx, float* colsum, void* stream);

/* dW[Np][Kp] (fp32) = dz[Mp][Np]^T . x[Mp][Kp] (K = batch). */
int mmad_fc_bwd_weight(int dtype, int Mp, int Np, int Kp, const void* dz, const void* x,
                       float* dw, void* stream);

/* The standalone Activation module (modules/activation.py:20-45) on fp32
 * [M][ld] rows of N values: act = any MMAD_ACT_* (softmax / logsoftmax over
 * each row, dim=-1, max-subtracted; logsigmoid = -softplus(-x); leaky slope
 * `slope`).  mmad_activation_bwd: dx from the forward OUTPUT y and dy
 * (sigmoid y(1-y), tanh 1-y^2, relu/leaky by the sign of y, logsigmoid
 * 1-exp(y), softmax y(dy - sum dy y), logsoftmax dy - exp(y) sum dy).
 * x / y / dy / dx may share ld; y may alias x (in place), dx may alias dy. */
int mmad_activation_fwd(int act, float slope, int M, int N, const float* x, int64_t ldx, float* y,
                        int64_t ldy, void* stream);
int mmad_activation_bwd(int act, float slope, int M, int N, const float* y, int64_t ldy,
                        const float* dy, int64_t lddy, float* dx, int64_t lddx, void* stream);

/* dW as mmad_fc_bwd_weight with torch.optim.Adam's step (as mmad_adam) fused
 * into the GEMM epilogue (loss.backward() + optimizer.step() for one
 * nn.Linear weight, models/auto_encoder.py:73-75): p/m/v fp32 [Np][Kp] are
 * updated in place, shadow (nullable, bf16 [Np][Kp]) receives bf16(p), dw
 * (nullable) the gradient itself.  Padding rows/columns of p/m/v must be zero
 * (they stay zero: their gradient is zero). */
int mmad_fc_bwd_weight_adam(int dtype, int Mp, int Np, int Kp, const void* dz, const void* x,
                            float* p, float* m, float* v, void* shadow, float* dw, float beta1,
                            float beta2, float eps, float step_size, float bc2_sqrt, void* stream);

/* Backward of BN(train) o Activation (layers/fc_layer.py:38-45):
 * dbeta = sum dy, dgamma = sum dy*xhat, da = gamma*rstd/M*(M dy - dbeta - xhat dgamma),
 * dz = da * act'(a).  Writes dz (dtype), dgamma/dbeta (fp32 [Np]) and db
 * partials ([Mp/128][Np], consumed by mmad_colsum).  ws: >= mmad_bn_act_bwd_ws(Mp,Np) bytes. */
size_t mmad_bn_act_bwd_ws(int Mp, int Np);
int mmad_bn_act_bwd(int dtype, int act, float slope, int M, int N, int Mp, int Np, const void* dy,
                    const void* a, const float* save_mean, const float* save_rstd,
                    const float* gamma, void* dz, float* dgamma, float* dbeta, float* db_partials,
                    void* ws, void* stream);

/* Backward of Activation alone (an FCLayer without BN, layers/fc_layer.py:38):
 * dz = dy * act'(a) from the activation output a (packed [Mp][Np], dtype;
 * rows >= M -> 0) and db partials fp32 [Mp/128][Np] (column sums of dz, the
 * bias gradient; reduce with mmad_colsum). */
int mmad_act_bwd(int dtype, int act, float slope, int M, int Mp, int Np, const void* dy,
                 const void* a, void* dz, float* db_partials, void* stream);

/* out[j] = scale * sum_{i<n_parts} partials[i*part_stride + j], j < N (Np padded -> 0). */
int mmad_colsum(int n_parts, int N, int Np, const float* partials, int part_stride, float scale,
                float* out, void* stream);

/* out[0] = scale * sum of n floats (single block, deterministic). */
int mmad_sum(int64_t n, const float* x, float scale, float* out, int accumulate, void* stream);
/* modules/loss.py:47-52, Loss('mse', reduction) called on its own (inside the
 * autoencoder it is fused into the last decoder GEMM): loss_out[0] = sum (mean
 * != 0: mean) of (y_hat - y)^2 over n fp32 elements, deterministic order.
 * work: device scratch of mmad_mse_loss_ws_floats() floats.  mmad_mse_grad:
 * d_yhat = g[0] * (2 or 2/n) * (y_hat - y), d_y = -d_yhat (either nullable;
 * g = the upstream scalar gradient on the device, nullable = 1). */
int mmad_mse_loss_ws_floats(void);
int mmad_mse_loss(int64_t n, const float* y_hat, const float* y, int mean, float* loss_out, float* work,
                  void* stream);
int mmad_mse_grad(int64_t n, const float* y_hat, const float* y, const float* g, int mean, float* d_yhat,
                  float* d_y, void* stream);

/* f32 [M][ld_x] -> packed dtype [Mp][Kp] (zero padding). */
int mmad_pack_input(int dtype, int M, int K, int Mp, int Kp, const float* x, int ld_x, void* out,
                    void* stream);

/* packed dtype [Mp][Np] -> f32 [M][ld_out] (valid region). */
int mmad_unpack_output(int dtype, int M, int N, int Np, const void* y, float* out, int ld_out,
                       void* stream);

/* torch.optim.Adam step (novelty_detection.py:90; amsgrad=False,
 * weight_decay=0) over a flat fp32 buffer of n params, rounded as torch's
 * CPU _single_tensor_adam rounds it:
 * m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
 * p += (-step_size * m) / (sqrt(v)/bc2_sqrt + eps); step_size = lr/(1-b1^t),
 * with 1-b1 and 1-b2 formed in double from the decimal each float beta came
 * from (0.9f -> 0.9), as torch forms them from the optimizer's Python floats.
 * shadow (nullable, bf16) receives bf16(p) for the first n_shadow elements. */
int mmad_adam(int64_t n, float* p, const float* g, float* m, float* v, float beta1, float beta2,
              float eps, float step_size, float bc2_sqrt, void* shadow, int64_t n_shadow,
              void* stream);

/* variational_info_bottleneck reparameterisation
 * (decorators/variational_info_bottleneck.py:22-24,34,37): enc_out [Mp][ld_enc]
 * (dtype) holds mu | logvar in cols [0,btl) | [btl,2btl) of the first B rows;
 * z[row = kk*B + b][c] = eps*exp(0.5*logvar) + mu written packed into
 * z (dtype, [Mpz][ld_z]) for kk < k.  eps: injected fp32 [k][B][btl]
 * (nullable -> Philox N(0,1) from seed/offset; the draw is stored to eps_out,
 * nullable).  deterministic != 0 -> z = mu (no_grad and not stochastic).
 * kl_partial (nullable): fp32 [Mp/128] partial sums of
 * -0.5*(1 + lv - mu^2 - exp(lv)) (build-defined KL, SURVEY §8 a10'). */
int mmad_vib_reparam_fwd(int dtype, int B, int btl, int k, const void* enc_out, int ld_enc,
                         const float* eps, float* eps_out, uint64_t seed, uint64_t offset,
                         int deterministic, void* z, int ld_z, float* kl_partial, void* stream);

/* Backward of the reparameterisation + beta*KL: dz [k*B rows][ld_dz] (dtype)
 * -> d_enc_out (dtype [Mp][ld_denc], mu|logvar columns); colsum (nullable)
 * receives column-sum partials [Mp/128][ld_denc] for the encoder's last bias. */
int mmad_vib_reparam_bwd(int dtype, int B, int btl, int k, const void* enc_out, int ld_enc,
                         const float* eps, const void* dz, int ld_dz, float beta_kl,
                         void* d_enc_out, int ld_denc, float* colsum, void* stream);

/* ------------------------------------------------------------------------
 * Whole-autoencoder executor (AutoEncoder.step / validate / forward and
 * get_diffs, models/auto_encoder.py:36-91, reconstruction_aggregation.py:6-37):
 * sequences the layer operators above on one stream with no host sync.
 * ---------------------------------------------------------------------- */
typedef struct mmad_ae mmad_ae;

/* widths: encoder widths [n_enc+1] then decoder widths [n_dec+1]; hidden
 * layers (all but the last of each module) are Linear->LeakyReLU(slope)->BN,
 * last layers Linear only (model_builder.py:21-37).  vib != 0: encoder output
 * is 2*btl (mu|logvar) and dec_widths[0] = btl. */
int mmad_ae_create(mmad_ae** out, int dtype, int n_enc, const int* enc_widths, int n_dec,
                   const int* dec_widths, int vib, float slope, float bn_eps, float bn_momentum);
void mmad_ae_destroy(mmad_ae* h);

/* Flat fp32 parameter layout (padded): all weights first ([Np][Kp] per layer,
 * encoder then decoder), then per layer bias[Np], gamma[Np], beta[Np].
 * info (int64[7] per layer): w_off, b_off, gamma_off (-1), beta_off (-1),
 * Kp, Np, bn_off (offset into the [2][n_bn] running-stat buffer, -1).
 * totals (int64[4]): n_params, n_weight (= bf16 shadow length), n_bn, n_layers. */
int mmad_ae_layout(const mmad_ae* h, int64_t* info, int64_t* totals);

/* Device workspace bytes for a batch of B windows and k VIB samples. */
int64_t mmad_ae_workspace_bytes(const mmad_ae* h, int B, int k);

/* Bind caller-owned device buffers (all fp32 flat, layout above).
 * shadow: bf16 weights (MMAD_BF16) or NULL (MMAD_F32 reads params). */
int mmad_ae_bind(mmad_ae* h, float* params, float* grads, float* adam_m, float* adam_v,
                 void* shadow, float* running /* [2][n_bn]: mean then var */);

/* Refresh the bf16 weight shadow from the fp32 params (after a host-side
 * load_state_dict or any external parameter write).  No-op for MMAD_F32. */
int mmad_ae_sync_shadow(mmad_ae* h, void* stream);

/* bf16 only: a second n_weight-element bf16 buffer (NULL turns it off).  The
 * fused step (mmad_ae_train_step) then writes the updated weights into the
 * other buffer while its backward still reads the current one, and the two
 * swap at the end of the step, so each layer's dW+Adam GEMM overlaps that
 * layer's bwd-data GEMM.  mmad_ae_sync_shadow refreshes both. */
int mmad_ae_set_shadow_pair(mmad_ae* h, void* alt);

/* the bf16 shadow the next kernels will read (changes after each fused step
 * when a pair is set) */
const void* mmad_ae_current_shadow(const mmad_ae* h);

/* AutoEncoder.step forward+backward (models/auto_encoder.py:57-73): x fp32
 * [B][ld_x]; writes grads and loss_out[0] (device fp32; sum-MSE, or
 * recon/k + beta*KL for VIB).  eps (VIB, nullable) as mmad_vib_reparam_fwd. */
int mmad_ae_train_fwd_bwd(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                          uint64_t seed, uint64_t offset, float beta_kl, float* loss_out,
                          void* ws, int64_t ws_bytes, void* stream);

/* One whole AutoEncoder.step (models/auto_encoder.py:57-77) with
 * optimizer.step() fused in: forward + sum-MSE + backward as in
 * mmad_ae_train_fwd_bwd, and each layer's Adam update (hyper-parameters as
 * mmad_ae_adam, step = t) issued on the executor's side stream right after
 * that layer's dW GEMM, overlapping the rest of the backward.  With a
 * communicator attached (mmad_ae_set_comm) the gradients are all-reduced per
 * layer before their Adam update and the returned loss is the global sum.
 * On return every kernel is enqueued and ordered before later work on
 * `stream`. */
int mmad_ae_train_step(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                       uint64_t seed, uint64_t offset, float beta_kl, float lr, float beta1,
                       float beta2, float adam_eps, int step, float* loss_out, void* ws,
                       int64_t ws_bytes, void* stream);

/* mmad_ae_train_step replayed as ONE captured hipGraph (the whole step's
 * ~45 kernels, side-stream dW/Adam overlap included) after a 64-byte
 * host->device copy of this call's values (x, loss_out, eps, seed/offset, the
 * Adam bias-correction terms of `step`): same arguments, same results bit for
 * bit.  The first call of a signature (B, k, ld_x, x alignment, eps given or
 * not, ws, beta_kl, Adam betas/eps) runs eagerly and captures; rebinding the
 * buffers drops the captures.  With a communicator or a shadow pair attached,
 * or if capture is unavailable, it runs the eager step instead. */
int mmad_ae_train_step_graph(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                             uint64_t seed, uint64_t offset, float beta_kl, float lr, float beta1,
                             float beta2, float adam_eps, int step, float* loss_out, void* ws,
                             int64_t ws_bytes, void* stream);
/* number of captured train-step graphs (-1 for a null handle) */
int mmad_ae_train_graph_count(const mmad_ae* h);

/* loss.backward() after mmad_ae_forward(train_bn=1) on the same workspace
 * (autograd path of AutoEncoder.forward): dxhat fp32 [B][ld] = dL/dx_hat;
 * writes all parameter gradients.  Not for the VIB model. */
int mmad_ae_backward(mmad_ae* h, const float* dxhat, int ld, int B, void* ws, int64_t ws_bytes,
                     void* stream);

/* ------------------------------------------------------------------------
 * Data-parallel gradient exchange (RCCL over xGMI)
 * The reference trains in one process (novelty_detection.py:90); with one
 * process per GPU the exchange is a sum all-reduce of the gradients (the loss
 * is sum-reduced, model_builder.py:42).  RCCL is resolved from the copy
 * already loaded in the process (torch's), so there is one RCCL instance.
 * ---------------------------------------------------------------------- */
typedef struct mmad_comm mmad_comm;
int mmad_comm_unique_id_bytes(void);
/* rank 0: fills out[mmad_comm_unique_id_bytes()] (host memory) */
int mmad_comm_get_unique_id(void* out);
/* every rank, with the current HIP device set to its GPU */
int mmad_comm_create(mmad_comm** out, const void* unique_id, int nranks, int rank);
/* single-GPU loopback communicator for testing the exchange schedule: its
 * "all-reduce" scales the bucket by `scale` (= the sum over `scale` identical
 * shards) after a short delay */
int mmad_comm_create_loopback(mmad_comm** out, float scale);
/* ... posing as rank `rank` of `nranks` (tests of the sharded step's shard
 * arithmetic on one GPU: its reduce-scatter scales this rank's slice of the
 * bucket -- the slice RCCL's in-place reduce-scatter writes -- and its
 * all-gather leaves the other ranks' shards untouched) */
int mmad_comm_create_loopback_ranks(mmad_comm** out, float scale, int nranks, int rank);
void mmad_comm_destroy(mmad_comm* c);
/* in-place fp32 sum all-reduce of buf[n] on stream */
int mmad_allreduce_bucket(mmad_comm* c, float* buf, int64_t n, void* stream);
/* this communicator's rank / number of ranks (a loopback communicator: the
 * rank / nranks given to its create call; 0 / 1 for mmad_comm_create_loopback) */
int mmad_comm_rank(const mmad_comm* c);
int mmad_comm_size(const mmad_comm* c);
/* sharded exchange, in place (n divisible by the rank count): sum
 * reduce-scatter of fp32 buf[n] leaving rank r's sum in buf[r*n/N, (r+1)*n/N);
 * all-gather of every rank's shard of buf[n] (dtype MMAD_F32 or MMAD_BF16).
 * Loopback: the reduce-scatter scales only this rank's slice
 * [r*n/N, (r+1)*n/N) by the loopback's scale (after the same short delay),
 * the all-gather does nothing. */
int mmad_reduce_scatter_bucket(mmad_comm* c, float* buf, int64_t n, void* stream);
/* the same on bf16 buf[n] (RCCL's bf16 sum; loopback: bf16(x * scale)) */
int mmad_reduce_scatter_bucket_bf16(mmad_comm* c, void* buf, int64_t n, void* stream);
int mmad_all_gather_bucket(mmad_comm* c, void* buf, int64_t n, int dtype, void* stream);
/* Attach (c != NULL) or detach a communicator.  With one attached,
 * mmad_ae_train_step runs the data-parallel step: each layer's dW lands in the
 * grads buffer, is all-reduced on the executor's comm stream as soon as it is
 * complete (overlapping the rest of the backward), then Adam-updated there;
 * bias/gamma/beta grads and the loss follow in one final bucket.  BatchNorm
 * statistics stay per shard (DDP semantics).
 * Sharded weight buckets (knob 28, default on; a bucket whose size the rank
 * count does not divide falls back to the all-reduce): reduce-scatter of the
 * fp32 gradient, Adam on this rank's 1/N of the bucket (p, m, v), then an
 * all-gather of the updated bf16 weight shadow (bf16 model: 4 + 2 bytes per
 * parameter on the wire instead of 8, the Adam state stream divided by N) or
 * of the fp32 weights (fp32 model).  The bf16 model's fp32 master weights and
 * every model's Adam moments are then current only on their owning rank:
 * mmad_ae_dp_sync_master (collective: every rank, same point) all-gathers
 * them; mmad_ae_dp_master_stale says whether one is due. */
int mmad_ae_set_comm(mmad_ae* h, mmad_comm* c);
/* Optional bf16 gradient exchange for the sharded buckets (NULL: off, the
 * default): `buf` is an n_weight-element bf16 scratch buffer; each sharded
 * bucket's fp32 gradient is rounded to bf16 into it, reduce-scattered in bf16
 * (half the bytes on the wire), and this rank's summed slice is widened back to
 * fp32 before its Adam.  Not the reference's arithmetic (its gradients are
 * summed in fp32): an opt-in for exchange-bound runs. */
int mmad_ae_set_grad_bf16(mmad_ae* h, void* buf);
int mmad_ae_dp_sync_master(mmad_ae* h, void* stream);
int mmad_ae_dp_master_stale(const mmad_ae* h);

/* optimizer.step() (models/auto_encoder.py:75) on the bound buffers. */
int mmad_ae_adam(mmad_ae* h, float lr, float beta1, float beta2, float eps, int step,
                 void* stream);
/* The same on the parameter range [off, off + n) of the flat buffers (off a
 * multiple of 4; the bf16 shadow is written where the range covers weights):
 * Adam is elementwise, so the ranges of a partition give mmad_ae_adam's bits.
 * Used by the torch-exchange data-parallel step, one range per bucket. */
int mmad_ae_adam_range(mmad_ae* h, float lr, float beta1, float beta2, float eps, int step,
                       int64_t off, int64_t n, void* stream);
/* Torch-exchange data parallelism (no counterpart; the path taken when the
 * native communicator is not attached): with dW events on, every
 * mmad_ae_train_fwd_bwd records one event after each layer's dW GEMM and one
 * after its bwd-data GEMM (the last reader of its weights);
 * mmad_ae_wait_dw makes `stream` wait for both, so a caller can all-reduce and
 * Adam-update a bucket while the rest of the backward runs.  mmad_ae_dw_plan
 * writes the weight buckets in backward order (the native exchange's plan,
 * knob 30): offset and length in the flat gradient buffer and the bucket's
 * lowest layer (the one to wait for); returns their count (< 0: error). */
int mmad_ae_dw_events(mmad_ae* h, int on);
int mmad_ae_wait_dw(mmad_ae* h, int layer, void* stream);
int mmad_ae_dw_plan(const mmad_ae* h, int max_n, int64_t* off, int64_t* n, int* layer_lo);

/* AutoEncoder.forward (models/auto_encoder.py:46-50): x_hat fp32 [B][ld_out].
 * train_bn != 0: batch-stat BN + running-stat update (module.train()).
 * loss_out (nullable): sum-MSE of x_hat vs x (AutoEncoder.validate). */
int mmad_ae_forward(mmad_ae* h, const float* x, int ld_x, int B, int train_bn, float* x_hat,
                    int ld_out, float* loss_out, void* ws, int64_t ws_bytes, void* stream);

/* get_diffs + per-window squared-diff sums (reconstruction_aggregation.py:6-37,
 * utils/metric.py:133,171): layer_sq fp32 [n_enc+1][B] with layer_sq[l][b] =
 * sum_c d_l[b][c]^2.  diffs (nullable): fp32 [B][sum widths] concatenated
 * d_0 | d_1 | ... (SAP/NAP layout). */
int mmad_ae_score(mmad_ae* h, const float* x, int ld_x, int B, float* layer_sq, float* diffs,
                  void* ws, int64_t ws_bytes, void* stream);

/* Streaming scoring pass (NoveltyDetecter.test -> get_diffs over a whole
 * dataset, novelty_detection.py:15-38 / reconstruction_aggregation.py:6-37,
 * BASELINE config C5): x fp32 [N][ld_x] in device memory, scored in batches of
 * `batch` windows (the last one ragged); layer_sq fp32, row l at
 * layer_sq + l*ld_sq (ld_sq >= N), same values as mmad_ae_score per batch.
 * ws sized by mmad_ae_workspace_bytes(h, batch, 1).
 * use_graph != 0: the first call for a given (x, ld_x, N, batch, layer_sq,
 * ld_sq, ws, weight buffer) runs eagerly and captures the pass as one hipGraph;
 * later calls replay it with a single hipGraphLaunch on `stream` (up to 8
 * passes cached per handle; weights and BN running statistics are read at
 * replay time, so training in between is seen). */
int mmad_ae_score_stream(mmad_ae* h, const float* x, int ld_x, int64_t N, int batch,
                         float* layer_sq, int64_t ld_sq, void* ws, int64_t ws_bytes, int use_graph,
                         void* stream);
/* Split-K health of the executor workspace `ws` (as mmad_gemm_status): a
 * no-op returning MMAD_OK unless split-K is enabled (tuning knob 4 > 1);
 * otherwise synchronises `stream` and returns MMAD_EHIP if any GEMM combine
 * of the calls since the last check timed out. */
int mmad_ae_status(mmad_ae* h, void* ws, int64_t ws_bytes, void* stream);

/* Kernel probe (measurement only; no reference counterpart): from now on the
 * executor brackets ONE GEMM launch per call with a pair of timing events on
 * the stream that launch runs on -- kind 0: the forward (or MSE / score) GEMM
 * of `layer`, kind 1: its dW GEMM (Adam fused in mmad_ae_train_step) -- for
 * the next `capacity` calls.  layer < 0 or capacity 0 turns it off.  A
 * probed launch on the main stream starts its clock only after the side
 * stream's earlier work (in probed calls only), so the pair brackets the
 * launch's own execution as a profiler's kernel record does.  Kinds 2 / 3:
 * the same launches (forward / dW) timed by events attached to the launch
 * itself (hipExtLaunchKernel start / stop: the kernel's own start and end) and
 * no wait for the side stream -- the launch as it runs in the step's schedule,
 * beside the side stream's work, cheap enough to stay on through a timed
 * region (bench.py's roofline).
 * mmad_ae_probe_read synchronises on the recorded events and writes up to
 * max_n durations (ms) in call order; returns how many (or < 0). */
int mmad_ae_probe(mmad_ae* h, int kind, int layer, int capacity);
int mmad_ae_probe_read(mmad_ae* h, float* ms, int max_n);
/* Layers (bit l) the last probed launch covered: one layer, or layers 0 and 1
 * when the main-stream tail ran its two Adam-fused dW GEMMs as one launch
 * (mmad_gemm_pair_kernel, MMAD_DW_PAIR). */
int mmad_ae_probe_layers(const mmad_ae* h);

/* number of cached score graphs (-1 for a null handle); drop them all */
int mmad_ae_graph_count(const mmad_ae* h);
int mmad_ae_clear_graphs(mmad_ae* h);

/* ------------------------------------------------------------------------
 * Anomaly-score metrics on the device (utils/metric.py, sklearn/numpy on the
 * host in the reference).  Scores fp32, labels uint8 (nonzero = anomaly,
 * novelty_detection.py:31-34), all device pointers; workspace caller-owned,
 * 256-byte aligned, sized by the *_ws_bytes queries.  Results fp64, device.
 * ---------------------------------------------------------------------- */
/* get_auc_roc :29-44 (roc_curve + auc; ties count one half, NaN with one
 * class) and get_auc_prc :97-116 (trapezoid over precision_recall_curve's
 * points): out[4] = auroc, aupr, n_pos, n_neg. */
size_t mmad_rank_metrics_ws_bytes(int64_t n);
int mmad_rank_metrics(int64_t n, const float* score, const uint8_t* label, double* out, void* ws,
                      size_t ws_bytes, void* stream);
/* get_f1_score :118-130 (threshold = np.quantile(valid, q), linear rule;
 * prediction test > threshold) and get_confusion_matrix :83-95 (test >=
 * threshold): out[10] = threshold, f1, p, r, precision, recall, tp, fp, fn,
 * tn (undefined ratios are NaN, as numpy's 0/0). */
size_t mmad_threshold_metrics_ws_bytes(int64_t n_valid);
int mmad_threshold_metrics(int64_t n_valid, const float* valid, int64_t n_test, const float* test,
                           const uint8_t* label, double q, double* out, void* ws, size_t ws_bytes,
                           void* stream);

/* HSR_Net multimodal fusion producer (utils/data_loaders.py:152-229; replaces
 * the per-window loop HSR_Net.forward :179-229 that TabularDataset runs at
 * :400-424).  One call fuses n windows.  Inputs fp32 device rows, each
 * nullable: r [n][3*32*32] (hand RGB), d [n][32*32] (head depth), t [n] (F/T
 * scalar), m [n][13] (MFCCs).  weights: fp32 [mmad_hsr_weight_count()] packed
 * conv1r w,b | conv2r | conv3r | conv1d | conv2d | conv3d | conv1l | conv2l
 * (torch layouts [co][ci][k..]).  unimodal == 0: r, d, t, m all required, row =
 * channel-major [27][8][8] = rgb 1024 | depth 512 | F/T 64 | mic 128 (1728);
 * unimodal != 0: the block of the last non-null modality of (r, d, t, m)
 * alone, as the reference keeps (:190-221).  out fp32 [n][ld_out]; columns
 * past the row width are not written.  The LiDAR branch (l) is never fed by
 * the reference and has no entry point. */
int mmad_hsr_weight_count(void);
int mmad_hsr_fuse(int n, const float* r, const float* d, const float* t, const float* m,
                  const float* weights, int unimodal, float* out, int ld_out, void* stream);

/* Sensor-stream normalisation of the dataset ingest (TabularDataset,
 * utils/data_loaders.py:233-434): norm_vec_np (:447-456) = per column
 * (v - min) / (max - min) over the n windows in float64, NaN (constant
 * column) -> 0, cast to fp32 -- for the hand-camera / head-depth pixel arrays
 * (:338-378), the F/T weight (:380-385) and the MFCCs (:386-394).
 * v: device [n][F] of type vtype (MMAD_SRC_*: the PNG arrays' uint8 / uint16
 * or the CSV's float64, converted exactly inside the kernel).
 * layout MMAD_NORM_FLAT: out fp32 [n][F]; MMAD_NORM_IMG24: F = C*24*32 in the
 * reference's HWC flatten, reinterpreted [C][24][32] (its .view) and
 * nearest-upsampled to [C][32][32] (its F.interpolate(size=32)): out fp32
 * [n][C*1024], ready for mmad_hsr_fuse.  ws: mmad_minmax_norm_ws_bytes. */
#define MMAD_SRC_F64 0
#define MMAD_SRC_U8 1
#define MMAD_SRC_U16 2
#define MMAD_SRC_I32 3
#define MMAD_SRC_F32 4
#define MMAD_NORM_FLAT 0
#define MMAD_NORM_IMG24 1
size_t mmad_minmax_norm_ws_bytes(int64_t n, int F);
int mmad_minmax_norm(int64_t n, int F, const void* v, int vtype, int layout, float* out, void* ws,
                     size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMAD_H_ */
