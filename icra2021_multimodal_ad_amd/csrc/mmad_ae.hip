// Whole-autoencoder executor (mmad_ae_* in include/mmad.h).
//
// Replaces the reference's per-op Python dispatch of AutoEncoder.step /
// validate / forward (models/auto_encoder.py:36-91) and get_diffs
// (reconstruction_aggregation.py:6-37): one host call enqueues the whole
// forward + backward (+ Adam) or scoring sequence, no host syncs, no device
// allocation (caller workspace).
//
// Train-mode dataflow per hidden layer l (Linear -> LeakyReLU -> BN):
//   fwd GEMM -> a_l + Welford partials in its epilogue -> bn_fold (mean, rstd,
//   scale s, shift t, running stats; W'_{l+1} = W_{l+1} diag(s) and the
//   partial bias sum_k t[k] W_{l+1}[n][k]) -> the consumer GEMM contracts the
//   raw a_l with W'; the normalised y_l is never written to HBM.  Backward: the
//   bwd-data GEMM epilogue emits the BN-backward column partials of dy_l;
//   bn_act_bwd_apply produces dz_l; the dW GEMM against the raw a_{l-1}, fixed
//   up in its epilogue (s[k] acc + t[k] db[n]), runs on a side stream with that
//   layer's Adam update fused into the epilogue (single-GPU step), overlapping
//   the remaining backward chain on the main stream.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mmad_common.h"
#include "mmad_gemm.h"
#include "mmad_ops.h"
#include "mmad_comm.h"

#define RET_IF(x)                    \
  do {                               \
    int r_ = (x);                    \
    if (r_ != MMAD_OK) return r_;    \
  } while (0)

// Executor events only order work between streams of this device, so they
// skip the system-scope fence (L2 writeback for host visibility) that a
// default event adds at record time.  Each record still leaves a ~5 us bubble
// on the main stream (~6 us with the fence; 0.513 vs 0.521 ms/step).
// Device-scope release/acquire (the same as a kernel boundary on one stream)
// still orders the data.  Knob 27 restores the default.
static unsigned ev_flags(int sysfence) {
  return sysfence ? (unsigned)hipEventDisableTiming
                  : (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence);
}

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
  // bf16 ping-pong: the fused step's Adam writes the new weights into
  // shadow_alt while this step's backward still reads shadow, then the two
  // swap; so a dW GEMM need not wait for its layer's bwd-data GEMM
  void* shadow_alt = nullptr;
  // side stream + events for the dW / Adam overlap (created at bind time)
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> ev_fork, ev_data;
  hipEvent_t ev_join = nullptr;
  hipEvent_t ev_loss = nullptr;   // fused step: forward done -> the loss reduction on the side stream
  // the schedule, copied from the tune table at create (include/mmad.h knobs
  // 16-27): one schedule per handle, whatever the table says later
  unsigned ev_flags_ = 0;
  int loss_side = 1;      // knob 23: reduce the loss on the side stream after the forward
  int side_prio_hi = 0;   // knob 26
  // knob 15: > 0 = the side stream is created behind a CU mask that leaves
  // this many CUs (evenly spaced over the mask) to the main stream alone
  int side_cu_held = 0;
  // data-parallel step: the small bucket (bias / gamma / beta grads + loss)
  // goes on the comm stream right after the bwd-data GEMM of this layer
  // (ahead of this layer's and the lower layers' weight buckets); knob 24
  int dp_small_at = 1;
  // data-parallel step: sharded weight buckets (knob 28); master_stale: the
  // bf16 model's fp32 master weights / every model's Adam moments are
  // current only on their owning rank since the last mmad_ae_dp_sync_master
  int dp_shard = 1;
  // data-parallel step: consecutive layers' weight gradients (backward
  // order) share one exchange bucket until it holds at least dp_bucket_mib
  // MiB of fp32 gradient (knob 30; 0 = one bucket per layer)
  int dp_bucket_mib = 8;
  // data-parallel step: from this many padded rows each side-stream dW GEMM
  // is issued as soon as its own dz is complete instead of with its bucket's
  // closing layer (knob 14; 0 = one fork per bucket)
  int dp_fork_rows = 1024;
  bool master_stale = false;
  int mse_tiles = 0;   // loss partials written by the last MSE GEMM
  // data parallelism: RCCL communicator (not owned), its stream and events
  mmad_comm* comm = nullptr;
  hipStream_t cstream = nullptr;
  std::vector<hipEvent_t> ev_dw;
  // torch-exchange data parallelism (mmad_ae_dw_events): the forward+backward
  // without Adam records ev_xdw[l] after dW_l and ev_xdata[l] after bwd-data of
  // l.  System-scope fences (unlike the executor's own events): the exchange
  // may read the gradients with a copy engine, which does not see the L2
  bool dw_events = false;
  std::vector<hipEvent_t> ev_xdw, ev_xdata;
  // optional bf16 gradient exchange (mmad_ae_set_grad_bf16): n_weight bf16
  void* grad_bf16 = nullptr;
  hipEvent_t ev_small = nullptr, ev_cdone = nullptr;
  // schedule study (knob 29): every side-stream dW + Adam GEMM held until the
  // main stream has enqueued the whole bwd-data chain (ev_hold), to separate
  // the chain's in-step contention from its barrier costs
  int side_hold = 0;
  // knob 33 (ping-pong steps): the side-stream dW + Adam GEMMs of the top
  // dw_late layers fork behind the layer's bwd-data + BN apply instead of at
  // its dz, so the largest dW does not share the CUs with the apply below it
  int dw_late = 0;
  // knob 34 (ping-pong steps): each side-stream dW's fork event (dz_l ready)
  // completed by the launch that produces dz_l (the BN-backward apply or the
  // bwd-data GEMM: hipExtLaunchKernel stop event) instead of a marker packet
  // recorded on the main stream before the bwd-data GEMM of l -- each marker
  // held the main stream's next dispatch ~5 us; the top layer's fork is the
  // loss reduction's wait on the MSE launch, already on the side stream
  int fork_on_kernel = 1;
  // knob 35 (ping-pong steps): from this layer down, side-stream dW GEMMs
  // fork in pairs -- every other layer's dz gets no fork event and its dW is
  // issued with the next lower layer's (where the side stream lags the chain
  // by more than a layer anyway, each fork saved is a ~5-us hold on the
  // main stream; 0 = every layer forks)
  int fork_pair_below = 0;
  hipEvent_t ev_hold = nullptr;
  // fused step: dW GEMMs of layers < dw_main run on the caller's stream
  // (knob 19; tools/sched_sweep.py: 0.499 ms (2) vs 0.512 (1) vs 0.523 (3));
  // keep_grads (knob 25): also write dW to the grads buffer
  int dw_main = 2;
  // ping-pong schedule per call from this many padded rows (bf16 with a
  // shadow pair; knob 20), with dw_main_ping main-stream dW GEMMs (knob 21):
  // VIB B=4096 0.941-0.945 vs 0.995-0.999 ms/step, B=1024 0.450-0.455 vs
  // 0.442-0.449 (profiles/r02bu_*, r02bv_*)
  int pair_rows = 4096;
  int dw_main_ping = 1;
  int keep_grads = 0;
  // train-mode BN: fold the batch statistics into the consumer's weights
  // (bn_fold_k; the bf16 throughput path) or normalise the activations into y
  // (bn_train_apply_k; the exact-fp32 parity path: folding contracts the raw,
  // un-centred activations and cancels the mean back out, which costs the
  // fp32 path ~10x the reference's rounding error on BN-producer layers).
  // Set at create from the dtype and knob 16.
  int fold = 1;
  // train-mode BN inside the producing GEMM (bn_mode 2, MMAD_BN_MODE): the
  // forward GEMM's epilogue finishes the batch statistics and writes y, the
  // bwd-data GEMM's epilogue writes dz (a per-column-tile barrier between the
  // blocks of one column, mmad_gemm_mfma.hip) -- no finalize / fold / apply
  // launches.  Layers whose grid cannot be co-resident fall back to mode 0
  // (apply kernels).  0 = apply kernels, 1 = fold, 2 = fused (knob 16).  Default: bf16
  // 2 up to bn_fused_rows padded rows per call (measured: D=2048 B=1024
  // 0.495 ms/step fused vs 0.531 apply vs 0.536 fold; B=4096 VIB 1.33 fused
  // vs 1.32 apply vs 1.27 fold -- more tiles per column, longer barrier
  // waits), fold above; fp32 0 (the parity path).
  int bn_mode = 0;
  // backward BN schedule override for the bf16 path (knob 17: -1 =
  // the forward's; 2 = fused into the bwd-data GEMMs whatever the forward did:
  // the fused backward needs only a, the saved mean / rstd and gamma, which
  // every forward schedule leaves)
  int bn_mode_bwd = -1;
  int bn_fused_rows = 2048;   // knob 18
  // fused step: record the "bwd-data of l done" event only every ev_every-th
  // side-stream layer (each record costs a bubble on the main stream); the dW
  // GEMMs of the layers in between wait for the next recorded one (knob 22;
  // c2 0.435-0.440 vs 0.442-0.444 with 1, profiles/r02bv_*)
  int ev_every = 2;
  // the main stream's hand-off events (bwd-data -> side-stream dW, MSE ->
  // side-stream loss) completed by the GEMM launch itself (knob 31)
  int ev_on_kernel = 1;
  // hipGraph cache for mmad_ae_score_stream: one captured graph per
  // (input, output, workspace, N, batch) pass, replayed with one launch
  struct ScoreGraph {
    const float* x; int64_t ld_x, N; int batch; float* sq; int64_t ld_sq; void* ws;
    const void* wts;   // weight operand base (the bf16 shadow may be re-pointed)
    hipGraphExec_t exec;
  };
  std::vector<ScoreGraph> graphs;
  hipStream_t gstream = nullptr;   // capture stream (the caller's may be the null stream)
  // kernel probe (mmad_ae_probe): timing events around ONE GEMM launch of
  // the step, on the stream it is launched on (bench roofline, in situ)
  mutable int probe_id = -1;
  mutable int probe_n = 0;
  mutable unsigned probe_mask = 0;    // layers the last probed launch covered (bit l)
  std::vector<hipEvent_t> probe_ev;   // [2 * capacity]: start, end pairs
  hipEvent_t probe_sync = nullptr;    // a main-stream probe's start waits for the side stream
  // probe kinds 2 / 3: the events ride on the launch itself (hipExtLaunchKernel
  // start / stop: the kernel's own start and end, as rocprofv3's kernel records)
  // and nothing waits for the side stream -- the launch as it runs in the
  // step's schedule, so the probe can stay on through a timed region
  bool probe_kev = false;
  // hipGraph-captured fused train steps (mmad_ae_train_step_graph): one per
  // call signature, replayed after a host->device copy of the per-call values
  // (a ring of pinned host slots, each reused only once its copy has run)
  struct TrainGraph {
    int B, k, ld_x, xvec, has_eps, dw_main, ev_every, keep_grads;
    const void* ws;
    const void* shadow;   // the bf16 shadow the captured kernels read / write
    float beta_kl, b1, b2, aeps;
    hipGraphExec_t exec;
  };
  std::vector<TrainGraph> tgraphs;
  static constexpr int kDynSlots = 64;
  MmadDyn* dyn_host = nullptr;
  hipEvent_t dyn_ev[kDynSlots] = {};
  bool dyn_used[kDynSlots] = {};
  int dyn_next = 0;
  bool capturing = false;
  bool graph_broken = false;
  // workspace whose split-K control block this handle has zeroed
  const void* ws_zeroed = nullptr;
  void clear_train_graphs() {
    for (auto& g : tgraphs) (void)hipGraphExecDestroy(g.exec);
    tgraphs.clear();
  }
  ~mmad_ae() {
    clear_train_graphs();
    for (auto e : dyn_ev)
      if (e) (void)hipEventDestroy(e);
    if (dyn_host) (void)hipHostFree(dyn_host);
    for (auto e : probe_ev) (void)hipEventDestroy(e);
    if (probe_sync) (void)hipEventDestroy(probe_sync);
    for (auto& g : graphs) (void)hipGraphExecDestroy(g.exec);
    if (gstream) (void)hipStreamDestroy(gstream);
    for (auto e : ev_fork) (void)hipEventDestroy(e);
    for (auto e : ev_data) (void)hipEventDestroy(e);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (ev_hold) (void)hipEventDestroy(ev_hold);
    if (ev_loss) (void)hipEventDestroy(ev_loss);
    for (auto e : ev_dw) (void)hipEventDestroy(e);
    for (auto e : ev_xdw) (void)hipEventDestroy(e);
    for (auto e : ev_xdata) (void)hipEventDestroy(e);
    if (ev_small) (void)hipEventDestroy(ev_small);
    if (ev_cdone) (void)hipEventDestroy(ev_cdone);
    if (cstream) (void)hipStreamDestroy(cstream);
    if (side) (void)hipStreamDestroy(side);
  }
};

struct LayerWS {
  void *out, *y, *dy, *dz;
  float *stats, *mean, *rstd, *scale, *shift, *dbpart, *rowsq;
  double* bnpart;   // fp64 BN-backward column partials [Mp/64][2][Np]
  // consumer of a train-mode BN producer: W*scale (GEMM dtype) and the
  // per-64-column partials of sum_k shift[k] W[n][k]
  void* wf;
  float* cpart;
  // this call: BN of the layer fused into its forward GEMM / into the
  // bwd-data GEMM of the next layer (bias gradient partials per 64 rows)
  bool fwd_fused, bwd_fused;
  unsigned* sync_f;   // fused-BN barrier counters (MMAD_BN_SYNC_WORDS each)
  unsigned* sync_b;
};
struct AeWS {
  int B, k, Mpe, Mpd;
  MmadDyn* dyn_dev = nullptr;    // device slot for the per-call values (graph-captured step)
  const MmadDyn* dyn = nullptr;  // set: kernels read x / loss / noise / Adam terms from dyn_dev
  void *xin, *zbuf, *dzin;
  float *eps, *klpart, *misc, *lossp;
  int64_t kl_parts;
  // split-K workspace per stream (0 = caller's stream, 1 = side stream);
  // the two control blocks are contiguous (one memset per call)
  float* sk_slab[2];
  unsigned* sk_ctl[2];
  size_t sk_ctl_bytes;   // both split-K control blocks + the fused-BN counters
  unsigned* bn_err;      // fused-BN barrier timeout word
  int bn_mode;           // this call's train-mode BN schedule (0 apply, 1 fold, 2 fused)
  int bn_mode_bwd;       // ... of the backward (2: fused into the bwd-data GEMMs; else the apply kernel)
  // this call's fused-step schedule: ping-pong the bf16 weight shadows (the
  // Adam of layer l writes the shadow the NEXT step reads, so dW_l waits only
  // for dz_l) and how many of the last dW GEMMs run on the main stream
  bool ping = false;
  int dw_main = 2;
  std::vector<LayerWS> l;
  int64_t bytes;
};

static size_t esz(int dtype) { return dtype == MMAD_BF16 ? 2 : 4; }

// can the dispatcher choose a split-K factor > 1 for this handle's GEMMs?
// (any dtype: a forced override, knob 4; bf16: the dW rule, when a dW
// override or the dW split target is set; fp32: knob 32's dW rule -- by
// default nothing splits)
static bool splitk_possible(int dtype) {
  const int o = mmad_splitk_override();
  if (o > 1) return true;
  if (o == 1) return false;
  if (dtype != MMAD_BF16) return mmad_splitk_dw_f32_blocks() > 0;
  return mmad_splitk_dw_override() > 1 || mmad_splitk_dw_blocks() > 0;
}

static void carve(const mmad_ae* h, int B, int k, char* base, AeWS& w) {
  int64_t off = 0;
  auto take = [&](int64_t bytes) -> char* {
    off = (off + 255) / 256 * 256;
    char* p = base ? base + off : nullptr;
    off += bytes;
    return p;
  };
  const size_t es = esz(h->dtype);
  {
    // split-K control words first: at a batch-independent offset, so
    // mmad_ae_status can find them whatever batch the last call used
    size_t slab = 0, ctl = 0;
    mmad_gemm_splitk_bytes(0, 0, &slab, &ctl);
    ctl = (ctl + 255) / 256 * 256;
    // + fused-BN barrier counters: 2 blocks per layer, then the error word
    const size_t bn_ctl = ((size_t)(2 * h->L.size() * MMAD_BN_SYNC_WORDS + 64) * 4 + 255) / 256 * 256;
    w.sk_ctl_bytes = 2 * ctl + bn_ctl;
    char* c = take((int64_t)w.sk_ctl_bytes);
    w.sk_ctl[0] = (unsigned*)c;
    w.sk_ctl[1] = c ? (unsigned*)(c + ctl) : nullptr;
    unsigned* bc = c ? (unsigned*)(c + 2 * ctl) : nullptr;
    w.bn_err = bc ? bc + 2 * h->L.size() * MMAD_BN_SYNC_WORDS : nullptr;
    w.l.resize(h->L.size());
    for (size_t i = 0; i < h->L.size(); ++i) {
      w.l[i].sync_f = bc ? bc + (2 * i) * MMAD_BN_SYNC_WORDS : nullptr;
      w.l[i].sync_b = bc ? bc + (2 * i + 1) * MMAD_BN_SYNC_WORDS : nullptr;
      w.l[i].fwd_fused = w.l[i].bwd_fused = false;
    }
  }
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
  w.dyn_dev = (MmadDyn*)take(sizeof(MmadDyn));
  w.dyn = nullptr;
  {
    // the split-K partial slabs (54.5 MB per stream) only when the current
    // knobs let the dispatcher split one of this handle's GEMMs; without a
    // slab it never splits.  Sized per call from the knobs in force, so a
    // later override grows the workspace the next size query reports (and a
    // caller that skipped the query gets "workspace too small", not an overrun)
    size_t slab = 0, ctl = 0;
    if (splitk_possible(h->dtype)) mmad_gemm_splitk_bytes(0, 0, &slab, &ctl);
    w.sk_slab[0] = slab ? (float*)take((int64_t)slab) : nullptr;
    w.sk_slab[1] = slab ? (float*)take((int64_t)slab) : nullptr;
  }
  {
    const AeLayer& last = h->L[nL - 1];
    w.lossp = (float*)take((int64_t)(w.Mpd / 64) * (last.Np / 64) * 4);
  }
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
    s.scale = (float*)take(a.Np * 4);
    s.shift = (float*)take(a.Np * 4);
    s.bnpart = (double*)take((int64_t)(Mp / 64) * 2 * a.Np * 8);
    s.dbpart = (float*)take((int64_t)(Mp / 64) * a.Np * 4);   // 128-row (apply) or 64-row (fused) parts
    s.rowsq = (float*)take((int64_t)(a.Np / 128) * Mp * 4);
    const bool folded = i > 0 && h->L[i - 1].bn;
    s.wf = folded ? take((int64_t)a.Np * a.Kp * es) : nullptr;
    s.cpart = folded ? (float*)take((int64_t)(a.Kp / 64) * a.Np * 4) : nullptr;
  }
  w.bytes = (off + 255) / 256 * 256;
}

// ---------------------------------------------------------------------------
int mmad_ae_create(mmad_ae** out, int dtype, int n_enc, const int* enc_widths, int n_dec,
                   const int* dec_widths, int vib, float slope, float bn_eps, float bn_momentum) {
  MMAD_CHECK_ARG(out != nullptr, "ae_create: null out");
  *out = nullptr;
  MMAD_CHECK_ARG(dtype == MMAD_F32 || dtype == MMAD_BF16, "ae_create: bad dtype %d", dtype);
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
  {
    // the schedule knobs (include/mmad.h 16-27), read once for this handle
    const int m = mmad_knob(16);
    h->fold = dtype == MMAD_BF16;
    h->bn_mode = dtype == MMAD_BF16 ? 2 : 0;
    if (m >= 0 && m <= 2) {
      h->bn_mode = m;
      h->fold = m != 0 && dtype == MMAD_BF16;   // fold: mode 1, mode 2's fallback
    }
    h->bn_mode_bwd = mmad_knob(17);
    h->bn_fused_rows = mmad_knob(18);
    h->dw_main = mmad_knob(19);
    h->pair_rows = mmad_knob(20);
    h->dw_main_ping = mmad_knob(21);
    h->ev_every = mmad_knob(22);
    h->ev_on_kernel = mmad_knob(31);
    h->loss_side = mmad_knob(23);
    h->dp_small_at = mmad_knob(24);
    h->keep_grads = mmad_knob(25);
    h->side_prio_hi = mmad_knob(26);
    h->side_cu_held = mmad_knob(15);
    h->dp_shard = mmad_knob(28);
    h->side_hold = mmad_knob(29);
    h->dw_late = mmad_knob(33);
    h->fork_on_kernel = mmad_knob(34);
    h->fork_pair_below = mmad_knob(35);
    h->dp_bucket_mib = mmad_knob(30) < 0 ? 0 : mmad_knob(30);
    h->dp_fork_rows = mmad_knob(14);
    h->ev_flags_ = ev_flags(mmad_knob(27));
  }
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
  h->clear_train_graphs();   // captured steps bake the buffer addresses in
  h->params = params;
  h->grads = grads;
  h->m = adam_m;
  h->v = adam_v;
  h->shadow = shadow;
  h->running = running;
  if (!h->side) {
    // lowest priority: the side stream fills CUs the critical chain leaves idle
    int least = 0, greatest = 0;
    MMAD_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    // (knob 26: the highest priority instead, for schedule sweeps)
    if (h->side_cu_held > 0) {
      // schedule study: the side stream's dW + Adam GEMMs kept off side_cu_held
      // CUs so the bwd-data / BN-apply chain always has CUs of its own.  The
      // masked stream is created blocking at the default priority (the API
      // takes neither), so the caller's stream must be a created non-blocking
      // one, not the legacy null stream, or every side launch serialises
      int dev = 0, ncu = 0;
      MMAD_HIP_CHECK(hipGetDevice(&dev));
      MMAD_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      const int held = std::min(h->side_cu_held, ncu - 1), stride = std::max(1, ncu / std::max(1, held));
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int i = 0, n_held = 0; i < ncu; ++i) {
        const bool hold = n_held < held && i % stride == stride - 1;
        n_held += hold;
        if (!hold) mask[i / 32] |= 1u << (i % 32);
      }
      MMAD_HIP_CHECK(hipExtStreamCreateWithCUMask(&h->side, (uint32_t)mask.size(), mask.data()));
    } else {
      MMAD_HIP_CHECK(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking,
                                                 h->side_prio_hi ? greatest : least));
    }
    const size_t n = h->L.size();
    h->ev_fork.resize(n);
    h->ev_data.resize(n);
    for (size_t i = 0; i < n; ++i) {
      MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_fork[i], h->ev_flags_));
      MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_data[i], h->ev_flags_));
    }
    MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_join, h->ev_flags_));
    MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_hold, h->ev_flags_));
    MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_loss, h->ev_flags_));
  }
  return MMAD_OK;
}

int mmad_ae_set_shadow_pair(mmad_ae* h, void* alt) {
  MMAD_CHECK_ARG(h && h->params, "ae_set_shadow_pair: unbound");
  MMAD_CHECK_ARG(!alt || h->dtype == MMAD_BF16, "ae_set_shadow_pair: bf16 handles only");
  MMAD_CHECK_ARG(alt != h->shadow, "ae_set_shadow_pair: alt aliases the shadow");
  h->shadow_alt = alt;
  return MMAD_OK;
}

const void* mmad_ae_current_shadow(const mmad_ae* h) { return h ? h->shadow : nullptr; }

int mmad_ae_sync_shadow(mmad_ae* h, void* stream) {
  MMAD_CHECK_ARG(h && h->params, "ae_sync_shadow: unbound");
  if (h->dtype != MMAD_BF16) return MMAD_OK;
  if (h->shadow_alt) RET_IF(mmad_to_bf16(h->n_weight, h->params, h->shadow_alt, stream));
  return mmad_to_bf16(h->n_weight, h->params, h->shadow, stream);
}

// the shadow the fused step's Adam writes (bf16 only)
static void* adam_shadow(const mmad_ae* h, const AeLayer& a, bool ping) {
  if (h->dtype != MMAD_BF16) return nullptr;
  return (char*)(ping && h->shadow_alt ? h->shadow_alt : h->shadow) + a.w_off * 2;
}

// ---------------------------------------------------------------------------
static const void* weights(const mmad_ae* h, const AeLayer& a) {
  if (h->dtype == MMAD_BF16) return (const char*)h->shadow + a.w_off * 2;
  return h->params + a.w_off;
}

// input of layer l; in train mode a BN producer's output stays pre-BN (a): the
// forward reads it against the folded weights, the dW GEMM fixes up with
// (scale, shift) in its epilogue
static const void* input_of(const mmad_ae* h, const AeWS& w, int l, bool train,
                            const float** scale, const float** shift) {
  *scale = *shift = nullptr;
  if (l == 0) return w.xin;
  if (h->vib && l == h->n_enc) return w.zbuf;
  const AeLayer& p = h->L[l - 1];
  const LayerWS& ps = w.l[l - 1];
  if (!p.bn) return ps.out;
  if (!train || w.bn_mode != 1) return ps.y;
  *scale = ps.scale;
  *shift = ps.shift;
  return ps.out;
}


static int prepare_ws(const mmad_ae* h, int B, int k, void* ws, int64_t ws_bytes, AeWS& w,
                      hipStream_t st) {
  MMAD_CHECK_ARG(B >= 1 && k >= 1, "bad batch B=%d k=%d", B, k);
  MMAD_CHECK_ARG(h->vib || k == 1, "k>1 needs the VIB head");
  carve(h, B, k, (char*)ws, w);
  MMAD_CHECK_ARG(ws && ws_bytes >= w.bytes, "workspace too small (%lld < %lld bytes)",
                 (long long)ws_bytes, (long long)w.bytes);
  MMAD_CHECK_ARG(((uintptr_t)ws) % 256 == 0, "workspace must be 256-byte aligned");
  // split-K arrival counters / flags must be zero before a split GEMM runs;
  // every split GEMM leaves them zero again, so a workspace is zeroed once
  // when this handle first sees it (and mmad_ae_status re-zeroes after a
  // timed-out combine); only when a split can be chosen at all
  w.bn_mode = h->bn_mode;
  w.ping = false;
  w.dw_main = h->dw_main;
  if (w.bn_mode == 2 && w.Mpd > h->bn_fused_rows) w.bn_mode = h->fold ? 1 : 0;
  if (w.bn_mode == 1 && !h->fold) w.bn_mode = 0;
  w.bn_mode_bwd = (h->bn_mode_bwd >= 0 && h->fold) ? h->bn_mode_bwd : w.bn_mode;
  if ((splitk_possible(h->dtype) || h->bn_mode == 2 || h->bn_mode_bwd == 2) &&
      ws != h->ws_zeroed) {
    MMAD_HIP_CHECK(hipMemsetAsync(w.sk_ctl[0], 0, w.sk_ctl_bytes, st));
    const_cast<mmad_ae*>(h)->ws_zeroed = ws;
  }
  return MMAD_OK;
}

// probe ids: PROBE_FWD + layer (forward / MSE / score GEMM of the layer),
// PROBE_DW + layer (its dW GEMM, with the fused Adam in the fused step)
enum { PROBE_FWD = 0, PROBE_DW = 64 };

// GEMM dispatch with the split-K workspace of the stream it runs on
// data-parallel weight buckets: walking the layers in backward order,
// consecutive layers join one bucket until it holds >= dp_bucket_mib MiB of
// fp32 gradient (layer 0 always closes the last).  The weights are one
// contiguous buffer in layer order, so a bucket of layers l_lo..l_hi is the
// range [w_off(l_lo), w_off(l_hi) + Np * Kp).  Fewer, larger buckets: fewer
// exchange calls and events on the host (the DP step was host-bound with one
// bucket per layer, profiles/r03z_*) and larger collectives.  The step and
// mmad_ae_dp_sync_master use the same plan; a sharded bucket's rank-r slice is
// [r * n / N, (r + 1) * n / N).  last_of[l] = the bucket whose lowest layer is
// l (-1 if none).
struct DpBucket {
  int l_hi, l_lo;
  int64_t off, n;
};
static void dp_plan(const mmad_ae* h, std::vector<DpBucket>& out) {
  out.clear();
  const int nL = (int)h->L.size();
  const int64_t min_n = (int64_t)h->dp_bucket_mib * (1 << 20) / 4;
  int hi = nL - 1;
  int64_t acc = 0;
  for (int l = nL - 1; l >= 0; --l) {
    acc += (int64_t)h->L[l].Np * h->L[l].Kp;
    if (acc >= min_n || l == 0) {
      out.push_back(DpBucket{hi, l, h->L[l].w_off, acc});
      hi = l - 1;
      acc = 0;
    }
  }
}

static int ae_gemm(const mmad_ae* h, const AeWS& w, int dt, int epi, const void* A, int lda,
                   const void* B, int ldb, int Mp, int Np, int K, GemmEpi ep, hipStream_t s,
                   int* cfg = nullptr, int probe = -1) {
  const int r = (h->side && s == h->side) ? 1 : 0;
  ep.sk_slab = w.sk_slab[r];
  ep.sk_ctl = w.sk_ctl[r];
  const bool rec = probe >= 0 && probe == h->probe_id && !h->capturing &&
                   2 * h->probe_n < (int)h->probe_ev.size();
  if (rec && !h->probe_kev && h->side && s != h->side && h->probe_sync) {
    // a probed main-stream launch starts its clock once the side stream's
    // earlier GEMMs are done: its blocks (a whole CU's LDS each on the tail
    // tiles) wait for those CUs anyway, and the event pair then brackets the
    // launch's own execution, first dispatch to completion, as rocprofv3's
    // kernel records do (without it the pair also held ~4 us of that wait on
    // the c2 tail: 31.2 vs 26.8 us, profiles/r08o_prof_c2)
    MMAD_HIP_CHECK(hipEventRecord(h->probe_sync, h->side));
    MMAD_HIP_CHECK(hipStreamWaitEvent(s, h->probe_sync, 0));
  }
  // kernel-attached events only where the launch carries no hand-off event
  const bool kev = rec && h->probe_kev && !ep.done_ev;
  if (kev) {
    ep.start_ev = h->probe_ev[2 * h->probe_n];
    ep.done_ev = h->probe_ev[2 * h->probe_n + 1];
  } else if (rec) {
    MMAD_HIP_CHECK(hipEventRecord(h->probe_ev[2 * h->probe_n], s));
  }
  const int rc = mmad_gemm_dispatch(dt, epi, A, lda, B, ldb, Mp, Np, K, ep, s, cfg);
  if (rc != MMAD_OK) return rc;
  if (rec) {
    if (!kev) MMAD_HIP_CHECK(hipEventRecord(h->probe_ev[2 * h->probe_n + 1], s));
    ++h->probe_n;
    h->probe_mask = 1u << (probe % 64);
  }
  return MMAD_OK;
}

static inline int rows_of(const AeWS& w, const AeLayer& a) { return a.enc ? w.B : w.B * w.k; }
static inline int prows_of(const AeWS& w, const AeLayer& a) { return a.enc ? w.Mpe : w.Mpd; }
static float* running_mean(const mmad_ae* h, const AeLayer& a) { return h->running + a.bn_off; }
static float* running_var(const mmad_ae* h, const AeLayer& a) {
  return h->running + h->n_bn + a.bn_off;
}

static GemmEpi fwd_epi(const mmad_ae* h, const AeWS& w, const AeLayer& a, const LayerWS& s,
                       int M, void* out, bool folded) {
  GemmEpi ep{};
  ep.M = M;
  ep.N = a.N;
  ep.out = out;
  ep.ldo = a.Np;
  ep.bias = h->params + a.b_off;
  ep.act = a.act;
  ep.slope = h->slope;
  ep.ldpart = a.Np;
  if (folded) {
    ep.bpart = s.cpart;
    ep.bparts = a.Kp / 64;
    ep.bpstride = a.Np;
  }
  (void)w;
  return ep;
}

// mode 0 = train (MSE-fused last layer), 1 = eval, 2 = train BN, plain last layer
// mse_done (nullable): an event the train-mode MSE GEMM launch completes itself
static int run_forward(mmad_ae* h, AeWS& w, const float* x, int ld_x, int mode, const float* eps,
                       uint64_t seed, uint64_t offset, hipStream_t st, hipEvent_t mse_done = nullptr) {
  const int dt = h->dtype;
  const int nL = (int)h->L.size();
  const int B = w.B, k = w.k;
  const bool train = mode != 1;
  RET_IF(mmad_pack_input_dyn(dt, B, h->L[0].K, w.Mpe, h->L[0].Kp, x, ld_x, w.xin, w.dyn, st));
  for (int l = 0; l < nL; ++l) {
    const AeLayer& a = h->L[l];
    LayerWS& s = w.l[l];
    const int M = rows_of(w, a), Mp = prows_of(w, a);
    const float *isc, *ish;
    const void* in = input_of(h, w, l, train, &isc, &ish);
    const bool folded = isc != nullptr;             // train mode, BN producer
    const void* wt = folded ? s.wf : weights(h, a);
    if (mode == 0 && l == nL - 1) {
      GemmEpi ep = fwd_epi(h, w, a, s, M, s.out, folded);
      ep.act = MMAD_ACT_NONE;
      ep.part = s.stats;
      ep.target = x;
      ep.ldt = ld_x;
      ep.tmod = B;
      ep.gscale = 2.0f / (float)k;
      ep.lossp = w.lossp;
      ep.dyn = w.dyn;
      ep.done_ev = mse_done;
      int cfg = 0;
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_MSE, in, a.Kp, wt, a.Kp, Mp, a.Np, a.Kp, ep, st, &cfg,
                     PROBE_FWD + l));
      h->mse_tiles = mmad_gemm_ntiles(cfg, Mp, a.Np);
    } else if (a.bn && train) {
      GemmEpi ep = fwd_epi(h, w, a, s, M, s.out, folded);
      ep.part = s.stats;
      s.fwd_fused = w.bn_mode == 2 && mmad_gemm_bn_fusable(dt, GEMM_EPI_FWD, Mp, a.Np);
      if (s.fwd_fused) {
        // BN finished inside the GEMM: a (for the backward) and y = BN(a)
        ep.bn_sync = s.sync_f;
        ep.bn_err = w.bn_err;
        ep.bn_gamma = h->params + a.g_off;
        ep.bn_beta = h->params + a.be_off;
        ep.bn_rmean = running_mean(h, a);
        ep.bn_rvar = running_var(h, a);
        ep.bn_mom = h->bn_mom;
        ep.bn_eps = h->bn_eps;
        ep.bn_save_mean = s.mean;
        ep.bn_save_rstd = s.rstd;
        ep.bn_y = s.y;
      }
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_FWD, in, a.Kp, wt, a.Kp, Mp, a.Np, a.Kp, ep, st, nullptr,
                     PROBE_FWD + l));
      if (s.fwd_fused) {
        // nothing left to launch
      } else if (w.bn_mode != 1) {
        // exact-fp32 path: normalise into y (the consumer GEMM and its dW read
        // y as the reference's layers do: no fold, no fix-up cancellation)
        RET_IF(mmad_bn_train_apply(dt, M, a.N, Mp, a.Np, s.out, s.stats, h->params + a.g_off,
                                   h->params + a.be_off, running_mean(h, a), running_var(h, a),
                                   h->bn_mom, h->bn_eps, s.mean, s.rstd, s.y, st));
      } else if (l + 1 < nL) {
        // statistics -> (scale, shift) -> folded into layer l+1's weights/bias
        const AeLayer& c = h->L[l + 1];
        LayerWS& cs = w.l[l + 1];
        RET_IF(mmad_bn_finalize_fold(dt, M, a.N, Mp, a.Np, s.stats, h->params + a.g_off,
                                     h->params + a.be_off, running_mean(h, a), running_var(h, a),
                                     h->bn_mom, h->bn_eps, s.mean, s.rstd, s.scale, s.shift,
                                     h->params + c.w_off, c.Np, cs.wf, cs.cpart, st));
      } else {
        RET_IF(mmad_bn_finalize(M, a.N, Mp, a.Np, s.stats, h->params + a.g_off,
                                h->params + a.be_off, running_mean(h, a), running_var(h, a),
                                h->bn_mom, h->bn_eps, s.mean, s.rstd, s.scale, s.shift, st));
      }
    } else if (a.bn) {
      RET_IF(mmad_bn_eval_affine(a.N, a.Np, h->params + a.g_off, h->params + a.be_off,
                                 running_mean(h, a), running_var(h, a), h->bn_eps, s.scale,
                                 s.shift, st));
      GemmEpi ep = fwd_epi(h, w, a, s, M, s.y, folded);
      ep.bn_scale = s.scale;
      ep.bn_shift = s.shift;
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_FWD, in, a.Kp, wt, a.Kp, Mp, a.Np, a.Kp, ep, st, nullptr,
                     PROBE_FWD + l));
    } else {
      GemmEpi ep = fwd_epi(h, w, a, s, M, s.out, folded);
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_FWD, in, a.Kp, wt, a.Kp, Mp, a.Np, a.Kp, ep, st, nullptr,
                     PROBE_FWD + l));
    }
    if (h->vib && l == h->n_enc - 1) {
      const AeLayer& d0 = h->L[h->n_enc];
      RET_IF(mmad_vib_reparam_fwd_dyn(dt, B, h->btl, k, s.out, a.Np, eps, w.eps, seed, offset,
                                      mode == 1 ? 1 : 0, w.zbuf, d0.Kp,
                                      mode == 0 ? w.klpart : nullptr, mode == 0 ? w.dyn : nullptr, st));
    }
  }
  return MMAD_OK;
}

// where the bias gradient partials of layer l live after the backward of l+1
struct BiasSrc { const float* src; int nparts, stride; };
static BiasSrc bias_src(const mmad_ae* h, const AeWS& w, int l, bool from_mse) {
  const AeLayer& a = h->L[l];
  const LayerWS& s = w.l[l];
  const int Mp = prows_of(w, a);
  const int nL = (int)h->L.size();
  if (l == nL - 1 && from_mse) return {s.stats, Mp / MMAD_PART_ROWS, 2 * a.Np};
  if (a.bn && s.bwd_fused) return {s.dbpart, Mp / 64, a.Np};   // fused bwd-data epilogue
  if (l == nL - 1 || a.bn || (h->vib && l == h->n_enc - 1)) return {s.dbpart, Mp / 128, a.Np};
  return {s.stats, Mp / MMAD_PART_ROWS, 2 * a.Np};  // bwd-data epilogue column sums
}

using AdamHyper = MmadAdamConsts;   // w1 = float(1 - beta1), w2 = float(1 - beta2), ...

// backward through every layer.  from_mse: the last layer's dz and bias
// partials come from the MSE-fused forward epilogue; otherwise the caller has
// packed dL/dx_hat into the last layer's dy buffer.  adam != null: each
// layer's Adam update runs on the side stream right after its dW GEMM.
struct PendingDW {
  const void *dz, *in;
  int lda, ldb, M, N, K;
  GemmEpi ep;
  int layer;
};

static int finish_reductions(mmad_ae* h, AeWS& w, bool biases, bool from_mse, float beta_kl,
                             float* loss_out, hipStream_t st);

// dp_loss (data-parallel fused step): the loss output; the bias / gamma / beta
// bucket and the loss are reduced and exchanged as soon as the backward chain
// has produced the last bias partials, ahead of layer 0's weight bucket
// side_after_mse: the side stream already waits for the MSE launch (the fused
// step's loss reduction), so the top layer's dW needs no fork of its own
static int run_backward(mmad_ae* h, AeWS& w, bool from_mse, float beta_kl, const AdamHyper* adam,
                        hipStream_t st, float* dp_loss = nullptr, bool side_after_mse = false) {
  const int dt = h->dtype;
  const int nL = (int)h->L.size();
  hipStream_t side = h->side;
  std::vector<PendingDW> pending;   // side-stream dW GEMMs waiting for a recorded event
  // ev_fork[l] completed by the launch that produced dz_l (knob 34)
  std::vector<char> fork_done(nL, 0);
  const bool fork_kev = h->fork_on_kernel && !h->capturing;
  // does layer l's side-stream dW (ping) get a fork event of its own (knob 35)?
  auto fork_ev = [&](int l) {
    const int P = h->fork_pair_below;
    if (P <= 0 || l > P || l == w.dw_main) return true;
    return (P - l) % 2 == 1;
  };
  auto forks_at_dz = [&](int l) {   // does layer l's side-stream dW fork behind dz_l (ping, not late)?
    return adam && !h->comm && w.ping && l >= w.dw_main && l < nL - h->dw_late && fork_ev(l);
  };
  std::vector<DpBucket> plan;       // data parallel: the exchange buckets (dp_plan)
  int next_bucket = 0;
  if (adam && h->comm) dp_plan(h, plan);
  // layer l's Adam terms for a dW epilogue: the weight tile's (ad_*, unless
  // weights_too is false) and the small segment [bias | gamma | beta]'s
  auto fill_adam = [&](GemmEpi& e, int l, bool weights_too) {
    const AeLayer& a = h->L[l];
    const BiasSrc bs = bias_src(h, w, l, from_mse);
    if (weights_too) {
      e.ad_p = h->params + a.w_off;
      e.ad_m = h->m + a.w_off;
      e.ad_v = h->v + a.w_off;
      e.ad_shadow = adam_shadow(h, a, w.ping);
      // the gradient is consumed by the fused Adam in registers; materialise
      // it only when asked (h->keep_grads)
      e.dw_nostore = h->keep_grads ? 0 : 1;
    }
    e.ad_w1 = adam->w1;
    e.ad_w2 = adam->w2;
    e.ad_eps = adam->eps;
    e.ad_step = adam->step_size;
    e.ad_bc2 = adam->bc2_sqrt;
    e.dyn = w.dyn;
    e.sm_p = h->params + a.b_off;
    e.sm_g = h->grads + a.b_off;
    e.sm_m = h->m + a.b_off;
    e.sm_v = h->v + a.b_off;
    e.sm_n = a.bn ? 3 * a.Np : a.Np;
    e.gb_src = bs.src;
    e.gb_parts = bs.nparts;
    e.gb_stride = bs.stride;
    e.sm_bN = a.N;
    e.sm_bNp = a.Np;
  };
  for (int l = nL - 1; l >= 0; --l) {
    const AeLayer& a = h->L[l];
    LayerWS& s = w.l[l];
    const int Mp = prows_of(w, a);
    const void* dz = (l == nL - 1) ? (from_mse ? s.out : s.dy) : (a.bn ? s.dz : s.dy);
    const float *isc, *ish;
    const void* in = input_of(h, w, l, true, &isc, &ish);
    GemmEpi dwe{};
    dwe.M = a.Np;
    dwe.N = a.Kp;
    dwe.out = h->grads + a.w_off;
    dwe.ldo = a.Kp;
    if (isc) {
      // dW against the raw producer activation, fixed up in the epilogue
      const BiasSrc gs = bias_src(h, w, l, from_mse);
      dwe.b_scale = isc;
      dwe.b_shift = ish;
      dwe.gb_src = gs.src;
      dwe.gb_parts = gs.nparts;
      dwe.gb_stride = gs.stride;
    }
    const bool dp = adam && h->comm;
    // the exchange bucket this layer closes (data parallel), if any
    const DpBucket* bk = nullptr;
    const DpBucket* cur = dp && next_bucket < (int)plan.size() ? &plan[next_bucket] : nullptr;
    if (cur && cur->l_lo == l) bk = &plan[next_bucket++];
    // ping-pong shadows (bf16): the fused Adam of dW_l writes the other
    // shadow, so dW_l may start as soon as dz_l is complete
    const bool ping = adam && !dp && w.ping && l >= w.dw_main;
    const bool late = ping && l >= nL - h->dw_late;
    // the top layer's dz is the MSE output, which the side stream has waited
    // for already (the loss reduction): no fork
    const bool fork_none = ping && !late && l == nL - 1 && from_mse && side_after_mse && fork_kev;
    if (ping && !late && !fork_none && !fork_done[l] && fork_ev(l)) {
      MMAD_HIP_CHECK(hipEventRecord(h->ev_fork[l], st));
    }
    // does the main stream record ev_data[l] (bwd-data of l done)?  Needed by
    // the DP exchange and by side-stream dW GEMMs (every ev_every-th layer;
    // the lowest side layer always records, flushing the deferred ones)
    const bool side_dw = adam && !dp && !ping && l >= w.dw_main;
    const bool rec = bk || (side_dw && (h->ev_every <= 1 || l == w.dw_main ||
                                        (l - w.dw_main) % h->ev_every == 0));
    bool ev_attached = false;   // ev_data[l] completed by the bwd-data launch (ev_on_kernel)
    if (dp) {
      // data parallel: below dp_fork_rows rows (host-bound steps, every event
      // call counts) the dW GEMMs of a bucket's layers are issued together
      // once the layer that closes it has its dz (one fork per bucket), then
      // the bucket's event
      // from dp_fork_rows rows the step is GPU-bound: a side-stream bucket's
      // dW GEMMs then start at their own dz (one fork each) instead of
      // queueing until the bucket's lowest layer
      const bool each = h->dp_fork_rows > 0 && Mp >= h->dp_fork_rows && cur &&
                        !(cur->l_hi < w.dw_main);
      if (each) {
        MMAD_HIP_CHECK(hipEventRecord(h->ev_fork[l], st));
        MMAD_HIP_CHECK(hipStreamWaitEvent(side, h->ev_fork[l], 0));
        // (a bucket whose upper layers were below the row threshold: their
        // dW GEMMs go first, so the bucket's event below covers them too)
        for (const PendingDW& q : pending)
          RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, q.dz, q.lda, q.in, q.ldb, q.M, q.N, q.K, q.ep,
                         side, nullptr, PROBE_DW + q.layer));
        pending.clear();
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, dz, a.Np, in, a.Kp, a.Np, a.Kp, Mp, dwe, side,
                       nullptr, PROBE_DW + l));
        if (bk) MMAD_HIP_CHECK(hipEventRecord(h->ev_dw[l], side));
      } else {
        pending.push_back(PendingDW{dz, in, a.Np, a.Kp, a.Np, a.Kp, Mp, dwe, l});
      }
      if (bk && !each) {
        // a bucket made only of the last dw_main layers of the chain runs its
        // dW GEMMs on the main stream, idle by then, instead of behind the
        // side stream's backlog (the exchange tail waits for them)
        const bool on_main = bk->l_hi < w.dw_main;
        hipStream_t ds = on_main ? st : side;
        if (!on_main) {
          MMAD_HIP_CHECK(hipEventRecord(h->ev_fork[l], st));
          MMAD_HIP_CHECK(hipStreamWaitEvent(side, h->ev_fork[l], 0));
        }
        for (const PendingDW& q : pending)
          RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, q.dz, q.lda, q.in, q.ldb, q.M, q.N, q.K, q.ep,
                         ds, nullptr, PROBE_DW + q.layer));
        pending.clear();
        MMAD_HIP_CHECK(hipEventRecord(h->ev_dw[l], ds));
      }
    } else if (!adam) {
      // fork: dz_l is complete on the main stream; dW_l overlaps the chain below
      MMAD_HIP_CHECK(hipEventRecord(h->ev_fork[l], st));
      MMAD_HIP_CHECK(hipStreamWaitEvent(side, h->ev_fork[l], 0));
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, dz, a.Np, in, a.Kp, a.Np, a.Kp, Mp, dwe, side,
                     nullptr, PROBE_DW + l));
      if (h->dw_events) MMAD_HIP_CHECK(hipEventRecord(h->ev_xdw[l], side));
    }
    if (l > 0) {
      const AeLayer& p = h->L[l - 1];
      LayerWS& ps = w.l[l - 1];
      const int M = rows_of(w, a);
      const int Mpp = prows_of(w, p);
      GemmEpi ep{};
      ep.M = M;
      ep.N = a.K;
      ep.ldo = a.Kp;
      ep.ldpart = a.Kp;
      // dz_{l-1} is produced below: its side-stream dW fork rides on that launch
      const bool attach = fork_kev && forks_at_dz(l - 1);
      if (h->vib && l == h->n_enc) {
        ep.out = w.dzin;
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_DATA, dz, a.Np, weights(h, a), a.Kp, Mp, a.Kp,
                                  a.Np, ep, st));
        RET_IF(mmad_vib_reparam_bwd(dt, w.B, h->btl, w.k, ps.out, p.Np, w.eps, w.dzin, a.Kp,
                                    beta_kl, ps.dy, p.Np, ps.dbpart, st));
      } else if (p.bn) {
        ep.out = ps.dy;
        ep.bn_a = ps.out;
        ep.bn_mean = ps.mean;
        ep.bn_rstd = ps.rstd;
        ep.bn_part = ps.bnpart;
        ps.bwd_fused = w.bn_mode_bwd == 2 && mmad_gemm_bn_fusable(dt, GEMM_EPI_BWD_DATA, Mp, a.Kp);
        if (ps.bwd_fused) {
          // BN + activation backward of layer l-1 inside this GEMM: dz directly
          ep.out = nullptr;
          ep.bn_sync = ps.sync_b;
          ep.bn_err = w.bn_err;
          ep.bn_gamma = h->params + p.g_off;
          ep.bn_dz = ps.dz;
          ep.bn_dgamma = h->grads + p.g_off;
          ep.bn_dbeta = h->grads + p.be_off;
          ep.bn_dbpart = ps.dbpart;
          ep.bn_act = p.act;
          ep.slope = h->slope;
        }
        if (rec && h->ev_on_kernel && !h->capturing) {
          ep.done_ev = h->ev_data[l];
          ev_attached = true;
        }
        if (attach && ps.bwd_fused && !ep.done_ev) {
          ep.done_ev = h->ev_fork[l - 1];
          fork_done[l - 1] = 1;
        }
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_DATA, dz, a.Np, weights(h, a), a.Kp, Mp, a.Kp,
                                  a.Np, ep, st));
        if (rec && !ev_attached) MMAD_HIP_CHECK(hipEventRecord(h->ev_data[l], st));
        if (!ps.bwd_fused) {
          RET_IF(mmad_bn_act_bwd_apply_ev(dt, p.act, h->slope, rows_of(w, p), p.N, Mpp, p.Np, ps.dy,
                                          ps.out, ps.mean, ps.rstd, h->params + p.g_off, ps.bnpart,
                                          Mpp / 64, ps.dz, h->grads + p.g_off, h->grads + p.be_off,
                                          ps.dbpart, st, attach ? h->ev_fork[l - 1] : nullptr));
          if (attach) fork_done[l - 1] = 1;
        }
      } else {
        ep.out = ps.dy;
        ep.part = ps.stats;
        if (rec && h->ev_on_kernel && !h->capturing) {
          ep.done_ev = h->ev_data[l];
          ev_attached = true;
        }
        if (attach && !ep.done_ev) {
          ep.done_ev = h->ev_fork[l - 1];
          fork_done[l - 1] = 1;
        }
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_DATA, dz, a.Np, weights(h, a), a.Kp, Mp, a.Kp,
                                  a.Np, ep, st));
      }
    }
    // torch exchange: W_l is read for the last time by the bwd-data of l
    if (!adam && h->dw_events && l > 0) MMAD_HIP_CHECK(hipEventRecord(h->ev_xdata[l], st));
    if (dp && dp_loss && l == (nL > h->dp_small_at ? h->dp_small_at : 0)) {
      // the last bwd-data (l = 1, just enqueued) has produced every bias
      // partial and the loss partials are the forward's: reduce them on the
      // main stream now and queue the small bucket's exchange + Adam on the
      // comm stream ahead of layer 1's and layer 0's weight buckets, so it
      // runs while their dW GEMMs still compute instead of after them
      RET_IF(finish_reductions(h, w, true, true, beta_kl, dp_loss, st));
      MMAD_HIP_CHECK(hipEventRecord(h->ev_small, st));
      MMAD_HIP_CHECK(hipStreamWaitEvent(h->cstream, h->ev_small, 0));
      const int64_t ns = h->n_params - h->n_weight;
      RET_IF(mmad_allreduce_pair(h->comm, h->grads + h->n_weight, ns, dp_loss, 1, h->cstream));
      RET_IF(mmad_adam_w(ns, h->params + h->n_weight, h->grads + h->n_weight, h->m + h->n_weight,
                       h->v + h->n_weight, adam->w1, adam->w2, adam->eps, adam->step_size,
                       adam->bc2_sqrt, nullptr, 0, h->cstream));
    }
    if (bk) {
      // data parallel: exchange the bucket this layer closes (layers
      // bk->l_hi .. l, one contiguous weight range) on the comm stream as soon
      // as its last dW GEMM is complete, then its Adam update (which rewrites
      // the bucket's weights, so it also waits for the main stream's bwd-data
      // of layer l, the last GEMM of the chain that reads them)
      if ((l == 0 || !(h->L[l - 1].bn) || (h->vib && l == h->n_enc)) && !ev_attached)
        MMAD_HIP_CHECK(hipEventRecord(h->ev_data[l], st));
      MMAD_HIP_CHECK(hipStreamWaitEvent(h->cstream, h->ev_data[l], 0));
      const int nr = mmad_comm_size(h->comm) > 0 ? mmad_comm_size(h->comm) : 1;
      MMAD_HIP_CHECK(hipStreamWaitEvent(h->cstream, h->ev_dw[l], 0));
      {
        const int64_t n = bk->n, boff = bk->off;
        if (h->dp_shard && n % nr == 0 && (n / nr) % 4 == 0) {
          // ZeRO-1 form: reduce-scatter, Adam on this rank's shard, all-gather
          // of the updated weights the next step reads (bf16 shadow / fp32 p)
          const int64_t cnt = n / nr, off = boff + (int64_t)mmad_comm_rank(h->comm) * cnt;
          if (h->grad_bf16) {
            // bf16 on the wire: round the bucket, reduce-scatter, widen this rank's slice
            char* gb = (char*)h->grad_bf16;
            RET_IF(mmad_to_bf16(n, h->grads + boff, gb + boff * 2, h->cstream));
            RET_IF(mmad_reduce_scatter_bucket_bf16(h->comm, gb + boff * 2, n, h->cstream));
            RET_IF(mmad_from_bf16(cnt, gb + off * 2, h->grads + off, h->cstream));
          } else {
            RET_IF(mmad_reduce_scatter_bucket(h->comm, h->grads + boff, n, h->cstream));
          }
          void* sh = h->dtype == MMAD_BF16 ? (void*)((char*)h->shadow + off * 2) : nullptr;
          RET_IF(mmad_adam_w(cnt, h->params + off, h->grads + off, h->m + off, h->v + off, adam->w1,
                           adam->w2, adam->eps, adam->step_size, adam->bc2_sqrt, sh,
                           h->dtype == MMAD_BF16 ? cnt : 0, h->cstream));
          if (h->dtype == MMAD_BF16)
            RET_IF(mmad_all_gather_bucket(h->comm, (char*)h->shadow + boff * 2, n, MMAD_BF16, h->cstream));
          else
            RET_IF(mmad_all_gather_bucket(h->comm, h->params + boff, n, MMAD_F32, h->cstream));
          if (nr > 1) h->master_stale = true;
        } else {
          RET_IF(mmad_allreduce_bucket(h->comm, h->grads + boff, n, h->cstream));
          void* sh = adam_shadow(h, a, w.ping);
          RET_IF(mmad_adam_w(n, h->params + boff, h->grads + boff, h->m + boff, h->v + boff,
                           adam->w1, adam->w2, adam->eps, adam->step_size, adam->bc2_sqrt,
                           sh, h->dtype == MMAD_BF16 ? n : 0, h->cstream));
        }
      }
    } else if (adam && !dp) {
      // dW_l with this layer's Adam update fused into its epilogue.  It rewrites
      // W_l, so it starts only once the main stream has finished reading W_l
      // (bwd-data of l); the rest of the chain keeps overlapping it.
      if (rec && !ev_attached && (l == 0 || !(h->L[l - 1].bn) || (h->vib && l == h->n_enc)))
        MMAD_HIP_CHECK(hipEventRecord(h->ev_data[l], st));
      fill_adam(dwe, l, true);
      // the last dW GEMMs of the chain go to the main stream, which is idle
      // by then, instead of queueing behind the side stream's backlog
      const bool on_main = l < w.dw_main;
      if (on_main) {
        dwe.tile_force = mmad_tile_adam_main_for(a.Np, a.Kp, Mp) + 1;
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, dz, a.Np, in, a.Kp, a.Np, a.Kp, Mp, dwe, st,
                       nullptr, PROBE_DW + l));
      } else if (h->side_hold) {
        pending.push_back(PendingDW{dz, in, a.Np, a.Kp, a.Np, a.Kp, Mp, dwe, l});
      } else if (ping && !late && !fork_ev(l)) {
        // no fork of its own: issued with the next lower layer's dW
        pending.push_back(PendingDW{dz, in, a.Np, a.Kp, a.Np, a.Kp, Mp, dwe, l});
      } else if (ping) {
        if (late) MMAD_HIP_CHECK(hipEventRecord(h->ev_fork[l], st));
        if (!fork_none) MMAD_HIP_CHECK(hipStreamWaitEvent(side, h->ev_fork[l], 0));
        for (const PendingDW& q : pending)
          RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, q.dz, q.lda, q.in, q.ldb, q.M, q.N, q.K, q.ep,
                         side, nullptr, PROBE_DW + q.layer));
        pending.clear();
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, dz, a.Np, in, a.Kp, a.Np, a.Kp, Mp, dwe, side,
                       nullptr, PROBE_DW + l));
      } else if (!rec) {
        pending.push_back(PendingDW{dz, in, a.Np, a.Kp, a.Np, a.Kp, Mp, dwe, l});
      } else {
        MMAD_HIP_CHECK(hipStreamWaitEvent(side, h->ev_data[l], 0));
        for (const PendingDW& q : pending)
          RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, q.dz, q.lda, q.in, q.ldb, q.M, q.N, q.K, q.ep,
                         side, nullptr, PROBE_DW + q.layer));
        pending.clear();
        RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, dz, a.Np, in, a.Kp, a.Np, a.Kp, Mp, dwe, side,
                       nullptr, PROBE_DW + l));
      }
    }
  }
  if (h->side_hold && !pending.empty()) {
    MMAD_HIP_CHECK(hipEventRecord(h->ev_hold, st));
    MMAD_HIP_CHECK(hipStreamWaitEvent(side, h->ev_hold, 0));
    for (const PendingDW& q : pending)
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_BWD_WEIGHT, q.dz, q.lda, q.in, q.ldb, q.M, q.N, q.K, q.ep, side,
                     nullptr, PROBE_DW + q.layer));
    pending.clear();
  }
  MMAD_CHECK_ARG(pending.empty(), "ae backward: deferred dW GEMMs left unissued");
  // join the side stream back into the main stream
  MMAD_HIP_CHECK(hipEventRecord(h->ev_join, side));
  MMAD_HIP_CHECK(hipStreamWaitEvent(st, h->ev_join, 0));
  return MMAD_OK;
}

// bias grads of every layer (when Adam did not finalise them) + the loss
static int finish_reductions(mmad_ae* h, AeWS& w, bool biases, bool from_mse, float beta_kl,
                             float* loss_out, hipStream_t st) {
  MmadReduceJobs jobs{};
  int n = 0, max_np = 1;
  const int nL = (int)h->L.size();
  if (biases) {
    for (int l = 0; l < nL; ++l) {
      const AeLayer& a = h->L[l];
      const BiasSrc bs = bias_src(h, w, l, from_mse);
      MmadReduceJob& j = jobs.j[n++];
      j.src = bs.src;
      j.dst = h->grads + a.b_off;
      j.nparts = bs.nparts;
      j.stride = bs.stride;
      j.N = a.N;
      j.Np = a.Np;
      j.scale = 1.f;
      max_np = a.Np > max_np ? a.Np : max_np;
    }
  }
  if (loss_out) {
    const AeLayer& last = h->L[nL - 1];
    MmadReduceJob& j = jobs.j[n++];
    j.scalar = 1;
    j.src = w.lossp;                        // one sum of d^2 per MSE-GEMM output tile
    j.dst = loss_out;
    j.nparts = 1;
    j.stride = 0;
    j.N = h->mse_tiles;
    j.Np = j.N;
    j.scale = 1.f / (float)w.k;
    if (h->vib) {
      j.src2 = w.klpart;
      j.n2 = (int)w.kl_parts;
      j.scale2 = beta_kl;
    }
  }
  if (n == 0) return MMAD_OK;
  jobs.dyn = loss_out ? w.dyn : nullptr;
  return mmad_reduce_jobs(jobs, n, max_np, st);
}

int mmad_ae_train_fwd_bwd(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                          uint64_t seed, uint64_t offset, float beta_kl, float* loss_out,
                          void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->running, "ae_train: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && loss_out, "ae_train: bad input");
  AeWS w;
  RET_IF(prepare_ws(h, B, k, ws, ws_bytes, w, (hipStream_t)stream));
  hipStream_t st = (hipStream_t)stream;
  RET_IF(run_forward(h, w, x, ld_x, 0, eps, seed, offset, st));
  RET_IF(run_backward(h, w, true, beta_kl, nullptr, st));
  return finish_reductions(h, w, true, true, beta_kl, loss_out, st);
}

static AdamHyper adam_hyper(float lr, float b1, float b2, float eps, int step) {
  return mmad_adam_consts(lr, b1, b2, eps, step);
}

int mmad_ae_train_step(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                       uint64_t seed, uint64_t offset, float beta_kl, float lr, float beta1,
                       float beta2, float adam_eps, int step, float* loss_out, void* ws,
                       int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->running && h->m && h->v,
                 "ae_train_step: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && loss_out, "ae_train_step: bad input");
  MMAD_CHECK_ARG(step >= 1, "ae_train_step: step must be >= 1");
  AeWS w;
  RET_IF(prepare_ws(h, B, k, ws, ws_bytes, w, (hipStream_t)stream));
  hipStream_t st = (hipStream_t)stream;
  const AdamHyper ah = adam_hyper(lr, beta1, beta2, adam_eps, step);
  // ping-pong schedule (bf16 with a shadow pair, large calls, single process)
  w.ping = h->shadow_alt && !h->comm && !h->capturing && w.Mpe >= h->pair_rows;
  if (w.ping) w.dw_main = h->dw_main_ping;
  // the side stream's loss reduction waits on the MSE launch's own completion
  const bool loss_ev_on_kernel = !h->comm && h->loss_side && h->ev_on_kernel && !h->capturing;
  RET_IF(run_forward(h, w, x, ld_x, 0, eps, seed, offset, st, loss_ev_on_kernel ? h->ev_loss : nullptr));
  if (!h->comm && !h->loss_side) {
    RET_IF(run_backward(h, w, true, beta_kl, &ah, st));
    RET_IF(finish_reductions(h, w, false, true, beta_kl, loss_out, st));
    if (w.ping) std::swap(h->shadow, h->shadow_alt);
    return MMAD_OK;
  }
  if (!h->comm) {
    // the loss needs only the forward's MSE (and KL) partials: reduce it on
    // the side stream now, off the main stream's tail (the backward joins the
    // side stream back into the caller's before the step ends)
    if (!loss_ev_on_kernel) MMAD_HIP_CHECK(hipEventRecord(h->ev_loss, st));
    MMAD_HIP_CHECK(hipStreamWaitEvent(h->side, h->ev_loss, 0));
    RET_IF(finish_reductions(h, w, false, true, beta_kl, loss_out, h->side));
    RET_IF(run_backward(h, w, true, beta_kl, &ah, st, nullptr, true));
    if (w.ping) std::swap(h->shadow, h->shadow_alt);
    return MMAD_OK;
  }
  // data parallel: per-layer weight buckets and (ahead of layer 0's) the
  // small bucket [all bias | gamma | beta grads] + the loss, each with its
  // Adam, on the comm stream (run_backward); then join
  RET_IF(run_backward(h, w, true, beta_kl, &ah, st, loss_out));
  MMAD_HIP_CHECK(hipEventRecord(h->ev_cdone, h->cstream));
  MMAD_HIP_CHECK(hipStreamWaitEvent(st, h->ev_cdone, 0));
  return MMAD_OK;
}

int mmad_ae_train_step_graph(mmad_ae* h, const float* x, int ld_x, int B, int k, const float* eps,
                             uint64_t seed, uint64_t offset, float beta_kl, float lr, float beta1,
                             float beta2, float adam_eps, int step, float* loss_out, void* ws,
                             int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->running && h->m && h->v,
                 "ae_train_step_graph: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && loss_out, "ae_train_step_graph: bad input");
  MMAD_CHECK_ARG(step >= 1, "ae_train_step_graph: step must be >= 1");
  if (h->comm || h->graph_broken)   // eager schedule for these
    return mmad_ae_train_step(h, x, ld_x, B, k, eps, seed, offset, beta_kl, lr, beta1, beta2,
                              adam_eps, step, loss_out, ws, ws_bytes, stream);
  AeWS w;
  hipStream_t st = (hipStream_t)stream;
  RET_IF(prepare_ws(h, B, k, ws, ws_bytes, w, st));
  const AdamHyper ah = adam_hyper(lr, beta1, beta2, adam_eps, step);
  // this call's values -> pinned slot -> the workspace's device slot
  if (!h->dyn_host) {
    MMAD_HIP_CHECK(hipHostMalloc((void**)&h->dyn_host, sizeof(MmadDyn) * mmad_ae::kDynSlots,
                                 hipHostMallocDefault));
    for (auto& e : h->dyn_ev) MMAD_HIP_CHECK(hipEventCreateWithFlags(&e, h->ev_flags_));
  }
  const int slot = h->dyn_next;
  h->dyn_next = (slot + 1) % mmad_ae::kDynSlots;
  if (h->dyn_used[slot]) MMAD_HIP_CHECK(hipEventSynchronize(h->dyn_ev[slot]));
  MmadDyn& d = h->dyn_host[slot];
  d.x = x;
  d.loss = loss_out;
  d.eps = eps;
  d.seed = seed;
  d.offset = offset;
  d.ad_step = ah.step_size;
  d.ad_bc2 = ah.bc2_sqrt;
  MMAD_HIP_CHECK(hipMemcpyAsync(w.dyn_dev, &d, sizeof(MmadDyn), hipMemcpyHostToDevice, st));
  MMAD_HIP_CHECK(hipEventRecord(h->dyn_ev[slot], st));
  h->dyn_used[slot] = true;
  const int xvec = ((uintptr_t)x % 16 == 0 && ld_x % 4 == 0) ? 1 : 0;
  for (auto& g : h->tgraphs) {
    if (g.B == B && g.k == k && g.ld_x == ld_x && g.xvec == xvec && g.has_eps == (eps != nullptr) &&
        g.ws == ws && g.shadow == h->shadow && g.dw_main == h->dw_main && g.ev_every == h->ev_every &&
        g.keep_grads == h->keep_grads && g.beta_kl == beta_kl && g.b1 == beta1 && g.b2 == beta2 &&
        g.aeps == adam_eps) {
      MMAD_HIP_CHECK(hipGraphLaunch(g.exec, st));
      return MMAD_OK;
    }
  }
  // first call of this signature: run it eagerly (reading the same device
  // slot; this also settles every GEMM tile choice, which cannot be timed
  // under capture), then capture the identical launch sequence
  w.dyn = w.dyn_dev;
  RET_IF(run_forward(h, w, x, ld_x, 0, eps, seed, offset, st));
  RET_IF(run_backward(h, w, true, beta_kl, &ah, st));
  RET_IF(finish_reductions(h, w, false, true, beta_kl, loss_out, st));
  if (!h->gstream) MMAD_HIP_CHECK(hipStreamCreateWithFlags(&h->gstream, hipStreamNonBlocking));
  hipGraph_t graph = nullptr;
  if (hipStreamBeginCapture(h->gstream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    h->graph_broken = true;
    (void)hipGetLastError();
    return MMAD_OK;
  }
  h->capturing = true;
  int rc = run_forward(h, w, x, ld_x, 0, eps, seed, offset, h->gstream);
  if (rc == MMAD_OK) rc = run_backward(h, w, true, beta_kl, &ah, h->gstream);
  if (rc == MMAD_OK) rc = finish_reductions(h, w, false, true, beta_kl, loss_out, h->gstream);
  h->capturing = false;
  const hipError_t ec = hipStreamEndCapture(h->gstream, &graph);
  hipGraphExec_t exec = nullptr;
  hipError_t ei = hipErrorUnknown;
  if (rc == MMAD_OK && ec == hipSuccess && graph)
    ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  if (graph) (void)hipGraphDestroy(graph);
  if (rc != MMAD_OK || ec != hipSuccess || ei != hipSuccess) {
    // this step already ran eagerly; later calls stay eager
    h->graph_broken = true;
    (void)hipGetLastError();
    return MMAD_OK;
  }
  if (h->tgraphs.size() >= 16) {
    (void)hipGraphExecDestroy(h->tgraphs.front().exec);
    h->tgraphs.erase(h->tgraphs.begin());
  }
  h->tgraphs.push_back({B, k, ld_x, xvec, eps != nullptr, h->dw_main, h->ev_every, h->keep_grads, ws,
                        h->shadow, beta_kl, beta1, beta2, adam_eps, exec});
  return MMAD_OK;
}

int mmad_ae_train_graph_count(const mmad_ae* h) { return h ? (int)h->tgraphs.size() : -1; }

int mmad_ae_set_comm(mmad_ae* h, mmad_comm* c) {
  MMAD_CHECK_ARG(h, "ae_set_comm: null handle");
  MMAD_CHECK_ARG(h->side, "ae_set_comm: bind the handle first");
  MMAD_CHECK_ARG(c == h->comm || !h->master_stale,
                 "ae_set_comm: the master weights are sharded over the ranks of the attached "
                 "communicator: mmad_ae_dp_sync_master on every rank first");
  if (c && !h->cstream) {
    // highest priority: the exchange must not queue behind the dW GEMMs
    int least = 0, greatest = 0;
    MMAD_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    MMAD_HIP_CHECK(hipStreamCreateWithPriority(&h->cstream, hipStreamNonBlocking, greatest));
    // the events RCCL's reads of a bucket wait on keep the system-scope
    // fence (a transport may move the bytes with a copy engine, which does
    // not see the L2); one per bucket and step
    h->ev_dw.resize(h->L.size());
    for (auto& e : h->ev_dw) MMAD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_small, hipEventDisableTiming));
    MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->ev_cdone, h->ev_flags_));
  }
  h->comm = c;
  return MMAD_OK;
}

int mmad_ae_dp_master_stale(const mmad_ae* h) { return h && h->master_stale ? 1 : 0; }

int mmad_ae_set_grad_bf16(mmad_ae* h, void* buf) {
  MMAD_CHECK_ARG(h && h->params, "ae_set_grad_bf16: unbound handle");
  MMAD_CHECK_ARG(!buf || ((uintptr_t)buf % 16 == 0), "ae_set_grad_bf16: buffer must be 16-byte aligned");
  h->grad_bf16 = buf;
  return MMAD_OK;
}

int mmad_ae_dw_events(mmad_ae* h, int on) {
  MMAD_CHECK_ARG(h && h->side, "ae_dw_events: bind the handle first");
  if (on && h->ev_xdw.empty()) {
    h->ev_xdw.resize(h->L.size());
    h->ev_xdata.resize(h->L.size());
    for (auto& e : h->ev_xdw) MMAD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : h->ev_xdata) MMAD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  h->dw_events = on != 0;
  return MMAD_OK;
}

int mmad_ae_wait_dw(mmad_ae* h, int layer, void* stream) {
  MMAD_CHECK_ARG(h && h->dw_events, "ae_wait_dw: dW events are off (mmad_ae_dw_events)");
  MMAD_CHECK_ARG(layer >= 0 && layer < (int)h->L.size(), "ae_wait_dw: bad layer %d", layer);
  MMAD_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, h->ev_xdw[layer], 0));
  if (layer > 0) MMAD_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, h->ev_xdata[layer], 0));
  return MMAD_OK;
}

int mmad_ae_dw_plan(const mmad_ae* h, int max_n, int64_t* off, int64_t* n, int* layer_lo) {
  MMAD_CHECK_ARG(h && h->params, "ae_dw_plan: unbound handle");
  std::vector<DpBucket> plan;
  dp_plan(h, plan);
  MMAD_CHECK_ARG(max_n >= (int)plan.size() && off && n && layer_lo,
                 "ae_dw_plan: room for %d buckets needed", (int)plan.size());
  for (size_t i = 0; i < plan.size(); ++i) {
    off[i] = plan[i].off;
    n[i] = plan[i].n;
    layer_lo[i] = plan[i].l_lo;
  }
  return (int)plan.size();
}

int mmad_ae_dp_sync_master(mmad_ae* h, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->m && h->v, "ae_dp_sync_master: unbound handle");
  if (!h->comm || !h->master_stale) return MMAD_OK;
  hipStream_t st = (hipStream_t)stream;
  const int nr = mmad_comm_size(h->comm);
  std::vector<DpBucket> plan;
  dp_plan(h, plan);
  for (const DpBucket& b : plan) {
    const int64_t n = b.n, boff = b.off;
    if (!(n % nr == 0 && (n / nr) % 4 == 0)) continue;   // an all-reduced bucket: already current
    if (h->dtype == MMAD_BF16) RET_IF(mmad_all_gather_bucket(h->comm, h->params + boff, n, MMAD_F32, st));
    RET_IF(mmad_all_gather_bucket(h->comm, h->m + boff, n, MMAD_F32, st));
    RET_IF(mmad_all_gather_bucket(h->comm, h->v + boff, n, MMAD_F32, st));
  }
  h->master_stale = false;
  return MMAD_OK;
}

int mmad_ae_backward(mmad_ae* h, const float* dxhat, int ld, int B, void* ws, int64_t ws_bytes,
                     void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads, "ae_backward: unbound handle");
  MMAD_CHECK_ARG(!h->vib, "ae_backward: the VIB model trains through mmad_ae_train_fwd_bwd");
  AeWS w;
  RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w, (hipStream_t)stream));
  hipStream_t st = (hipStream_t)stream;
  const int nL = (int)h->L.size();
  const AeLayer& last = h->L[nL - 1];
  LayerWS& s = w.l[nL - 1];
  MMAD_CHECK_ARG(dxhat && ld >= last.N, "ae_backward: bad dxhat");
  RET_IF(mmad_pack_input(h->dtype, B, last.N, w.Mpd, last.Np, dxhat, ld, s.dy, st));
  RET_IF(mmad_matrix_colsum_partials(h->dtype, B, w.Mpd, last.Np, s.dy, s.dbpart, st));
  RET_IF(run_backward(h, w, false, 0.f, nullptr, st));
  return finish_reductions(h, w, true, false, 0.f, nullptr, st);
}

int mmad_ae_adam(mmad_ae* h, float lr, float beta1, float beta2, float eps, int step,
                 void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->m && h->v, "ae_adam: unbound handle");
  MMAD_CHECK_ARG(step >= 1, "ae_adam: step must be >= 1");
  const AdamHyper ah = adam_hyper(lr, beta1, beta2, eps, step);
  return mmad_adam_w(h->n_params, h->params, h->grads, h->m, h->v, ah.w1, ah.w2, eps, ah.step_size,
                   ah.bc2_sqrt, h->dtype == MMAD_BF16 ? h->shadow : nullptr,
                   h->dtype == MMAD_BF16 ? h->n_weight : 0, stream);
}

int mmad_ae_adam_range(mmad_ae* h, float lr, float beta1, float beta2, float eps, int step,
                       int64_t off, int64_t n, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->grads && h->m && h->v, "ae_adam_range: unbound handle");
  MMAD_CHECK_ARG(step >= 1, "ae_adam_range: step must be >= 1");
  MMAD_CHECK_ARG(off >= 0 && n >= 0 && off + n <= h->n_params && off % 4 == 0,
                 "ae_adam_range: bad range [%lld, +%lld)", (long long)off, (long long)n);
  const AdamHyper ah = adam_hyper(lr, beta1, beta2, eps, step);
  // the bf16 shadow covers the weights [0, n_weight)
  void* sh = nullptr;
  int64_t nsh = 0;
  if (h->dtype == MMAD_BF16 && off < h->n_weight) {
    sh = (char*)h->shadow + off * 2;
    nsh = h->n_weight - off < n ? h->n_weight - off : n;
  }
  return mmad_adam_w(n, h->params + off, h->grads + off, h->m + off, h->v + off, ah.w1, ah.w2, eps,
                   ah.step_size, ah.bc2_sqrt, sh, nsh, stream);
}

int mmad_ae_forward(mmad_ae* h, const float* x, int ld_x, int B, int train_bn, float* x_hat,
                    int ld_out, float* loss_out, void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->running, "ae_forward: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K, "ae_forward: bad input");
  AeWS w;
  RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w, (hipStream_t)stream));
  hipStream_t st = (hipStream_t)stream;
  RET_IF(run_forward(h, w, x, ld_x, train_bn ? 2 : 1, nullptr, 0x5eed, 0, st));
  const AeLayer& last = h->L.back();
  const void* xh = w.l.back().out;
  if (x_hat) RET_IF(mmad_unpack_output(h->dtype, B, last.N, last.Np, xh, x_hat, ld_out, st));
  if (loss_out) {
    RET_IF(mmad_sse_partials(h->dtype, B, last.N, last.Np, xh, x, ld_x, w.misc, 256, st));
    RET_IF(mmad_sum(256, w.misc, 1.f, loss_out, 0, st));
  }
  return MMAD_OK;
}

// one batch of the scoring pass on a prepared workspace; layer_sq row l at
// layer_sq + l*ld_sq
static int score_batch(mmad_ae* h, const float* x, int ld_x, int B, float* layer_sq,
                       int64_t ld_sq, float* diffs, AeWS& w, hipStream_t st) {
  const int dt = h->dtype;
  const int nL = (int)h->L.size();
  RET_IF(mmad_pack_input(dt, B, h->L[0].K, w.Mpe, h->L[0].Kp, x, ld_x, w.xin, st));
  int ld_diff = h->L[0].K;
  for (int e = 0; e < h->n_enc; ++e) ld_diff += h->L[e].N;
  // pass 1: eval forward; the decoder's last layer scores d0 = x_hat - x
  for (int l = 0; l < nL; ++l) {
    const AeLayer& a = h->L[l];
    LayerWS& s = w.l[l];
    const int M = rows_of(w, a), Mp = prows_of(w, a);
    const float *isc, *ish;
    const void* in = input_of(h, w, l, false, &isc, &ish);
    GemmEpi ep = fwd_epi(h, w, a, s, M, a.bn ? s.y : s.out, false);
    if (a.bn) {
      RET_IF(mmad_bn_eval_affine(a.N, a.Np, h->params + a.g_off, h->params + a.be_off,
                                 running_mean(h, a), running_var(h, a), h->bn_eps, s.scale,
                                 s.shift, st));
      ep.bn_scale = s.scale;
      ep.bn_shift = s.shift;
    }
    if (l == nL - 1) {
      ep.ref = w.xin;
      ep.ldref = a.Np;
      ep.rowsq = s.rowsq;
      ep.ldrow = Mp;
      ep.diff = diffs;
      ep.lddiff = ld_diff;
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_SCORE, in, a.Kp, weights(h, a), a.Kp, Mp, a.Np, a.Kp,
                                ep, st));
    } else {
      RET_IF(ae_gemm(h, w, dt, GEMM_EPI_FWD, in, a.Kp, weights(h, a), a.Kp, Mp, a.Np, a.Kp,
                                ep, st));
    }
    if (h->vib && l == h->n_enc - 1) {
      RET_IF(mmad_vib_reparam_fwd(dt, B, h->btl, 1, s.out, a.Np, nullptr, nullptr, 0, 0, 1, w.zbuf,
                                  h->L[h->n_enc].Kp, nullptr, st));
    }
  }
  // pass 2: x_hat through the encoder, diff against pass-1 activations
  const void* cur = w.l[nL - 1].out;
  int coff = h->L[0].K;
  for (int e = 0; e < h->n_enc; ++e) {
    const AeLayer& a = h->L[e];
    LayerWS& s = w.l[e];
    GemmEpi ep = fwd_epi(h, w, a, s, B, s.dy, false);
    if (a.bn) {
      ep.bn_scale = s.scale;
      ep.bn_shift = s.shift;
    }
    ep.ref = a.bn ? s.y : s.out;
    ep.ldref = a.Np;
    ep.rowsq = s.rowsq;
    ep.ldrow = w.Mpe;
    ep.diff = diffs ? diffs + coff : nullptr;
    ep.lddiff = ld_diff;
    RET_IF(ae_gemm(h, w, dt, GEMM_EPI_SCORE, cur, a.Kp, weights(h, a), a.Kp, w.Mpe, a.Np,
                              a.Kp, ep, st));
    coff += a.N;
    cur = s.dy;
  }
  // per-window sums: layer_sq[0] from the decoder's last layer, [1+e] from pass 2
  MmadReduceJobs jobs{};
  const AeLayer& last = h->L[nL - 1];
  jobs.j[0] = MmadReduceJob{w.l[nL - 1].rowsq, layer_sq, last.Np / 128, w.Mpd, B, B, 1.f, 0,
                            nullptr, 0, 0.f};
  for (int e = 0; e < h->n_enc; ++e)
    jobs.j[e + 1] = MmadReduceJob{w.l[e].rowsq, layer_sq + (size_t)(e + 1) * ld_sq,
                                  h->L[e].Np / 128, w.Mpe, B, B, 1.f, 0, nullptr, 0, 0.f};
  MMAD_CHECK_ARG(h->n_enc + 1 <= MMAD_MAX_REDUCE_JOBS, "too many encoder layers");
  return mmad_reduce_jobs(jobs, h->n_enc + 1, B, st);
}

int mmad_ae_score(mmad_ae* h, const float* x, int ld_x, int B, float* layer_sq, float* diffs,
                  void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->running, "ae_score: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && layer_sq, "ae_score: bad args");
  AeWS w;
  RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w, (hipStream_t)stream));
  return score_batch(h, x, ld_x, B, layer_sq, B, diffs, w, (hipStream_t)stream);
}

// the whole N-window pass, batch by batch, on stream st
static int score_pass(mmad_ae* h, const float* x, int ld_x, int64_t N, int batch, float* layer_sq,
                      int64_t ld_sq, void* ws, int64_t ws_bytes, hipStream_t st) {
  for (int64_t s0 = 0; s0 < N; s0 += batch) {
    const int B = (int)std::min<int64_t>(batch, N - s0);
    AeWS w;
    RET_IF(prepare_ws(h, B, 1, ws, ws_bytes, w, st));
    RET_IF(score_batch(h, x + s0 * ld_x, ld_x, B, layer_sq + s0, ld_sq, nullptr, w, st));
  }
  return MMAD_OK;
}

int mmad_ae_score_stream(mmad_ae* h, const float* x, int ld_x, int64_t N, int batch,
                         float* layer_sq, int64_t ld_sq, void* ws, int64_t ws_bytes, int use_graph,
                         void* stream) {
  MMAD_CHECK_ARG(h && h->params && h->running, "ae_score_stream: unbound handle");
  MMAD_CHECK_ARG(x && ld_x >= h->L[0].K && layer_sq && N >= 1 && batch >= 1 && ld_sq >= N,
                 "ae_score_stream: bad args (N=%lld batch=%d ld_sq=%lld)", (long long)N, batch,
                 (long long)ld_sq);
  hipStream_t st = (hipStream_t)stream;
  if (!use_graph) return score_pass(h, x, ld_x, N, batch, layer_sq, ld_sq, ws, ws_bytes, st);
  for (auto& g : h->graphs) {
    if (g.x == x && g.ld_x == ld_x && g.N == N && g.batch == batch && g.sq == layer_sq &&
        g.ld_sq == ld_sq && g.ws == ws && g.wts == weights(h, h->L[0])) {
      MMAD_HIP_CHECK(hipGraphLaunch(g.exec, st));
      return MMAD_OK;
    }
  }
  // first pass of this shape: run it eagerly (that also settles every GEMM
  // tile choice, which cannot be timed under capture), then capture the same
  // launches on the handle's capture stream for the next calls
  RET_IF(score_pass(h, x, ld_x, N, batch, layer_sq, ld_sq, ws, ws_bytes, st));
  if (!h->gstream) MMAD_HIP_CHECK(hipStreamCreateWithFlags(&h->gstream, hipStreamNonBlocking));
  hipGraph_t graph = nullptr;
  MMAD_HIP_CHECK(hipStreamBeginCapture(h->gstream, hipStreamCaptureModeThreadLocal));
  const int rc = score_pass(h, x, ld_x, N, batch, layer_sq, ld_sq, ws, ws_bytes, h->gstream);
  const hipError_t ec = hipStreamEndCapture(h->gstream, &graph);
  if (rc != MMAD_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  MMAD_HIP_CHECK(ec);
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  MMAD_HIP_CHECK(ei);
  if (h->graphs.size() >= 8) {   // bounded cache: drop the oldest pass
    (void)hipGraphExecDestroy(h->graphs.front().exec);
    h->graphs.erase(h->graphs.begin());
  }
  h->graphs.push_back({x, ld_x, N, batch, layer_sq, ld_sq, ws, weights(h, h->L[0]), exec});
  return MMAD_OK;
}

int mmad_ae_status(mmad_ae* h, void* ws, int64_t ws_bytes, void* stream) {
  MMAD_CHECK_ARG(h, "ae_status: null handle");
  // no split-K GEMM / fused-BN barrier can have run unless the dtype /
  // override / BN mode allows one
  if ((!splitk_possible(h->dtype) && h->bn_mode != 2 && h->bn_mode_bwd != 2) || !ws)
    return MMAD_OK;
  AeWS w;
  carve(h, 1, 1, (char*)ws, w);
  MMAD_CHECK_ARG(ws_bytes >= w.bytes, "ae_status: workspace too small");
  for (int r = 0; r < 2; ++r)
    RET_IF(mmad_gemm_read_status(w.sk_ctl[r], (hipStream_t)stream, "ae_status"));
  if ((h->bn_mode == 2 || h->bn_mode_bwd == 2) && w.bn_err) {
    unsigned word = 0;
    MMAD_HIP_CHECK(hipMemcpyAsync(&word, w.bn_err, sizeof(word), hipMemcpyDeviceToHost, (hipStream_t)stream));
    MMAD_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    if (word) {
      // re-zero every control word (a barrier that gave up may have left
      // counters raised) for the next call
      MMAD_HIP_CHECK(hipMemsetAsync(w.sk_ctl[0], 0, w.sk_ctl_bytes, (hipStream_t)stream));
      MMAD_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
      mmad_set_error("ae_status: a fused BatchNorm column barrier timed out; the outputs of that "
                     "call are invalid");
      return MMAD_EHIP;
    }
  }
  return MMAD_OK;
}

int mmad_ae_probe(mmad_ae* h, int kind, int layer, int capacity) {
  MMAD_CHECK_ARG(h, "ae_probe: null handle");
  MMAD_CHECK_ARG(kind >= 0 && kind <= 3,
                 "ae_probe: kind must be 0 / 1 (forward / dW GEMM) or 2 / 3 (the same, kernel-attached events)");
  MMAD_CHECK_ARG(capacity >= 0 && capacity <= 4096, "ae_probe: capacity out of range");
  MMAD_CHECK_ARG(layer < 0 || layer < (int)h->L.size(), "ae_probe: bad layer %d", layer);
  for (auto e : h->probe_ev) (void)hipEventDestroy(e);
  h->probe_ev.clear();
  h->probe_n = 0;
  h->probe_id = -1;
  h->probe_mask = 0;
  h->probe_kev = kind >= 2;
  if (layer < 0 || capacity == 0) return MMAD_OK;
  h->probe_ev.resize(2 * (size_t)capacity, nullptr);
  for (auto& e : h->probe_ev) MMAD_HIP_CHECK(hipEventCreate(&e));
  if (!h->probe_sync) MMAD_HIP_CHECK(hipEventCreateWithFlags(&h->probe_sync, hipEventDisableTiming));
  h->probe_id = ((kind & 1) == 0 ? PROBE_FWD : PROBE_DW) + layer;
  return MMAD_OK;
}

int mmad_ae_probe_layers(const mmad_ae* h) { return h ? (int)h->probe_mask : -1; }

int mmad_ae_probe_read(mmad_ae* h, float* ms, int max_n) {
  if (!h || !ms || max_n < 0) {
    mmad_set_error("ae_probe_read: bad arguments");
    return MMAD_EINVAL;
  }
  const int n = std::min(h->probe_n, max_n);
  for (int i = 0; i < n; ++i) {
    MMAD_HIP_CHECK(hipEventSynchronize(h->probe_ev[2 * i + 1]));
    MMAD_HIP_CHECK(hipEventElapsedTime(&ms[i], h->probe_ev[2 * i], h->probe_ev[2 * i + 1]));
  }
  return n;
}

int mmad_ae_graph_count(const mmad_ae* h) { return h ? (int)h->graphs.size() : -1; }

int mmad_ae_clear_graphs(mmad_ae* h) {
  MMAD_CHECK_ARG(h, "ae_clear_graphs: null handle");
  for (auto& g : h->graphs) (void)hipGraphExecDestroy(g.exec);
  h->graphs.clear();
  return MMAD_OK;
}
