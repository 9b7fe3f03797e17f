// Internal GEMM interface (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>

// split-K control block: per-launch arrival counters + flags use fewer than
// MMAD_SK_ERR_WORD words (mmad_gemm_splitk checks); this word records a combine that timed out (sticky until read
// by mmad_gemm_status / mmad_ae_status)
#define MMAD_SK_ERR_WORD 8191
#define MMAD_SK_SLAB_TILES 832

enum GemmEpiKind {
  GEMM_EPI_FWD = 0,         // y = BNaffine(act(acc + bias)); optional Welford partials
  GEMM_EPI_MSE = 1,         // dz = gscale*(acc + bias - target); partials (sum dz, sum d^2)
  GEMM_EPI_BWD_DATA = 2,    // dx = acc; optional column-sum partials
  GEMM_EPI_BWD_WEIGHT = 3,  // dW = acc (fp32 out)
  GEMM_EPI_SCORE = 4,       // as FWD (eval) + row-sum of (y - ref)^2, optional diff out
};

struct GemmEpi {
  int M, N;              // valid rows / cols of the output
  void* out;             // output, ld = ldo elements
  int ldo;
  const float* bias;     // [Np]
  int act;
  float slope;
  const float* bn_scale; // eval-mode BN affine (nullable)
  const float* bn_shift;
  float* part;           // partials [Mp/32][2][ldpart]
  int ldpart;
  const float* target;   // MSE target (fp32 user input), ld = ldt
  int ldt;
  int tmod;              // MSE target row = row % tmod (k-expanded VIB decoder)
  float gscale;          // MSE gradient scale (2 for sum-MSE, 2/k for VIB)
  const void* ref;       // SCORE reference activations (same dtype as out)
  int ldref;
  float* rowsq;          // SCORE row partials [Np/128][ldrow]: sum_j colw[j]*(y-ref)^2
  const float* colw;     // SCORE per-column weights (nullable = 1); ref nullable = 0
  int ldrow;
  float* diff;           // SCORE optional fp32 diff output
  int lddiff;
  // FWD/MSE: folded train-mode BN of the producer: bias += sum_p bpart[p][n]
  const float* bpart;    // [bparts][bpstride] (nullable)
  int bparts, bpstride;
  // BWD_WEIGHT on a train-mode BN producer's raw activation a (x = a*s + t):
  // dW = b_scale[k] * (dz^T a) + b_shift[k] * db[n], db[n] = sum_p gb_src[p][n]
  const float* b_scale;  // indexed by k (nullable)
  const float* b_shift;
  const float* gb_src;
  int gb_parts, gb_stride;
  // BWD_DATA: BatchNorm-backward column partials of the produced dy
  const void* bn_a;      // pre-BN activation, same shape/ld as out (nullable)
  const float* bn_mean;
  const float* bn_rstd;
  double* bn_part;       // [Mp/64][2][ldo]: (sum dy, sum dy*xhat), fp64
  // MSE: one loss partial (sum d^2) per output tile, [mmad_gemm_ntiles(plan)]
  float* lossp;
  // BWD_WEIGHT: torch.optim.Adam step fused into the epilogue (nullable p).
  // Weight tile: p/m/v share the dW layout (ld = ldo); shadow gets bf16(p).
  float* ad_p;
  float* ad_m;
  float* ad_v;
  void* ad_shadow;
  float ad_w1, ad_w2, ad_eps, ad_step, ad_bc2;   // Adam: w = float(1 - beta) (mmad_adam_consts)
  int dw_nostore;        // with ad_p: do not materialise dW (Adam consumed it)
  // ... and the layer's small segment [bias | gamma | beta], spread over all
  // blocks; the first bNp elements take g = sum of bias partials.
  float* sm_p;
  float* sm_g;
  float* sm_m;
  float* sm_v;
  int sm_n;
  int sm_bN, sm_bNp;     // bias entries (valid / padded); their g = db from gb_src
  // split-K (nullable = off): fp32 partial-tile slabs and the per-tile
  // arrival counter + flag words (zero before a launch; every launch leaves
  // them zero).  Sizes: mmad_gemm_splitk_bytes.  The split factor itself is
  // a deterministic function of the shape (mmad_gemm_splitk).
  float* sk_slab;
  unsigned* sk_ctl;
  // set by the launcher: split factor, XCD-aware grouped tile order
  int splitk;
  int tiles_n, group_m;
  int persist_tiles;   // persistent grid (knob 12): every block loops over these tiles
  int tile_force;        // caller's tile choice + 1 (0 = none; ignored if it does not fit)
  // graph-captured step (nullable): MSE target = dyn->x, Adam step terms
  // from dyn (see MmadDyn)
  const MmadDyn* dyn;
  // Train-mode BatchNorm fused into the producing GEMM (bn_sync != null):
  // the tiles_m blocks of one output column tile publish their column
  // partials (sc1 stores), meet at a counter barrier (bn_sync[tn] arrivals,
  // reset by the last arriver, which bumps the generation word
  // bn_sync[MMAD_BN_EXIT + tn] the others poll; zero before the first launch)
  // and each finishes the whole-batch statistics for its columns itself.
  // Needs every block of the grid co-resident (mmad_gemm_bn_fusable), S = 1.
  //  FWD: part = Welford partials; writes out = a (pre-BN activation) and
  //       bn_y = BN(a) = a*scale + shift; the tm == 0 blocks write
  //       bn_save_mean/rstd and update the running statistics (nullable).
  //  BWD_DATA: bn_part = fp64 (sum dy, sum dy*xhat) per 64 rows; writes
  //       bn_dz = act'(a) * dBN(dy) (out unused), bn_dbpart = per-64-row
  //       column sums of dz, and (tm == 0) bn_dgamma / bn_dbeta.
  unsigned* bn_sync;
  unsigned* bn_err;      // sticky timeout word (barrier never completed)
  const float* bn_gamma;
  const float* bn_beta;
  float* bn_rmean;
  float* bn_rvar;
  float bn_mom, bn_eps;
  float* bn_save_mean;
  float* bn_save_rstd;
  void* bn_y;
  void* bn_dz;
  float* bn_dgamma;
  float* bn_dbeta;
  float* bn_dbpart;
  int bn_act;            // BWD_DATA: the BN producer's activation (act' from a)
  int dbg;               // diagnostics (tools/gemm_phase): 1 skip main loop, 2 skip epilogue,
                         // 4 force the split-K combine's timeout path (tests),
                         // 8 skip the FWD Welford partial stores
  // host only (nullable): an event completed by the launch itself
  // (hipExtLaunchKernel's stop event) instead of a separate hipEventRecord
  // behind it, whose marker packet holds the stream's next dispatch
  hipEvent_t done_ev;
  // host only (nullable): an event that takes the launch's start time
  // (hipExtLaunchKernel's start event; the executor's in-step kernel probe)
  hipEvent_t start_ev;
};

int mmad_knob(int k);          // the tune table (mmad_tune_set)
int mmad_group_override();

int mmad_tile_override();
int mmad_autotune_enabled();
int mmad_dbg_override();
int mmad_persist_override();   // knob 12
int mmad_splitk_override();   // 0 = shape rule; 1, 2, 4, 8, 16 = forced split factor
int mmad_splitk_dw_override();     // the same for the dW GEMMs only (knob 9)
int mmad_splitk_dw_blocks();       // dW split rule: target 64x64-tile blocks (knob 10)
int mmad_splitk_dw_min_stages();   // dW split rule: minimum K stages per slice (knob 11)
int mmad_splitk_dw_f32_blocks();   // fp32 dW split rule from 2048 rows: target blocks (knob 32)
int mmad_tile_adam_override();  // >= 0: tile of the Adam-fused dW GEMMs (-2: shape rule)
int mmad_tile_adam_for(int Mp, int Np, int K);   // ... for a shape
int mmad_tile_adam_main_override();  // >= 0: ... of those on the main stream
int mmad_tile_adam_main_for(int Mp, int Np, int K);   // ... for a shape (-2: rule)
int mmad_tile_epi_override(int epi);  // >= 0: tile of this epilogue's GEMMs

// tile configuration a problem will run with (autotuned on first dispatch of
// the shape; a static heuristic before that / when tuning is off)
int mmad_gemm_plan(int Mp, int Np, int K, int epi, int dtype);
// output tiles of a configuration (= MSE loss partials written)
int mmad_gemm_ntiles(int cfg, int Mp, int Np);
// upper bound of mmad_gemm_ntiles over all configurations
int mmad_gemm_tiles(int Mp, int Np);

// split-K factor the dispatcher uses for a shape when the caller provides
// split-K workspace (1, 2, 4, 8 or 16; a function of the shape and epilogue
// only, so every tile configuration of a shape accumulates in the same order)
int mmad_gemm_splitk(int Mp, int Np, int K, int dtype, int epi);
// split-K workspace sufficient for every launch (shape-independent bound)
void mmad_gemm_splitk_bytes(int Mp, int Np, size_t* slab_bytes, size_t* ctl_bytes);
// read (and clear) the timeout word of a split-K control block after syncing
// `s`: MMAD_OK, or MMAD_EHIP with the error string set
int mmad_gemm_read_status(unsigned* ctl, hipStream_t s, const char* who);

// offset of the generation words inside a fused-BN barrier block; words per block
#define MMAD_BN_EXIT 64
#define MMAD_BN_SYNC_WORDS 128
// can a GEMM with the fused train-mode BN epilogue (bn_sync) run this shape:
// is there a fitting tile configuration whose whole grid is co-resident on
// the current device?  (the per-column-tile barrier needs every block of a
// column resident; with the whole grid resident, work of other streams can
// delay it but never block it)
bool mmad_gemm_bn_fusable(int dtype, int epi, int Mp, int Np);

// cfg_used (nullable) receives the tile configuration launched
int mmad_gemm_dispatch(int dtype, int epi, const void* A, int lda, const void* B, int ldb, int Mp,
                       int Np, int K, const GemmEpi& ep, hipStream_t s, int* cfg_used = nullptr);
