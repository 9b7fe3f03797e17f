// Internal (non-ABI) launchers shared by the executor.
#pragma once
#include <stdint.h>

#include "mmad_common.h"

int mmad_matrix_colsum_partials(int dtype, int M, int Mp, int Np, const void* x, float* part,
                                void* stream);
int mmad_sum2d(int rows, int cols, const float* x, int64_t ld, float scale, float* out,
               int accumulate, void* stream);
int mmad_sse_partials(int dtype, int M, int N, int Np, const void* y, const float* x, int ldx,
                      float* part, int nparts, void* stream);
int mmad_to_bf16(int64_t n, const float* x, void* y, void* stream);
int mmad_from_bf16(int64_t n, const void* x, float* y, void* stream);
int64_t mmad_vib_kl_parts(int B, int k, int ld_z);
// as the C-ABI forms, with the per-call values read from `dyn` (nullable)
int mmad_pack_input_dyn(int dtype, int M, int K, int Mp, int Kp, const float* x, int ld_x,
                        void* out, const MmadDyn* dyn, void* stream);
int mmad_vib_reparam_fwd_dyn(int dtype, int B, int btl, int k, const void* enc_out, int ld_enc,
                             const float* eps, float* eps_out, uint64_t seed, uint64_t offset,
                             int deterministic, void* z, int ld_z, float* kl_partial,
                             const MmadDyn* dyn, void* stream);

#define MMAD_MAX_REDUCE_JOBS 24
struct MmadReduceJob {
  const float* src;   // partials, row i at src + i*stride
  float* dst;         // [Np] (column job) or [1] (scalar job)
  int nparts, stride, N, Np;
  float scale;
  int scalar;         // 1: dst[0] = scale*sum(all) + scale2*sum(src2[0:n2])
  const float* src2;
  int n2;
  float scale2;
};
struct MmadReduceJobs {
  MmadReduceJob j[MMAD_MAX_REDUCE_JOBS];
  const MmadDyn* dyn;   // non-null: scalar jobs write dyn->loss (graph-captured step)
};
int mmad_reduce_jobs(const MmadReduceJobs& jobs, int n_jobs, int max_np, void* stream);

// One Adam segment.  If bsrc != null the first bNp elements take their
// gradient from bias partials: g[e] = sum_i bsrc[i*bstride + e] (e < bN,
// else 0), written back to g (the bias grad is finalised inside the update).
struct MmadAdamSeg {
  float* p; float* g; float* m; float* v; void* shadow; int64_t n;
  const float* bsrc; int bparts, bstride, bN, bNp;
};
// Adam constants as torch.optim.Adam forms them from its double hyper-
// parameters (recovered from the floats: mmad_decimal_of); w = float(1 - beta)
struct MmadAdamConsts { float w1, w2, eps, step_size, bc2_sqrt; };
double mmad_decimal_of(float f);
MmadAdamConsts mmad_adam_consts(float lr, float beta1, float beta2, float eps, int step);
// flat Adam with the constants already formed (w1, w2: MmadAdamConsts)
int mmad_adam_w(int64_t n, float* p, const float* g, float* m, float* v, float w1, float w2,
                float eps, float step_size, float bc2_sqrt, void* shadow, int64_t n_shadow,
                void* stream);
// mmad_adam_w with the step terms read from `dyn` when non-null (graph capture)
int mmad_adam_dyn(int64_t n, float* p, const float* g, float* m, float* v, float w1, float w2,
                  float eps, float step_size, float bc2_sqrt, void* shadow, int64_t n_shadow,
                  const MmadDyn* dyn, void* stream);
int mmad_adam2(const MmadAdamSeg& s0, const MmadAdamSeg& s1, float w1, float w2, float eps,
               float step_size, float bc2_sqrt, void* stream);

int mmad_bn_finalize(int M, int N, int Mp, int Np, const float* stats, const float* gamma,
                     const float* beta, float* running_mean, float* running_var, float momentum,
                     float eps, float* save_mean, float* save_rstd, float* scale, float* shift,
                     void* stream);
// train-mode BN finalize of a producer layer (Np columns) fused with the
// fold into its consumer's weights: wout[n][k] = W[n][k] * scale[k] (dtype of
// the GEMM), cpart[k/64][n] = sum_{k in block} shift[k] * W[n][k].
// W: fp32 master [Nc_p][Np]; grid (Np/64) x (Nc_p/64).
int mmad_bn_finalize_fold(int dtype, int M, int N, int Mp, int Np, const float* stats,
                          const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float momentum, float eps, float* save_mean,
                          float* save_rstd, float* scale, float* shift, const float* W, int Nc_p,
                          void* wout, float* cpart, void* stream);
int mmad_bn_act_bwd_apply(int dtype, int act, float slope, int M, int N, int Mp, int Np,
                          const void* dy, const void* a, const float* save_mean,
                          const float* save_rstd, const float* gamma, const double* part,
                          int nparts, void* dz, float* dgamma, float* dbeta, float* db_partials,
                          void* stream);
// the same, with `done` (nullable) completed by the launch itself
// (hipExtLaunchKernel stop event: no marker packet behind it)
int mmad_bn_act_bwd_apply_ev(int dtype, int act, float slope, int M, int N, int Mp, int Np,
                             const void* dy, const void* a, const float* save_mean,
                             const float* save_rstd, const float* gamma, const double* part,
                             int nparts, void* dz, float* dgamma, float* dbeta, float* db_partials,
                             void* stream, void* done);
