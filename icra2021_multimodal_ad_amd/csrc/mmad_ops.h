// Internal (non-ABI) launchers shared by the executor.
#pragma once
#include <stdint.h>

int mmad_matrix_colsum_partials(int dtype, int M, int Mp, int Np, const void* x, float* part,
                                void* stream);
int mmad_sum2d(int rows, int cols, const float* x, int64_t ld, float scale, float* out,
               int accumulate, void* stream);
int mmad_sse_partials(int dtype, int M, int N, int Np, const void* y, const float* x, int ldx,
                      float* part, int nparts, void* stream);
int mmad_to_bf16(int64_t n, const float* x, void* y, void* stream);
int64_t mmad_vib_kl_parts(int B, int k, int ld_z);
