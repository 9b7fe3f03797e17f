// Shared device/host helpers for the MI355X (gfx950) autoencoder hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/mmad.h"

typedef __bf16 bf16;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int uint4v __attribute__((ext_vector_type(4)));
typedef unsigned int uint2v __attribute__((ext_vector_type(2)));

#define MMAD_LDS __attribute__((address_space(3)))

// Padding granule for every feature / batch dimension of the packed layouts
// (see DESIGN.md "Data layout in HBM"): GEMM tiles never need K/N masking.
#define MMAD_PAD 128
// Rows per BatchNorm / column-sum partial written by GEMM epilogues.
#define MMAD_PART_ROWS 32

static inline int mmad_roundup(int x, int g) { return (x + g - 1) / g * g; }

// Per-call values of a train step that a captured hipGraph reads from device
// memory instead of kernel arguments (the executor copies a fresh block in
// before each replay): the input windows, the loss destination, the VIB noise
// source and the Adam bias-correction terms of this step.
struct MmadDyn {
  const float* x;        // input windows [B][ld_x] (also the MSE target)
  float* loss;           // loss destination (device fp32 [1])
  const float* eps;      // injected VIB noise [k][B][btl] or null (Philox)
  unsigned long long seed, offset;
  float ad_step, ad_bc2; // Adam lr/(1-b1^t), sqrt(1-b2^t)
  float pad[2];
};

// ---- error reporting (thread-local, no exceptions across the ABI) -------
void mmad_set_error(const char* fmt, ...);
#define MMAD_CHECK_ARG(cond, ...)                                      \
  do {                                                                 \
    if (!(cond)) { mmad_set_error(__VA_ARGS__); return MMAD_EINVAL; }  \
  } while (0)
#define MMAD_HIP_CHECK(expr)                                                   \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess) {                                                    \
      mmad_set_error("HIP error %d (%s) at %s:%d", (int)e_, hipGetErrorString(e_), \
                     __FILE__, __LINE__);                                      \
      return MMAD_EHIP;                                                        \
    }                                                                          \
  } while (0)
#define MMAD_LAUNCH_CHECK() MMAD_HIP_CHECK(hipGetLastError())

// ---- element conversion ---------------------------------------------------
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16>(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

// activation enum shared with the ABI (modules/activation.py:20-45)
__device__ __forceinline__ float apply_act(float z, int act, float slope) {
  switch (act) {
    case MMAD_ACT_LEAKYRELU: return z > 0.f ? z : z * slope;
    case MMAD_ACT_RELU: return z > 0.f ? z : 0.f;
    case MMAD_ACT_SIGMOID: return 1.f / (1.f + __expf(-z));
    case MMAD_ACT_TANH: return tanhf(z);
    default: return z;
  }
}
// the piecewise-linear activations (LeakyReLU / ReLU / none) as one
// branch-free form z > 0 ? z : lo(z): inside the fully unrolled GEMM
// epilogues a per-element `switch` on the (uniform) activation became one
// scalar branch tree per element -- ~17k instructions of epilogue code, most
// of a 256x256 tile's epilogue time in instruction fetch.  Same values as
// apply_act for these three (z * 1 == z exactly; ReLU's 0 is +0).
__host__ __device__ __forceinline__ bool act_is_linear_piecewise(int act) {
  return act == MMAD_ACT_LEAKYRELU || act == MMAD_ACT_RELU || act == MMAD_ACT_NONE;
}
__device__ __forceinline__ float act_lo_slope(int act, float slope) {
  return act == MMAD_ACT_LEAKYRELU ? slope : (act == MMAD_ACT_NONE ? 1.f : 0.f);
}
__device__ __forceinline__ float apply_act_pw(float z, bool relu, float lo_slope) {
  const float lo = relu ? 0.f : z * lo_slope;
  return z > 0.f ? z : lo;
}
// derivative expressed through the activation OUTPUT a (all supported acts
// are monotone so the output determines the branch / value)
// (act is uniform: selects instead of a switch, so an unrolled per-element
// loop stays one straight-line block instead of a branch chain per element)
__device__ __forceinline__ float act_grad_from_out(float a, int act, float slope) {
  const bool step = act == MMAD_ACT_LEAKYRELU || act == MMAD_ACT_RELU;
  const float neg = act == MMAD_ACT_LEAKYRELU ? slope : 0.f;
  float g = act == MMAD_ACT_SIGMOID ? a * (1.f - a) : 1.f;
  g = act == MMAD_ACT_TANH ? 1.f - a * a : g;
  return step ? (a > 0.f ? 1.f : neg) : g;
}

// torch.optim.Adam element update, as torch's _single_tensor_adam computes it
// on the CPU (the reference's optimizer, novelty_detection.py:90, in the form
// its golden vectors were generated in: torch-CPU) -- every rounding step in
// torch's CPU order (checked against torch 2.10 CPU kernels).  The
// reference's default device run (--gpu_id 0, model_builder.py:50-51) would
// take torch's foreach CUDA path, whose addcdiv rounds p + s * (m / denom)
// instead of p + (s * m) / denom: that form is not pinned here (no CUDA
// reference run exists to pin it against):
//   exp_avg.lerp_(g, 1 - b1)            m = fma(w1, g - m, m)   (w1 < 0.5)
//   exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
//                                       v = fma(w2 * g, g, v * b2)
//   denom = (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
//   param.addcdiv_(exp_avg, denom, value=-step_size)
//                                       p = p + (-step_size * m) / denom
// w1 = float(1 - b1), w2 = float(1 - b2) are formed from the DOUBLE betas
// (mmad_adam_consts: the decimal the float came from); b2 = float(1 - w2)
// recovers torch's float(beta2) exactly.  Until round 5 the update was
// m = fma(b1, m, (1 - b1) g), v = fma(b2, v, (1 - b2) g^2) with 1 - b
// formed in float (1 - 0.999f = 0.00099998713, 1.3e-5 below torch's 0.001)
// and bc2 from the float beta2: a systematic ~-5e-6 relative step size that
// the teacher-forced test (tests/test_gpu_teacher.py) found.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float w1,
                                          float w2, float eps, float step, float bc2) {
  const float b2 = (float)(1.0 - (double)w2);
  const float d = g - m;
  m = w1 < 0.5f ? fmaf(w1, d, m) : fmaf(w1 - 1.f, d, g);
  v = fmaf(w2 * g, g, v * b2);
  const float denom = __fdiv_rn(__fsqrt_rn(v), bc2) + eps;
  p = p + __fdiv_rn(-step * m, denom);
}

__device__ __forceinline__ void adam4(floatx4& p, floatx4& m, floatx4& v, floatx4 g, float w1,
                                      float w2, float eps, float step, float bc2) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float pe = p[e], me = m[e], ve = v[e];
    adam_elem(pe, me, ve, g[e], w1, w2, eps, step, bc2);
    p[e] = pe;
    m[e] = me;
    v[e] = ve;
  }
}

// v[lane ^ 16] and v[lane ^ 32] for every lane of the wave through the gfx950
// lane-swap VALU ops (v_permlane16_swap_b32: odd 16-lane rows of vdst <->
// even rows of vsrc; v_permlane32_swap_b32: lanes 32-63 of vdst <-> lanes
// 0-31 of vsrc), called with vdst = vsrc = v: one VALU op + a select, no LDS
// round trip (__shfl_xor lowers to ds_bpermute_b32, ~100+ cycles of latency
// per dependent step in the GEMM epilogues' column reductions).  The values
// are exactly those of __shfl_xor(v, 16 / 32) (tools/permlane_check.hip).
__device__ __forceinline__ float lane_xor16(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(float, (__lane_id() & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float lane_xor32(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (__lane_id() & 32) ? r[0] : r[1]);
}
// (x + x^16) + (x^32 + x^48) in every lane: the same association as
// x += shfl_xor(x, 16); x += shfl_xor(x, 32)
__device__ __forceinline__ float sum_lane_groups(float x) {
  x += lane_xor16(x);
  return x + lane_xor32(x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
