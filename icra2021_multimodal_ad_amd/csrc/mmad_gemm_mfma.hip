// MFMA GEMM for the fc_module encoder/decoder stack on gfx950 (CDNA4).
//
// One kernel template covers the three contractions of an FCLayer
// (layers/fc_layer.py:37-48 forward; its autograd backward):
//   forward      y  = x  . W^T  (+bias, act, BN-eval affine | BN-train stats
//                                 | MSE grad/loss | score-diff epilogues)
//   backward-dx  dx = dz . W     (B operand is MN-major: W stored [out][in])
//   backward-dW  dW = dz^T . x   (both operands MN-major: K = batch)
// Operands stay in the caller's row-major packed layout; an MN-major operand
// is transposed on the LDS read side with ds_read_b64_tr_b16 (bf16) or plain
// per-k reads (f32), so no transposed copies are ever materialised in HBM.
//
// Block tiles (CFG), one block per CU:
//   0: 128x128, 512 threads (waves 2x4, wave tile 64x32), 4-stage ring
//   1: 256x128, 512 threads (waves 4x2, wave tile 64x64), 3-stage ring
//   2: 128x256, 512 threads (waves 2x4, wave tile 64x64), 3-stage ring
//   3:  64x64,  256 threads (waves 2x2, wave tile 32x32), 4-stage ring
//   4:  64x128, 256 threads (waves 2x2, wave tile 32x64), 5-stage ring
//   5: 128x128, 256 threads (waves 2x2, wave tile 64x64), 4-stage ring
// The 8-wave tiles run two waves per SIMD (one wave's LDS reads and barrier
// wait hide behind the other's MFMAs) and carry the large layers; the small
// tiles give the narrow layers enough blocks.  Which one a shape gets is
// measured on first use (mmad_gemm_dispatch autotune): the accumulation
// order over K is the same for every tile, so the choice never changes a
// result bit.
// K stage = 128 bytes of K per operand row (BK = 64 bf16 / 32 f32), staged
// global -> LDS by global_load_lds (16 B/lane, no registers), NS-stage ring
// with a counted vmcnt and a raw s_barrier so NS-2 stages stay in flight
// across every barrier.
//
// LDS images:
//  * K-major operand: [rows][128 B], 16-byte chunk j stored at j ^ ((row>>1)&7)
//    -> conflict-free ds_read_b128 (natural k order) / ds_read_b64 pairs.
//  * MN-major operand: [BK][rows*esize], 16-byte chunk XOR-swizzled per k-row
//    so the tr-reads of one 32-lane half (8 k-rows) hit disjoint banks.
// bf16 k-slot order inside one 32-deep MFMA step: lane group g (= lane>>4)
// owns k = 8g..8g+7 in both operands whatever their layout (one ds_read_b128
// from a K-major image, two ds_read_b64_tr_b16 from an MN-major one).  The
// backward GEMMs used a permuted order {4g..4g+3} U {16+4g..16+4g+3} before,
// which cost the K-major operand two ds_read_b64 per fragment and measured
// 2x the LDS cycles of the forward loop (SQ_LDS_BANK_CONFLICT 1.7M vs 13k).
#include "mmad_common.h"
#include "mmad_gemm.h"

#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>

namespace {

constexpr int MMAD_KB = 128;   // bytes of K per LDS row per stage

template <int CFG> struct Cfg;
template <> struct Cfg<0> { static constexpr int BM = 128, BN = 128, WM = 2, WN = 4, NS = 4, NT = 512; };
template <> struct Cfg<1> { static constexpr int BM = 256, BN = 128, WM = 4, WN = 2, NS = 3, NT = 512; };
template <> struct Cfg<2> { static constexpr int BM = 128, BN = 256, WM = 2, WN = 4, NS = 3, NT = 512; };
template <> struct Cfg<3> { static constexpr int BM = 64, BN = 64, WM = 2, WN = 2, NS = 4, NT = 256; };
template <> struct Cfg<4> { static constexpr int BM = 64, BN = 128, WM = 2, WN = 2, NS = 5, NT = 256; };
template <> struct Cfg<5> { static constexpr int BM = 128, BN = 128, WM = 2, WN = 2, NS = 4, NT = 256; };
// 256x256, 8 waves (2 x 4, wave tile 128x64), a 2-slot ring: twice the
// operand reuse of 256x128 (128 FLOP per staged byte), for the large-row
// bf16 GEMMs of the forward / score / MSE epilogues without the fused BN
// (C5 scoring at 65,536 rows; a round-3 stand-alone loop study, since removed: 0.47-0.55 of peak at
// 16384 x 2048 x 1664 vs 0.33 for 256x128); its epilogue staging fills LDS
constexpr int CFG_BIG = 6;
template <> struct Cfg<6> { static constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NS = 2, NT = 512; };
// 7: 256x256, CFG 6's loop with the MFMA operands swapped (W first): each
// lane's accumulator quad is then 4 consecutive COLUMNS of one output row, so
// the forward / score epilogue stores from registers -- one v_permlane16_swap
// pair turns two column tiles' quads into a 16-byte chunk per lane, 64 B per
// row per store instruction -- with no LDS staging round trip (the score row
// sums meet across the two waves of a 128-column group in 4 KB of LDS).
// Eval forward / score only (no column partials: the BN statistics need the
// row-quad layout); the dispatcher runs CFG 6 in its place otherwise (same
// tile, same bits).
constexpr int CFG_XST = 7;
template <> struct Cfg<7> { static constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NS = 2, NT = 512; };
// 8: 256x256, FOUR waves (2 x 2, wave tile 128x128: 256 accumulator
// registers per lane, in AGPRs), otherwise CFG 7 (swapped operands,
// register-direct epilogue).  One wave per SIMD: per 32-deep step a wave
// issues 64 MFMAs against 16 fragment reads, a third fewer LDS reads per MFMA
// than the 8-wave 128x64 wave tiles.  Compiled in its own translation unit
// (this file with MMAD_GEMM_B4_TU, csrc/Makefile) WITHOUT the VGPR-form MFMA
// flag the other tiles use: 256 + ~150 registers need the AGPR half of the
// file; the host side reaches it through mmad_gemm_b4_launch.
constexpr int CFG_B4 = 8;
template <> struct Cfg<8> { static constexpr int BM = 256, BN = 256, WM = 2, WN = 2, NS = 2, NT = 256; };
// 9: CFG 1 (256x128, 8 waves of 64x64) with CFG 7's swapped operands and
// register-direct epilogue: the large-row forward / score GEMMs whose output
// width is not a multiple of 256 (C5: every layer but the 2048-wide ones)
constexpr int CFG_XST1 = 9;
template <> struct Cfg<9> { static constexpr int BM = 256, BN = 128, WM = 4, WN = 2, NS = 3, NT = 512; };
constexpr int NCFG = 10;
// capacity-cache keys pack (device, dtype, epilogue, cfg) into one integer
// with 8 slots per epilogue field and 16 per cfg field
static_assert(NCFG <= 16, "widen the cfg field of the capacity-cache keys");
constexpr int CFG_BM[NCFG] = {128, 256, 128, 64, 64, 128, 256, 256, 256, 256};
constexpr int CFG_BN[NCFG] = {128, 128, 256, 64, 128, 128, 256, 256, 256, 128};
constexpr int CFG_NT[NCFG] = {512, 512, 512, 256, 256, 256, 512, 512, 256, 512};
inline bool is_big(int cfg) { return cfg == CFG_BIG || cfg == CFG_XST || cfg == CFG_B4; }
inline bool is_xst(int cfg) { return cfg == CFG_XST || cfg == CFG_B4 || cfg == CFG_XST1; }
// the row-quad tile a register-direct one falls back to (same tile shape)
inline int xst_base(int cfg) { return cfg == CFG_XST1 ? 1 : CFG_BIG; }
// the 256x256 tiles: bf16 operands, forward-type epilogues, no fused BN
template <typename T, int EPI>
constexpr bool big_ok() {
  return sizeof(T) == 2 && (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_MSE || EPI == GEMM_EPI_SCORE);
}
inline bool big_ok_rt(int dtype, int epi) {
  return dtype == MMAD_BF16 && (epi == GEMM_EPI_FWD || epi == GEMM_EPI_MSE || epi == GEMM_EPI_SCORE);
}
// the register-direct 256x256 tile: eval forward / score, piecewise-linear
// activations (act_is_linear_piecewise: declared in mmad_common.h)
template <typename T, int EPI>
constexpr bool xst_ok() {
  return sizeof(T) == 2 && (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_SCORE);
}
inline bool xst_ok_rt(int dtype, int epi, const GemmEpi& ep) {
  return dtype == MMAD_BF16 && (epi == GEMM_EPI_FWD || epi == GEMM_EPI_SCORE) && !ep.part && !ep.bpart &&
         act_is_linear_piecewise(ep.act);
}

template <typename T, bool KMAJ, int ROWS, int NT>
struct Img {
  static constexpr int ES = sizeof(T);
  static constexpr int KB = MMAD_KB;
  static constexpr int BK = KB / ES;                  // K per stage
  static constexpr int RB = KMAJ ? KB : ROWS * ES;    // bytes per LDS row
  static constexpr int BYTES = ROWS * KB;             // image bytes (both layouts)
  static constexpr int CPROW = RB / 16;               // 16 B chunks per LDS row
  static constexpr int CHUNKS = BYTES / 16 / NT;      // global_load_lds per thread
  static_assert(CHUNKS >= 1 && BYTES % (16 * NT) == 0, "image/threads mismatch");
};

// 16-byte-chunk XOR swizzle of LDS row `r` (an involution):
//  * K-major, 128 B rows: (r>>1)&7;
//  * MN-major bf16 (rows are k): one transposed read of a 32-lane half covers
//    k rows {0..3, 8..11} (+4 for the second read) of a 32-deep step, 32 B of
//    each; >= 256 B rows start every k row on bank 0, so the XOR takes
//    (k&3) | ((k>>3)&1)<<2 (even chunk steps of 8 banks); 128 B rows alternate
//    bank halves by k parity, so (k>>1)&1 | ((k>>3)&1)<<1 (the XOR must stay
//    inside the row's 8 chunks).  Conflict-free for both reads of a half;
//  * MN-major f32 (rows >= 256 B): r&7 (spreads the 4-row-apart ds_read_b32 groups).
template <typename T, bool KMAJ, int RB>
__device__ __forceinline__ int swz(int r) {
  static_assert(KMAJ || RB >= (sizeof(T) == 2 ? 128 : 256), "MN-major row too short for its swizzle");
  if constexpr (KMAJ) return (r >> 1) & 7;
  else if constexpr (sizeof(T) == 2)
    return RB >= 256 ? (((r & 3) | (((r >> 3) & 1) << 2)) << 1)
                     : ((((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1);
  else return r & 7;
}

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4) into the wave's
// 1 KiB at `dst` (wave-uniform), as inline asm.  Through the builtin, hipcc's
// wait-count pass tracks the DMA as an LDS write it cannot tell apart from
// the transposing fragment reads (ds_read_b64_tr_b16) of other ring slots
// and puts an s_waitcnt vmcnt(0) in front of them -- inside the main loop
// that drains the whole NS-stage ring every K stage.  Hidden from that pass,
// the ring is ordered exactly as designed: counted vmcnt + workgroup barrier
// before a slot is read, a barrier before it is refilled.  (Compiler-tracked
// loads only see MORE operations outstanding than they count, so their own
// waits stay correct, just stricter.)
__device__ __forceinline__ void dma16(const void* src, char* dst) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(MMAD_LDS void*)dst);
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}

// issue one stage of one operand: global -> LDS, 16 B per lane, no registers
template <typename T, bool KMAJ, int ROWS, int NT>
__device__ __forceinline__ void issue_stage(char* img, const T* __restrict__ G, int ld, int r0,
                                            int k0, int tid) {
  using I = Img<T, KMAJ, ROWS, NT>;
  constexpr int EPC = 16 / sizeof(T);
#pragma unroll
  for (int i = 0; i < I::CHUNKS; ++i) {
    const int p = NT * i + tid;                        // LDS position (16 B units)
    const int row = p / I::CPROW;
    const int j = (p % I::CPROW) ^ swz<T, KMAJ, I::RB>(row);
    const T* src = KMAJ ? G + (size_t)(r0 + row) * ld + k0 + j * EPC
                        : G + (size_t)(k0 + row) * ld + r0 + j * EPC;
    dma16(src, img + (NT * i + (tid & ~63)) * 16);
  }
}

// chunk i (< Img::CHUNKS) of one stage of one operand (issue_stage = all i)
template <typename T, bool KMAJ, int ROWS, int NT>
__device__ __forceinline__ void issue_chunk(char* img, const T* __restrict__ G, int ld, int r0, int k0,
                                            int tid, int i) {
  using I = Img<T, KMAJ, ROWS, NT>;
  constexpr int EPC = 16 / sizeof(T);
  const int p = NT * i + tid;
  const int row = p / I::CPROW;
  const int j = (p % I::CPROW) ^ swz<T, KMAJ, I::RB>(row);
  const T* src = KMAJ ? G + (size_t)(r0 + row) * ld + k0 + j * EPC
                      : G + (size_t)(k0 + row) * ld + r0 + j * EPC;
  dma16(src, img + (NT * i + (tid & ~63)) * 16);
}

// ---- bf16 fragment reads (16x16x32 MFMA operand) ---------------------------
// Natural k order for both layouts: lane group g owns k = 8g..8g+7 (K-major:
// one ds_read_b128; MN-major: two ds_read_b64_tr_b16 of k rows 8g..8g+3 and
// 8g+4..8g+7).  (NAT = false, the older permuted order {4g..4g+3} U
// {16+4g..16+4g+3}, is kept for the K-major reader only.)
template <bool KMAJ, bool NAT, int ROWS>
__device__ __forceinline__ bf16x8 frag_bf16(const char* img, int rbase, int kk, int lane) {
  using I = Img<bf16, KMAJ, ROWS, 256>;   // RB only
  const int g = lane >> 4;
  if constexpr (KMAJ) {
    const int m = rbase + (lane & 15);
    const int f = swz<bf16, true, I::RB>(m);
    if constexpr (NAT) {
      return *(const bf16x8*)(img + m * I::RB + (((kk * 4 + g) ^ f) << 4));
    } else {
      const int c1 = (kk * 8 + g) ^ (f << 1);          // 8-byte units
      const int c2 = (kk * 8 + 4 + g) ^ (f << 1);
      bf16x4 lo = *(const bf16x4*)(img + m * I::RB + c1 * 8);
      bf16x4 hi = *(const bf16x4*)(img + m * I::RB + c2 * 8);
      return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  } else {
    static_assert(NAT, "MN-major reads deliver the natural k order");
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int k1 = kk * 32 + 8 * g + q, k2 = k1 + 4;
    const int byte = (rbase + 4 * p) * 2;
    const int j = byte >> 4, within = byte & 15;
    const MMAD_LDS char* base = (const MMAD_LDS char*)img;
    short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (MMAD_LDS short4v*)(base + k1 * I::RB + ((j ^ swz<bf16, false, I::RB>(k1)) << 4) + within));
    short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (MMAD_LDS short4v*)(base + k2 * I::RB + ((j ^ swz<bf16, false, I::RB>(k2)) << 4) + within));
    bf16x4 l4 = __builtin_bit_cast(bf16x4, lo);
    bf16x4 h4 = __builtin_bit_cast(bf16x4, hi);
    return __builtin_shufflevector(l4, h4, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// ---- f32 fragment reads (16x16x4 MFMA, 4 steps per 16-deep chunk) -------
template <bool KMAJ, int ROWS>
__device__ __forceinline__ floatx4 frag_f32(const char* img, int rbase, int kc, int lane) {
  using I = Img<float, KMAJ, ROWS, 256>;  // RB only
  const int g = lane >> 4;
  if constexpr (KMAJ) {
    const int m = rbase + (lane & 15);
    const int j = (kc * 4 + g) ^ swz<float, true, I::RB>(m);
    return *(const floatx4*)(img + m * I::RB + j * 16);
  } else {
    const int col = rbase + (lane & 15);
    const int j = col >> 2, within = (col & 3) * 4;
    floatx4 r;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = kc * 16 + 4 * g + s;
      r[s] = *(const float*)(img + k * I::RB + ((j ^ swz<float, false, I::RB>(k)) << 4) + within);
    }
    return r;
  }
}

// every phase of the main loop pinned in issue order
#define MMAD_SB() __builtin_amdgcn_sched_barrier(0)

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- pipelined main-loop helpers -------------------------------------------
// One K stage (128 B of K per operand row) = two sub-steps: 32-deep bf16
// MFMA steps, or 16-deep f32 steps (4 x 16x16x4 MFMAs each).
template <typename T> struct SubFrag;
template <> struct SubFrag<bf16> { using F = bf16x8; };
template <> struct SubFrag<float> { using F = floatx4; };

template <typename T, bool AK, bool BK_, bool NAT, int BM, int BN, int TM, int TN>
__device__ __forceinline__ void read_sub(const char* sa, const char* sb, int ra, int rb, int sub,
                                         int lane, typename SubFrag<T>::F (&fa)[TM],
                                         typename SubFrag<T>::F (&fb)[TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if constexpr (sizeof(T) == 2) fa[i] = frag_bf16<AK, NAT, BM>(sa, ra + i * 16, sub, lane);
    else fa[i] = frag_f32<AK, BM>(sa, ra + i * 16, sub, lane);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if constexpr (sizeof(T) == 2) fb[j] = frag_bf16<BK_, NAT, BN>(sb, rb + j * 16, sub, lane);
    else fb[j] = frag_f32<BK_, BN>(sb, rb + j * 16, sub, lane);
  }
}

// MFMAs of fragment rows i in [H*TM/2, (H+1)*TM/2): a sub-step is issued as
// two such groups with the next fragment reads between them
// row_hook(i) runs after the MFMAs of fragment row i: the next stage's
// LDS-DMA is spread over them (a burst of DMA issues right after the barrier
// delays the MFMAs behind it: +10-12 % in the round-3 loop study, profiles/r03c_*)
struct NoHook {
  __device__ __forceinline__ void operator()(int) const {}
};
// (SW: the operands swapped -- W first -- for the register-direct epilogue)
template <typename T, int TM, int TN, int H, bool SW = false, typename Hook = NoHook>
__device__ __forceinline__ void mma_half(floatx4 (&acc)[TM][TN], const typename SubFrag<T>::F (&fa)[TM],
                                         const typename SubFrag<T>::F (&fb)[TN], Hook row_hook = Hook{}) {
#pragma unroll
  for (int i = H * TM / 2; i < (H + 1) * TM / 2; ++i) {
    row_hook(i);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (sizeof(T) == 2) {
        acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0)
                       : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
      }
    }
  }
}

// lgkmcnt(0) as a real s_waitcnt (vmcnt/expcnt at max) so the compiler's own
// counter bookkeeping sees it
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// no more issues: stage t+1 must land, rem = nt-t-2 later stages may stay in flight
template <int NL>
__device__ __forceinline__ void wait_tail(int rem) {
  if (rem >= 3) wait_vmcnt<3 * NL>();
  else if (rem == 2) wait_vmcnt<2 * NL>();
  else if (rem == 1) wait_vmcnt<NL>();
  else wait_vmcnt<0>();
}

// the same with X more (younger) loads allowed in flight: the dW GEMM's Adam
// state prefetch, issued after the last ring DMA
template <int NL, int X>
__device__ __forceinline__ void wait_tail_x(int rem) {
  static_assert(3 * NL + X <= 63, "vmcnt range");
  if (rem >= 3) wait_vmcnt<3 * NL + X>();
  else if (rem == 2) wait_vmcnt<2 * NL + X>();
  else if (rem == 1) wait_vmcnt<NL + X>();
  else wait_vmcnt<X>();
}

__device__ __forceinline__ void block_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- cross-workgroup hand-off of the fused-BN column partials -------------
// Agent-scope relaxed atomics lower to sc1 global loads / stores (L1
// bypassed, written through): producers store every partial sc1, wait for
// their stores, meet at a workgroup barrier, and one lane adds to the column
// counter; one lane polls it with sc1 loads, the block joins it at a barrier
// and then reads the partials with sc1 loads only (MI355X_MICROARCH.md,
// hand-off table row 1: no release / acquire fences needed).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((unsigned*)p, __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __builtin_bit_cast(float, __hip_atomic_load((unsigned*)p, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}

// Barrier of the `target` blocks sharing one output column tile: counter
// ctr[0] and generation word ctr[MMAD_BN_EXIT].  Each block reads the
// generation (`gen0`, read before it arrives: the caller loads it early),
// adds one arrival; the last arriver resets the counter and bumps the
// generation, the others poll the generation (sc1).  The counter is zero
// again when the barrier opens, whatever tile configuration used it last.
// Bounded: a barrier that does not open within ~2^20 polls (about a second)
// sets the sticky error word and returns false (the caller skips its
// outputs; the host reports it through mmad_ae_status) instead of hanging.
__device__ __forceinline__ unsigned col_gen(const unsigned* ctr) {
  return __hip_atomic_load(ctr + MMAD_BN_EXIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// arrive: after every wave's partial stores have landed, one lane adds an
// arrival; the last arriver resets the counter and opens the barrier
__device__ __forceinline__ void col_arrive(unsigned* ctr, unsigned target, int tid, unsigned* shw) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's partial stores landed
  __syncthreads();                                   // ... and every other wave's
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned last = 0u;
    if (old + 1u == target) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(ctr + MMAD_BN_EXIT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = 1u;
    }
    shw[1] = last;   // read by lane 0 only (col_wait)
  }
}
// wait: lane 0 polls the generation word unless its block arrived last; the
// block joins it at a workgroup barrier (then reads the partials, sc1)
__device__ __forceinline__ bool col_wait(unsigned* ctr, unsigned gen0, unsigned* err, int tid,
                                         unsigned* shw) {
  if (tid == 0) {
    unsigned ok = shw[1];
    for (unsigned spins = 0; !ok && spins < (1u << 20); ++spins) {
      if (col_gen(ctr) != gen0) {
        ok = 1u;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    shw[0] = ok;
  }
  __syncthreads();
  return shw[0] != 0u;
}

}  // namespace

// -------------------------------------------------------------------------
// Train-mode BatchNorm of the producer layer never touches the operands here:
// the forward folds it into the consumer's weights and bias (bn_fold_k: the
// B operand is W*scale, the bias gets sum_k shift*W via bpart partials), the
// dW GEMM contracts the raw activation and fixes up in the epilogue
// (dW = scale[k] * acc + shift[k] * db[n]).  Every GEMM is a plain MFMA
// contraction.
// XCD-aware order (1-D grid).  Under round-robin dispatch, blocks with equal
// bid % 8 share an XCD (speed only, never correctness); each such set gets a
// contiguous range of logical blocks lt; the S split-K blocks of one output
// tile are consecutive in lt (one XCD), and tiles are grouped group_m M-tiles
// at a time so every XCD works on a compact rectangle whose A/B panels stay
// in its L2.
struct TileCoord {
  int tm, tn, tile, sk;
};
__device__ __forceinline__ TileCoord tile_coord(const GemmEpi& ep, int bid, int nblk, int S) {
  TileCoord tc;
  const int ntl = nblk / S;
  const int q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
  const int lt = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  tc.tile = lt / S;
  tc.sk = lt - tc.tile * S;
  const int tiles_m = ntl / ep.tiles_n;
  const int per_group = ep.group_m * ep.tiles_n;
  const int first_m = (tc.tile / per_group) * ep.group_m;
  const int gsz = min(tiles_m - first_m, ep.group_m);
  tc.tm = first_m + (tc.tile % per_group) % gsz;
  tc.tn = (tc.tile % per_group) / gsz;
  return tc;
}

// The body of one output tile; `bid` / `nblk` = the block index / block count.
// Persistent CFG 7 (mmad_gemm_kernel_p): `pre` = this tile's first two K
// stages were issued by the previous tile's epilogue; `next_bid` >= 0 = issue
// that tile's first two stages at the start of this tile's epilogue (its
// stores then drain under the next tile's prologue instead of before it).
// (PST: the persistent kernel's own instantiation -- shared with the ordinary
// kernel, the body's lambdas would have two callers and stay out of line)
template <typename T, typename TO, bool AK, bool BK_, int CFG, int EPI, bool PST = false>
__device__ __forceinline__ void gemm_body(const T* __restrict__ A, int lda, const T* __restrict__ B,
                                          int ldb, int K, const GemmEpi& ep, const int bid,
                                          const int nblk, const int tid_in, const bool pre = false,
                                          const int next_bid = -1) {
  using C = Cfg<CFG>;
  constexpr int BM = C::BM, BN = C::BN, WM = C::WM, WN = C::WN, NS = C::NS, NT = C::NT;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;   // 16x16 MFMA tiles per wave
  constexpr int NW = NT / 64;
  static_assert(WM * WN == NW && TM % 2 == 0, "wave grid");
  using IA = Img<T, AK, BM, NT>;
  using IB = Img<T, BK_, BN, NT>;
  // bf16: every operand layout delivers the natural k order (lane group g owns
  // k = 8g..8g+7), so a K-major operand is one ds_read_b128 per fragment
  constexpr bool NAT = true;
  constexpr int SLOT = IA::BYTES + IB::BYTES;
  constexpr int NL = IA::CHUNKS + IB::CHUNKS;          // vm ops per thread per stage
  constexpr bool FWDLIKE = EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_MSE || EPI == GEMM_EPI_SCORE;
  constexpr bool BIG = CFG == CFG_BIG || CFG == CFG_XST || CFG == CFG_B4;
  constexpr bool XST = CFG == CFG_XST || CFG == CFG_B4 || CFG == CFG_XST1;
  static_assert(!BIG || big_ok<T, EPI>(), "256x256 tile: bf16 forward-type epilogues only");
  static_assert(!XST || xst_ok<T, EPI>(), "CFG 7 / 8 / 9: bf16 eval forward / score only");
  // prefetched bias partials per lane (none for the 256x256 tile: its
  // 128 accumulator registers leave no room to hold them across the loop)
  constexpr int QB = BIG ? 0 : 8;
  constexpr int QG = 32;                               // prefetched dW row-sum partials
  constexpr int OSTRIDE = BN * (int)sizeof(TO) + 16;
  constexpr int OBYTES = BM * OSTRIDE + (EPI == GEMM_EPI_BWD_DATA ? BM * BN / 2 : 0);   // + fp64 [BM/16][BN]
  // fused train-mode BN: per-column merge results (2 x fp64 [BN]) + a flag word
  // (fwd: 4 chunk-group Welford merges + scale/shift; bwd-data: the sums --
  // its chunk-group sums reuse the fp64 piece scratch)
  constexpr int XBYTES = BIG ? 0
                         : EPI == GEMM_EPI_FWD ? 12 * BN * 8 + 2 * BN * 4 + 64
                         : EPI == GEMM_EPI_BWD_DATA ? 6 * BN * 8 + 64 : 0;
  // transposed epilogue staging (bf16 outputs of the forward-type epilogues
  // without a fused BN): the tile goes to LDS column-major, 8 B per lane per
  // MFMA fragment (ds_write_b64), and comes back row-major, 16 B per lane,
  // through ds_read_b64_tr_b16 (tstage_* below); column stride CS, 8-byte
  // granules XOR-swizzled by (col >> 1) & 7: conflict-free on both sides
  constexpr bool TSTG = sizeof(TO) == 2 && (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_MSE ||
                                            EPI == GEMM_EPI_SCORE);
  constexpr int TCS = BM * 2 + 64;
  constexpr int TBYTES = TSTG ? BN * TCS : 0;
  constexpr int LDS_A = (NS * SLOT > OBYTES + XBYTES) ? NS * SLOT : OBYTES + XBYTES;
  constexpr int LDS_BYTES = LDS_A > TBYTES ? LDS_A : TBYTES;
  static_assert((NS - 1) * NL <= 63, "vmcnt range");
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = tid_in, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int S = ep.splitk > 1 ? ep.splitk : 1;
  const int ntl = nblk / S;                 // output tiles
  const TileCoord tc = tile_coord(ep, bid, nblk, S);
  const int tm = tc.tm, tn = tc.tn, tile = tc.tile, sk = tc.sk;
  const int m0 = tm * BM, n0 = tn * BN;
  const int Ks = K / S, kbase = sk * Ks;
  const int nt = (ep.dbg & 1) ? 0 : Ks / IA::BK;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- epilogue constants, loaded before the main loop: their latency hides
  // under it instead of stalling the epilogue.  (Ordinary loads older than
  // every LDS-DMA of the ring; only used after the loop.)
  const int g = lane >> 4, c = lane & 15;
  const int rw = m0 + wm * 16 * TM;  // first row of this wave
  const int cw = n0 + wn * 16 * TN;  // first col of this wave
  float e_b[TN], e_s[TN], e_t[TN], e_p[TN][QB > 0 ? QB : 1];
  // (the 256x256 tile loads them after the loop: no registers to spare)
  auto load_epi_consts = [&]() {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = cw + j * 16 + c;
      e_b[j] = ep.bias ? ep.bias[col] : 0.f;
      e_s[j] = ep.bn_scale ? ep.bn_scale[col] : 1.f;
      e_t[j] = ep.bn_shift ? ep.bn_shift[col] : 0.f;
      if (EPI != GEMM_EPI_SCORE && ep.bpart) {
        // folded-BN bias partials: lane group g takes partials g, g+4, ...
#pragma unroll
        for (int q = 0; q < QB; ++q) {
          const int pp = min(g + 4 * q, ep.bparts - 1);
          e_p[j][q] = ep.bpart[(size_t)pp * ep.bpstride + col];
        }
      }
    }
  };
  if constexpr (FWDLIKE && !BIG && !XST) load_epi_consts();

  // fused BN: this column's barrier generation, read before this block can
  // arrive (its latency hides under the main loop)
  unsigned gen0 = 0u;
  if constexpr (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_BWD_DATA) {
    if (ep.bn_sync && tid == 0) gen0 = col_gen(ep.bn_sync + tn);
  }
  // BatchNorm parameters / statistics of this thread's column (tid % BN, the
  // epilogues' column), read before the main loop: their round trip hides
  // under it instead of following the loop or the column barrier
  float bnp_g = 0.f, bnp_b = 0.f, bnp_rm = 0.f, bnp_rv = 0.f, bnp_mu = 0.f, bnp_rs = 0.f;
  if constexpr ((EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_BWD_DATA) && !BIG) {
    const int bc = n0 + tid % BN;
    const int bcc = bc < ep.N ? bc : ep.N - 1;   // clamped: an unconditional load
    if constexpr (EPI == GEMM_EPI_FWD) {
      if (ep.bn_sync) {
        bnp_g = ep.bn_gamma[bcc];
        bnp_b = ep.bn_beta[bcc];
        if (ep.bn_rmean && tm == 0) {
          bnp_rm = ep.bn_rmean[bcc];
          bnp_rv = ep.bn_rvar[bcc];
        }
      }
    } else {
      if (ep.bn_part) {
        bnp_mu = ep.bn_mean[bc];
        bnp_rs = ep.bn_rstd[bc];
      }
      if (ep.bn_sync) bnp_g = ep.bn_gamma[bcc];
    }
  }
  float e_g[QG];
  // db[n] (bias gradient of this layer's output n) is needed by the dW fix-up
  // (BN producer) and by the fused bias Adam (column-tile-0 blocks)
  const bool need_db = EPI == GEMM_EPI_BWD_WEIGHT && ep.gb_src &&
                       (ep.b_scale || (ep.sm_p && tn == 0));
  if constexpr (EPI == GEMM_EPI_BWD_WEIGHT) {
    if (ep.b_scale) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = cw + j * 16 + c;
        e_s[j] = ep.b_scale[col];
        e_t[j] = ep.b_shift[col];
      }
    }
    if (need_db) {
      // db[n] partials of this block's rows, one row per thread (tid < BM)
      if (tid < BM) {
#pragma unroll
        for (int q = 0; q < QG; ++q) {
          const int pp = min(q, ep.gb_parts - 1);
          e_g[q] = ep.gb_src[(size_t)pp * ep.gb_stride + m0 + tid];
        }
      }
    }
  }

  auto issue = [&](int s) {
    char* base = smem + (s % NS) * SLOT;
    const int k0 = kbase + s * IA::BK;
    issue_stage<T, AK, BM, NT>(base, A, lda, m0, k0, tid);
    issue_stage<T, BK_, BN, NT>(base + IA::BYTES, B, ldb, n0, k0, tid);
  };
  // chunk q (< NL) of stage s: A chunks first, then B
  auto issue_q = [&](int s, int q) {
    char* base = smem + (s % NS) * SLOT;
    const int k0 = kbase + s * IA::BK;
    // persistent body: the chunk's source address is recomputed at every
    // issue (an opaque thread index): hoisted out of the K loop, the 64-bit
    // addresses of every chunk stay live across it and spill, and each
    // scratch reload's vmcnt wait drains the DMA ring
    int t = tid;
    if constexpr (PST) asm volatile("" : "+v"(t));
    if (q < IA::CHUNKS) issue_chunk<T, AK, BM, NT>(base, A, lda, m0, k0, t, q);
    else issue_chunk<T, BK_, BN, NT>(base + IA::BYTES, B, ldb, n0, k0, t, q - IA::CHUNKS);
  };

  // ---- main loop: NS-slot LDS ring, all slots in flight; fragment registers
  // double-buffered one sub-step ahead.  Per stage t:
  //   F1 <- (t, sub 1) issued between the two MFMA halves of F0 = (t, sub 0);
  //   wait stage t+1 landed + own reads of slot t done; barrier; refill slot t
  //   with stage t+NS; F0 <- (t+1, sub 0) between the two halves of F1.
  // The loop bodies are straight-line (peeled: issue phase / tail / last) so
  // hipcc's lgkmcnt bookkeeping stays exact, and sched_barriers pin the order.
  using FR = typename SubFrag<T>::F;
  const int ra = wm * 16 * TM, rb = wn * 16 * TN;
  // Adam-fused dW: the first chunk group of the tile's p / m / v is loaded
  // right after the ring's last DMA issue, so its HBM round trip runs under
  // the K loop's last NS-1 stages instead of after the loop (the tail waits
  // let these APF younger loads stay in flight; APF = 0: not prefetched)
  constexpr int A_CPR = BN * (int)sizeof(TO) / 16;
  constexpr int A_ITERS = BM * A_CPR / NT;
  constexpr int A_AG = A_ITERS < 4 ? A_ITERS : 4;
  // (not for the 8-wave 256x128 / 128x256 tiles: their 48 prefetch registers
  // spill beside the larger accumulator set)
  constexpr bool APF_OK = EPI == GEMM_EPI_BWD_WEIGHT && !BIG && CFG != 1 && CFG != 2 &&
                          3 * NL + 3 * A_AG <= 63;
  floatx4 pf_p[A_AG], pf_m[A_AG], pf_v[A_AG];
  bool pf = false;
  auto adam_prefetch = [&]() {
#pragma unroll
    for (int u = 0; u < A_AG; ++u) {
      const int idx = u * NT + tid;
      const size_t off = (size_t)(m0 + idx / A_CPR) * ep.ldo + n0 + (idx % A_CPR) * (16 / (int)sizeof(TO));
      pf_p[u] = *(const floatx4*)(ep.ad_p + off);
      pf_m[u] = *(const floatx4*)(ep.ad_m + off);
      pf_v[u] = *(const floatx4*)(ep.ad_v + off);
    }
  };
  // the layer's small Adam segment [bias | gamma | beta] this block updates in
  // its epilogue (bias: the column-tile-0 blocks, one row per thread; gamma |
  // beta: 4 per thread of the first tiles): read before the main loop, as
  // nothing else writes it during this launch and its gradients are final
  float smp_p = 0.f, smp_m = 0.f, smp_v = 0.f;
  floatx4 smq_g{}, smq_p{}, smq_m{}, smq_v{};
  bool smq = false;
  if constexpr (APF_OK) {
    if (ep.sm_p) {
      if (tn == 0 && tid < BM && m0 + tid < ep.sm_bNp) {
        smp_p = ep.sm_p[m0 + tid];
        smp_m = ep.sm_m[m0 + tid];
        smp_v = ep.sm_v[m0 + tid];
      }
      const int i4 = ep.sm_bNp + (tile * NT + tid) * 4;
      if (i4 < ep.sm_n) {
        smq_g = *(const floatx4*)(ep.sm_g + i4);
        smq_p = *(const floatx4*)(ep.sm_p + i4);
        smq_m = *(const floatx4*)(ep.sm_m + i4);
        smq_v = *(const floatx4*)(ep.sm_v + i4);
        smq = true;
      }
    }
  }
  // bwd-data with the BatchNorm-backward partials: this thread's pre-BN
  // activations a (16 rows x PPT pieces of one column, the epilogue's own
  // pattern) prefetched the same way, raw (converted only where used)
  constexpr int B_NG = NT / BN, B_PIECES = BM / 16;
  constexpr int B_PPT = (B_PIECES + B_NG - 1) / B_NG;
  constexpr bool BPF_OK = EPI == GEMM_EPI_BWD_DATA && !BIG && B_PIECES % B_NG == 0 && B_PPT <= 2 &&
                          3 * NL + 16 * B_PPT <= 63;
  TO pf_a[BPF_OK ? B_PPT : 1][16];
  bool pfa = false;
  auto bn_a_prefetch = [&]() {
    const TO* an = (const TO*)ep.bn_a;
    const int cc = tid % BN, grp = tid / BN;
#pragma unroll
    for (int u = 0; u < B_PPT; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        pf_a[u][r] = an[(size_t)(m0 + (grp + u * B_NG) * 16 + r) * ep.ldo + n0 + cc];
  };
  if constexpr (BIG) {
    // 256x256 tile (bf16, both operands K-major): a 2-slot ring, one barrier
    // per stage after both 32-deep sub-steps; the fragment registers of a
    // sub-step are re-read row by row under the MFMAs that free them (their
    // lifetimes do not overlap, so the 128 accumulators fit beside them), and
    // stage t+2 is issued over the MFMA rows of stage t+1's first sub-step
    // (the round-3 loop study's "256x256 nb2 st0 di1", profiles/r03d_*)
    if (nt > 0) {
      FR fa[2][TM], fb[2][TN];
      auto rd = [&](int t, int kk, int sl) {
        const char* base = smem + (t % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[sl][i] = frag_bf16<true, true, BM>(base, ra + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[sl][j] = frag_bf16<true, true, BN>(base + IA::BYTES, rb + j * 16, kk, lane);
      };
      int pend = -1;
      // diagnostics (dbg bit 16, loop studies only): no DMA after the
      // prologue (the MFMAs read stale slots)
      const bool d_nodma = ep.dbg & 16;
      if (!(PST && pre)) {
        issue(0);
        if (nt > 1) issue(1);
      }
      // (pre: the previous tile's epilogue stores are younger than these
      // stages -- wait for everything)
      if (nt > 1 && !(PST && pre)) wait_vmcnt<NL>();
      else wait_vmcnt<0>();
      block_barrier();
      rd(0, 0, 0);
      for (int t = 0; t < nt; ++t) {
        const char* base = smem + (t % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = XST ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[0][j], fa[0][i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
          if (pend >= 0 && !d_nodma) {
#pragma unroll
            for (int q = 0; q < NL; ++q)
              if (q * TM / NL == i) issue_q(pend, q);
          }
          if (i == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
              fb[1][j] = frag_bf16<true, true, BN>(base + IA::BYTES, rb + j * 16, 1, lane);
          }
          fa[1][i] = frag_bf16<true, true, BM>(base, ra + i * 16, 1, lane);
        }
        pend = -1;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = XST ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[1][j], fa[1][i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
        if (t + 1 < nt) {
          wait_vmcnt<0>();                   // stage t+1 landed (the only one in flight)
          wait_lgkm0();
          block_barrier();                   // stage t+1 visible; slot t free
          if (t + 2 < nt) pend = t + 2;
          rd(t + 1, 0, 0);
        }
      }
    }
  } else if (nt > 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (s < nt) issue(s);
    if (nt >= NS) wait_vmcnt<(NS - 1) * NL>();
    else wait_vmcnt<0>();
    block_barrier();
    FR f0a[TM], f0b[TN], f1a[TM], f1b[TN];
    read_sub<T, AK, BK_, NAT, BM, BN, TM, TN>(smem, smem + IA::BYTES, ra, rb, 0, lane, f0a, f0b);
    wait_lgkm0();
    auto step = [&](int t, auto issue_c, auto last_c, auto pf_c) {
      constexpr bool ISSUE = decltype(issue_c)::value, LAST = decltype(last_c)::value;
      constexpr bool PF = decltype(pf_c)::value;   // the Adam prefetch is in flight
      const char* sa = smem + (t % NS) * SLOT;
      mma_half<T, TM, TN, 0, XST>(acc, f0a, f0b);
      MMAD_SB();
      read_sub<T, AK, BK_, NAT, BM, BN, TM, TN>(sa, sa + IA::BYTES, ra, rb, 1, lane, f1a, f1b);
      MMAD_SB();
      mma_half<T, TM, TN, 1, XST>(acc, f0a, f0b);
      MMAD_SB();
      if constexpr (!LAST) {
        if constexpr (ISSUE) {
          wait_vmcnt<(NS - 2) * NL>();
        } else if constexpr (PF && APF_OK) {
          wait_tail_x<NL, 3 * A_AG>(nt - t - 2);
        } else if constexpr (PF && BPF_OK) {
          wait_tail_x<NL, 16 * B_PPT>(nt - t - 2);
        } else {
          wait_tail<NL>(nt - t - 2);
        }
        wait_lgkm0();
        block_barrier();                     // stage t+1 visible; slot t free
        MMAD_SB();
      }
      // stage t+NS into the freed slot t, spread over this sub-step's MFMA rows
      auto dma_row = [&](int i) {
        if constexpr (ISSUE) {
#pragma unroll
          for (int q = 0; q < NL; ++q)
            if (q * TM / NL == i) issue_q(t + NS, q);
        }
      };
      mma_half<T, TM, TN, 0, XST>(acc, f1a, f1b, dma_row);
      MMAD_SB();
      if constexpr (!LAST) {
        const char* sn = smem + ((t + 1) % NS) * SLOT;
        read_sub<T, AK, BK_, NAT, BM, BN, TM, TN>(sn, sn + IA::BYTES, ra, rb, 0, lane, f0a, f0b);
      }
      MMAD_SB();
      mma_half<T, TM, TN, 1, XST>(acc, f1a, f1b, dma_row);
      MMAD_SB();
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    int t = 0;
    bool apf = false;
    if constexpr (APF_OK) apf = ep.ad_p != nullptr && nt > NS;
    if constexpr (BPF_OK) apf = ep.bn_part != nullptr && ep.bn_a != nullptr && nt > NS;
    if (apf) {
      // the last issuing stage, then the prefetch behind its DMA
      for (; t < nt - NS - 1; ++t) step(t, T_{}, F_{}, F_{});
      step(t++, T_{}, F_{}, F_{});
      MMAD_SB();
      if constexpr (APF_OK) {
        adam_prefetch();
        pf = true;
      }
      if constexpr (BPF_OK) {
        bn_a_prefetch();
        pfa = true;
      }
      MMAD_SB();
      for (; t < nt - 1; ++t) step(t, F_{}, F_{}, T_{});
      step(nt - 1, F_{}, T_{}, T_{});
    } else {
      for (; t < nt - NS; ++t) step(t, T_{}, F_{}, F_{});
      for (; t < nt - 1; ++t) step(t, F_{}, F_{}, F_{});
      step(nt - 1, F_{}, T_{}, F_{});
    }
  }

  // ---- split-K combine (ticket first, no spin on a block that has not run):
  // the first S-1 blocks of a tile to finish publish their partial tile as an
  // sc1 (write-through) slab + flag; the last one adds the slabs in split
  // order (p0 + p1 + ... : independent of arrival order) and runs the
  // epilogue.  Counters / flags start at 0 (caller memset) and the last block
  // resets them, so consecutive launches on one stream reuse them.
  // (the 256x256 tile never splits: its combine would need a second set of
  // 128 accumulator registers; the dispatcher does not pick it for a split)
  if (!BIG && S > 1) {
    unsigned* cnt = ep.sk_ctl + tile;
    unsigned* flg = ep.sk_ctl + ntl + (size_t)tile * S;
    __syncthreads();
    unsigned* shw = (unsigned*)smem;
    if (tid == 0) shw[0] = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned ticket = shw[0];
    float* slab_t = ep.sk_slab + (size_t)tile * S * (BM * BN);
    const int frag0 = w * TM * TN;
    if (ticket + 1 < (unsigned)S) {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(slab_t + (size_t)sk * (BM * BN), 0, BM * BN * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, acc[i][j]), rs,
                                                 ((frag0 + i * TN + j) * 64 + lane) * 16, 0, 16 /*sc1*/);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flg + sk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {
      // a slice that never publishes (it cannot happen with every block of
      // the grid resident or queued, but a bounded spin must not combine a
      // stale slab): flag the launch as failed and skip the epilogue; the
      // host reads the word with mmad_gemm_status / mmad_ae_status.
      // dbg bit 4 forces the timeout path (tests).
      unsigned timed_out = 0u;
      for (int s2 = 0; s2 < S; ++s2) {
        if (s2 == sk) continue;
        bool ok = false;
        if (!(ep.dbg & 4)) {
          for (unsigned spins = 0; spins < (1u << 24); ++spins) {
            if (__hip_atomic_load(flg + s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
              ok = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        if (!ok) timed_out = 1u;
        __hip_atomic_store(flg + s2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (timed_out)
        __hip_atomic_store(ep.sk_ctl + MMAD_SK_ERR_WORD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      shw[1] = timed_out;
    }
    __syncthreads();
    if (shw[1]) return;
    asm volatile("" ::: "memory");           // every slab load below is sc1
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slab_t, 0, S * BM * BN * 4, 0x00020000);
    // Every load is unconditional and issued before any use (a select of
    // "register or load" per fragment would make hipcc branch around each
    // load and wait for it: one memory round trip per fragment).
    if (S == 2) {
      // p0 + p1 == p1 + p0 (IEEE addition commutes): arrival order is irrelevant
      const int other = (1 - sk) * BM * BN * 4;
      floatx4 ob[TM][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          ob[i][j] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, other + ((frag0 + i * TN + j) * 64 + lane) * 16, 0, 16));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] += ob[i][j];
    } else {
      // ((p0 + p1) + p2) + ... in split order, G slabs per round trip (slot
      // sk was never written: loaded anyway, then replaced by acc).  G = 2
      // / 1 for the larger wave tiles (register budget: no spills).
      constexpr int G = TM * TN <= 4 ? 4 : (TM * TN <= 8 ? 2 : 1);
      floatx4 r[TM][TN];
      for (int t0 = 0; t0 < S; t0 += G) {
        floatx4 lb[G][TM][TN];
#pragma unroll
        for (int u = 0; u < G; ++u)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              lb[u][i][j] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                            rs, (t0 + u) * BM * BN * 4 + ((frag0 + i * TN + j) * 64 + lane) * 16, 0, 16));
              asm volatile("" : "+v"(lb[u][i][j]));   // materialise: no branch around the load
            }
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int t = t0 + u;
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const floatx4 e = t == sk ? acc[i][j] : lb[u][i][j];
              r[i][j] = t == 0 ? e : r[i][j] + e;
            }
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = r[i][j];
    }
  }

  if (ep.dbg & 2) {  // diagnostics: main loop only (keep acc live)
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) sum += acc[i][j][0];
    if (sum == 1.2345e-30f) ((float*)ep.out)[tid] = sum;
    return;
  }
  if constexpr (XST) {
    if (PST && next_bid >= 0) {
      // persistent: the next tile's first two K stages into the ring now (every
      // wave has consumed its last fragments: the barrier orders the refill)
      __syncthreads();
      const TileCoord nc = tile_coord(ep, next_bid, nblk, 1);
#pragma unroll
      for (int st2 = 0; st2 < 2; ++st2) {
        if (st2 < nt) {
          char* base = smem + st2 * SLOT;
          issue_stage<T, AK, BM, NT>(base, A, lda, nc.tm * BM, st2 * IA::BK, tid);
          issue_stage<T, BK_, BN, NT>(base + IA::BYTES, B, ldb, nc.tn * BN, st2 * IA::BK, tid);
        }
      }
    }
    // ===================== CFG 7 epilogue (registers -> HBM) ================
    // acc[i][j] of lane (c, g): output row rw + i*16 + c, columns
    // cw + j*16 + 4g .. +3 (W was the MFMA's first operand).  Per element the
    // same arithmetic as the row-quad epilogue below: act(acc + bias), then
    // the BN-eval affine, masked outside M x N, rounded to bf16.  Column tiles
    // 2h and 2h+1 are stored together: v_permlane16_swap of their quads gives
    // lane g the 8 columns 8(g>>1) .. +7 of tile 2h + (g&1) (16 B).
    // (piecewise-linear activations only: LeakyReLU / ReLU / none; sigmoid /
    // tanh layers run on CFG 6, xst_ok_rt)
    const bool pw_relu = ep.act == MMAD_ACT_RELU;
    const float pw_lo = act_lo_slope(ep.act, ep.slope);
    auto cvec = [&](const float* p, int col, float dflt) -> floatx4 {
      return p ? *(const floatx4*)(p + col) : floatx4{dflt, dflt, dflt, dflt};
    };
    TO* out = (TO*)ep.out;
    const int jl = g & 1, coff = 8 * (g >> 1);
    // score: every reference chunk of the tile loaded in one round trip when
    // they fit (TM x TN/2 <= 8 chunks: the 256x128 tile), per column pair
    // otherwise
    constexpr bool REF_ALL = EPI == GEMM_EPI_SCORE && TM * (TN / 2) <= 8;
    uint4v rall[REF_ALL ? TN / 2 : 1][REF_ALL ? TM : 1];
    if constexpr (REF_ALL) {
      // (one branch around the whole group: a per-chunk "ref ? load : 0"
      // becomes a branch and a wait per load)
      if (ep.ref) {
#pragma unroll
        for (int h = 0; h < TN / 2; ++h)
#pragma unroll
          for (int i = 0; i < TM; ++i)
            rall[h][i] = *(const uint4v*)((const TO*)ep.ref + (size_t)(rw + i * 16 + c) * ep.ldref + cw +
                                          (2 * h + jl) * 16 + coff);
      } else {
#pragma unroll
        for (int h = 0; h < TN / 2; ++h)
#pragma unroll
          for (int i = 0; i < TM; ++i) rall[h][i] = uint4v{0u, 0u, 0u, 0u};
      }
    }
    float rsum[EPI == GEMM_EPI_SCORE ? TM : 1];   // this wave's 64-column row sums (WN = 4)
    float rsum2[EPI == GEMM_EPI_SCORE ? TM : 1][2];   // (WN = 2) the two 64-column halves
#pragma unroll
    for (int h = 0; h < TN / 2; ++h) {
      floatx4 cb[2], cs[2], ct[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int col = cw + (2 * h + u) * 16 + 4 * g;
        cb[u] = cvec(ep.bias, col, 0.f);
        cs[u] = cvec(ep.bn_scale, col, 1.f);
        ct[u] = cvec(ep.bn_shift, col, 0.f);
      }
      const int col0 = cw + (2 * h + jl) * 16 + coff;   // this lane's chunk after the swap
      uint4v rvs[EPI == GEMM_EPI_SCORE ? TM : 1];
      if constexpr (EPI == GEMM_EPI_SCORE) {
        if constexpr (REF_ALL) {
#pragma unroll
          for (int i = 0; i < TM; ++i) rvs[i] = rall[h][i];
        } else if (ep.ref) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            rvs[i] = *(const uint4v*)((const TO*)ep.ref + (size_t)(rw + i * 16 + c) * ep.ldref + col0);
        } else {
#pragma unroll
          for (int i = 0; i < TM; ++i) rvs[i] = uint4v{0u, 0u, 0u, 0u};
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = rw + i * 16 + c;
        unsigned d[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int j = 2 * h + u;
          bf16x4 q;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = cw + j * 16 + 4 * g + r;
            float v = acc[i][j][r];
            v = fmaf(apply_act_pw(v + cb[u][r], pw_relu, pw_lo), cs[u][r], ct[u][r]);
            v = (row < ep.M && col < ep.N) ? v : 0.f;
            q[r] = (bf16)v;
          }
          const uint2v qq = __builtin_bit_cast(uint2v, q);
          d[u][0] = qq[0];
          d[u][1] = qq[1];
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(d[0][0], d[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(d[0][1], d[1][1], false, false);
        const uint4v v = uint4v{s0[0], s1[0], s0[1], s1[1]};
        if (out) *(uint4v*)(out + (size_t)row * ep.ldo + col0) = v;
        if constexpr (EPI == GEMM_EPI_SCORE) {
          const TO* pv = (const TO*)&v;
          const TO* pr = (const TO*)&rvs[i];
          float wv[8];
#pragma unroll
          for (int e = 0; e < 8; e += 4) {
            const floatx4 w4 = cvec(ep.colw, col0 + e, 1.f);
            wv[e] = w4[0]; wv[e + 1] = w4[1]; wv[e + 2] = w4[2]; wv[e + 3] = w4[3];
          }
          float sq = 0.f, dd[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            dd[e] = to_f32<TO>(pv[e]) - to_f32<TO>(pr[e]);
            sq = fmaf(dd[e] * dd[e], wv[e], sq);
          }
          if (ep.diff && row < ep.M) {
            float* dp = ep.diff + (size_t)row * ep.lddiff + col0;
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (col0 + e < ep.N) dp[e] = dd[e];
          }
          // chunks 4h + {0, 1, 2, 3} of the wave's 8 sit in lanes g = 0, 2,
          // 1, 3: (k0 + k1) + (k2 + k3), the row-major butterfly's order
          sq += lane_xor32(sq);
          sq += lane_xor16(sq);
          if constexpr (TN == 4) {
            rsum[i] = h == 0 ? sq : rsum[i] + sq;
          } else {
            // 128 columns per wave: ((Q0 + Q1) + (Q2 + Q3)), written here
            static_assert(TN == 8, "one 128-column group per wave");
            if (h == 0 || h == 2) rsum2[i][h >> 1] = sq;
            else rsum2[i][h >> 1] = rsum2[i][h >> 1] + sq;
            if (h == 3 && g == 0)
              ep.rowsq[(size_t)(cw >> 7) * ep.ldrow + row] = rsum2[i][0] + rsum2[i][1];
          }
        }
      }
    }
    if constexpr (EPI == GEMM_EPI_SCORE && TN == 4) {
      // the two waves of a 128-column group: (k0..k7) + (k8..k15), through
      // [WN][BM] floats of LDS (a persistent block's: behind the ring, which
      // its next tile's stages fill; otherwise at its start)
      static_assert(!PST || NS * SLOT + WN * BM * 4 <= LDS_BYTES, "row-sum exchange beside the ring");
      float* srs = (float*)(smem + (PST ? NS * SLOT : 0));
      __syncthreads();                           // ring reads / every wave's row sums below
      if (g == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i) srs[wn * BM + wm * 16 * TM + i * 16 + c] = rsum[i];
      }
      __syncthreads();
      constexpr int GROUPS = BN / 128;
      static_assert(WN == 2 * GROUPS && NT >= GROUPS * BM, "two waves per 128-column group");
      if (tid < GROUPS * BM) {
        const int gi = tid / BM, rl = tid % BM;
        const float tot = srs[(2 * gi) * BM + rl] + srs[(2 * gi + 1) * BM + rl];
        ep.rowsq[(size_t)((n0 >> 7) + gi) * ep.ldrow + m0 + rl] = tot;
      }
    }
    return;
  }
  if constexpr (FWDLIKE && BIG) load_epi_consts();
  // ===================== epilogue, register phase ==========================
  // per-call values of a graph-captured step come from device memory
  const float* tgt = ep.target;
  float ad_step = ep.ad_step, ad_bc2 = ep.ad_bc2;
  if (ep.dyn) {
    if constexpr (EPI == GEMM_EPI_MSE) tgt = ep.dyn->x;
    if constexpr (EPI == GEMM_EPI_BWD_WEIGHT) {
      ad_step = ep.dyn->ad_step;
      ad_bc2 = ep.dyn->ad_bc2;
    }
  }
  float db_own = 0.f;                        // db[m0 + tid] (tid < BM, need_db)
  if constexpr (EPI == GEMM_EPI_BWD_WEIGHT) {
    if (need_db && tid < BM) {
      // sequential partial order (= the flat reduction's)
#pragma unroll
      for (int q = 0; q < QG; ++q) db_own += q < ep.gb_parts ? e_g[q] : 0.f;
      for (int q = QG; q < ep.gb_parts; ++q) db_own += ep.gb_src[(size_t)q * ep.gb_stride + m0 + tid];
    }
    if (ep.b_scale) {
      __syncthreads();                       // ring LDS no longer read
      float* gbl = (float*)smem;
      if (tid < BM) gbl[tid] = db_own;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float db = gbl[wm * 16 * TM + i * 16 + 4 * g + r];
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j][r] = fmaf(e_s[j], acc[i][j][r], e_t[j] * db);
        }
    }
  }
  // activations: the piecewise-linear ones (LeakyReLU / ReLU / none, the hot
  // path) are applied branch-free inside the register phase below; the
  // others (sigmoid / tanh, FWD / SCORE only) by a pre-pass over the
  // accumulators, acc = act(acc + bias) -- the same value the fused form
  // computes -- after which the register phase applies no activation.  One
  // instance of the register phase either way (two instances cost registers:
  // spills in the 256-row tiles).
  const bool pw_act = !FWDLIKE || EPI == GEMM_EPI_MSE || act_is_linear_piecewise(ep.act);
  const bool pw_relu = ep.act == MMAD_ACT_RELU;
  const float pw_lo = act_lo_slope(ep.act, ep.slope);
  float ebias[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = cw + j * 16 + c;
    float bias = 0.f;
    if constexpr (FWDLIKE) {
      bias = e_b[j];
      if (EPI != GEMM_EPI_SCORE && ep.bpart) {
        // + sum_k shift[k] W[n][k]: lane-group sums, then ((g0+g1)+(g2+g3))
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < QB; ++q) t += g + 4 * q < ep.bparts ? e_p[j][q] : 0.f;
        for (int p = 4 * QB + g; p < ep.bparts; p += 4) t += ep.bpart[(size_t)p * ep.bpstride + col];
        t = sum_lane_groups(t);
        bias += t;
      }
    }
    ebias[j] = bias;
  }
  if constexpr (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_SCORE) {
    if (!pw_act) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = apply_act(acc[i][j][r] + ebias[j], ep.act, ep.slope);
    }
  }
  // MSE: every target value of this lane's accumulators loaded up front, all
  // in flight together (issued inside the loop below they went out a column
  // fragment at a time, one HBM round trip each); the fragment registers of
  // the finished K loop hold them.  Same values, same arithmetic.  c3's MSE
  // GEMM (4096 x 1658 -> 2048) 51.2 -> 39.9 us on its tile, c2's 18.9 -> 16.0
  // (profiles/r10/r10h_mse_target_prefetch_ab.jsonl).  bf16 only: the fp32
  // tiles would spill.
  constexpr bool TPF = EPI == GEMM_EPI_MSE && sizeof(T) == 2 && TM * TN <= 16;
  float tpf[TPF ? TN : 1][TPF ? TM : 1][4];
  if constexpr (TPF) {
    int trow[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) trow[i][r] = (rw + i * 16 + 4 * g + r) % ep.tmod;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = cw + j * 16 + c;
      const int cc = col < ep.N ? col : ep.N - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) tpf[j][i][r] = tgt[(size_t)trow[i][r] * ep.ldt + cc];
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = cw + j * 16 + c;
    const bool cvalid = col < ep.N;
    const float bias = ebias[j];
    float sc = 1.f, sh = 0.f;
    if constexpr (FWDLIKE) {
      sc = e_s[j];
      sh = e_t[j];
    }
    float s1[TM / 2], s2[TM / 2];
#pragma unroll
    for (int p = 0; p < TM / 2; ++p) { s1[p] = 0.f; s2[p] = 0.f; }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rw + i * 16 + 4 * g + r;
        const bool valid = cvalid && row < ep.M;
        float v = acc[i][j][r];
        if (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_SCORE) {
          // pinned: tile-independent (act already applied by the pre-pass
          // when it is not piecewise-linear)
          const float a = apply_act_pw(v + bias, pw_relu, pw_lo);
          v = fmaf(pw_act ? a : v, sc, sh);
          v = valid ? v : 0.f;
          s1[i >> 1] += v;
        } else if (EPI == GEMM_EPI_MSE) {
          // unconditional load at a clamped column (row % tmod is always a
          // target row): a load guarded per element makes hipcc branch around
          // each one and wait for it, one round trip per element
          const float tv = TPF ? tpf[TPF ? j : 0][TPF ? i : 0][r]
                               : tgt[(size_t)(row % ep.tmod) * ep.ldt + (col < ep.N ? col : ep.N - 1)];
          const float d = valid ? v + bias - tv : 0.f;
          v = ep.gscale * d;
          s1[i >> 1] += v;
          s2[i >> 1] += d * d;
        } else if (EPI == GEMM_EPI_BWD_DATA) {
          v = valid ? v : 0.f;
          s1[i >> 1] += v;
        }
        acc[i][j][r] = v;
      }
    }
    if (ep.part) {
#pragma unroll
      for (int p = 0; p < TM / 2; ++p) {
        float a1 = s1[p];
        if constexpr (EPI == GEMM_EPI_BWD_DATA) {
          // (the same value through ds_bpermute: the lane-swap form's two
          // temporaries per reduction spill the fused-BN bwd-data tiles)
          a1 += __shfl_xor(a1, 16);
          a1 += __shfl_xor(a1, 32);
        } else {
          a1 = sum_lane_groups(a1);
        }
        const int crow = rw + p * 32;
        const int chunk = crow / MMAD_PART_ROWS;
        float* part = ep.part + (size_t)chunk * 2 * ep.ldpart;
        if (EPI == GEMM_EPI_FWD) {
          // Welford partial: mean and M2 of the valid rows of this 32-row chunk
          int cnt = ep.M - crow;
          cnt = cnt < 0 ? 0 : (cnt > 32 ? 32 : cnt);
          const float mean = cnt > 0 ? a1 / (float)cnt : 0.f;
          float q = 0.f;
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = crow + ii * 16 + 4 * g + r;
              const float dv = acc[2 * p + ii][j][r] - mean;
              q += (row < ep.M) ? dv * dv : 0.f;
            }
          q = sum_lane_groups(q);
          if (g == 0 && !(ep.dbg & 8)) {
            if (ep.bn_sync) {   // handed to the other blocks of this column: sc1
              st_sc1(part + col, mean);
              st_sc1(part + ep.ldpart + col, q);
            } else {
              part[col] = mean;
              part[ep.ldpart + col] = q;
            }
          }
        } else if (EPI == GEMM_EPI_MSE) {
          float a2 = s2[p];
          a2 = sum_lane_groups(a2);
          if (g == 0) { part[col] = a1; part[ep.ldpart + col] = a2; }
        } else if (EPI == GEMM_EPI_BWD_DATA) {
          if (g == 0) part[col] = a1;
        }
      }
    }
  }


  // ===================== epilogue, LDS-staged coalesced store ===============
  // fused BN (forward): the Welford partials are out -- arrive at the column
  // barrier now, store the a tile while the other blocks catch up
  unsigned* bn_shw = (unsigned*)(smem + OBYTES + XBYTES - 64);
  if constexpr (EPI == GEMM_EPI_FWD && !BIG) {
    if (ep.bn_sync) col_arrive(ep.bn_sync + tn, (unsigned)(ntl / ep.tiles_n), tid, bn_shw);
  }
  __syncthreads();  // main-loop LDS no longer read
  if constexpr (EPI == GEMM_EPI_MSE) {
    if (ep.lossp) {
      // one loss partial per output tile: sum of d^2 = sum (dz/gscale)^2
      float lt_sum = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) lt_sum += acc[i][j][r] * acc[i][j][r];
      lt_sum = wave_sum(lt_sum) / (ep.gscale * ep.gscale);
      float* red = (float*)smem;
      if (lane == 0) red[w] = lt_sum;
      __syncthreads();
      if (tid == 0) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += red[q];
        ep.lossp[tile] = t;
      }
      __syncthreads();
    }
  }
  // transposed staging for this tile.  Only the non-256 FWD tiles can carry a
  // fused BN (whose epilogue re-stages row-major): for every other forward-
  // type tile the choice is a compile-time constant, so the row-major path is
  // not instantiated beside it (registers).  dbg 512 (A/B): row-major b16.
  constexpr bool TSTG_ONLY = TSTG && (EPI != GEMM_EPI_FWD || BIG);
  const bool tstg = TSTG_ONLY ? true : (TSTG && !ep.bn_sync && !(ep.dbg & 512));
  auto tsw = [](int col) { return ((col >> 1) & 7) << 3; };
  if (TSTG && tstg) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int rl0 = wm * 16 * TM + i * 16 + 4 * g;
        const int cl = wn * 16 * TN + j * 16 + c;
        bf16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = (bf16)acc[i][j][r];
        *(bf16x4*)(smem + cl * TCS + ((rl0 * 2) ^ tsw(cl))) = q;
      }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = wm * 16 * TM + i * 16 + 4 * g + r;
          const int cl = wn * 16 * TN + j * 16 + c;
          *(TO*)(smem + rl * OSTRIDE + cl * (int)sizeof(TO)) = from_f32<TO>(acc[i][j][r]);
        }
  }
  __syncthreads();
  constexpr int CPR = BN * (int)sizeof(TO) / 16;  // 16-byte chunks per output row
  constexpr int OEPC = 16 / (int)sizeof(TO);
  constexpr int ITERS = BM * CPR / NT;
  constexpr int CPR128 = 128 * (int)sizeof(TO) / 16;  // chunks per 128-column score group
  TO* out = (TO*)ep.out;
  if (EPI == GEMM_EPI_BWD_WEIGHT && ep.ad_p) {
    // torch.optim.Adam on the dW tile (4 fp32 per chunk), same formula as
    // adam_k.  p/m/v of AG chunks are loaded before any of them is stored
    // (the three state arrays may alias as far as the compiler knows).
    constexpr int AG = ITERS < 4 ? ITERS : 4;
    static_assert(ITERS % AG == 0, "Adam chunk groups");
#pragma unroll
    for (int i0 = 0; i0 < ITERS; i0 += AG) {
      floatx4 P[AG], Mm[AG], Vv[AG];
      size_t off[AG];
#pragma unroll
      for (int u = 0; u < AG; ++u) {
        const int idx = (i0 + u) * NT + tid;
        const int rl = idx / CPR, ch = idx % CPR;
        off[u] = (size_t)(m0 + rl) * ep.ldo + n0 + ch * OEPC;
      }
      static_assert(AG == A_AG && CPR == A_CPR, "prefetch group = first epilogue group");
      if (i0 == 0 && pf) {
        // the first group was loaded under the K loop (adam_prefetch)
#pragma unroll
        for (int u = 0; u < AG; ++u) {
          P[u] = pf_p[u];
          Mm[u] = pf_m[u];
          Vv[u] = pf_v[u];
        }
      } else {
#pragma unroll
        for (int u = 0; u < AG; ++u) {
          P[u] = *(const floatx4*)(ep.ad_p + off[u]);
          Mm[u] = *(const floatx4*)(ep.ad_m + off[u]);
          Vv[u] = *(const floatx4*)(ep.ad_v + off[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < AG; ++u) {
        const int idx = (i0 + u) * NT + tid;
        const int rl = idx / CPR, ch = idx % CPR;
        const uint4v v = *(const uint4v*)(smem + rl * OSTRIDE + ch * 16);
        if (!ep.dw_nostore) *(uint4v*)(out + off[u]) = v;
        adam4(P[u], Mm[u], Vv[u], __builtin_bit_cast(floatx4, v), ep.ad_w1, ep.ad_w2, ep.ad_eps,
              ad_step, ad_bc2);
        bf16x4 sh;
#pragma unroll
        for (int e = 0; e < 4; ++e) sh[e] = (bf16)P[u][e];
        *(floatx4*)(ep.ad_p + off[u]) = P[u];
        *(floatx4*)(ep.ad_m + off[u]) = Mm[u];
        *(floatx4*)(ep.ad_v + off[u]) = Vv[u];
        if (ep.ad_shadow) *(bf16x4*)((bf16*)ep.ad_shadow + off[u]) = sh;
      }
    }
  } else if (TSTG && tstg) {
    // read back row-major: iteration u covers a 16-row x 32-column block
    // (row block rb = wave's, column block cb); lane (n = lane & 15, g = lane >> 4)
    // gets row rbase + n, columns cbase + 8g .. + 7 (two tr-reads of 4), one
    // 16-B store.  A wave walks its row blocks, and per row block the column
    // blocks in order, so the 4 blocks of a 128-column score group are
    // consecutive iterations of one lane.
    constexpr int RB = BM / 16, CB = BN / 32, RBW = RB / NW, NB = RBW * CB;
    static_assert(!TSTG || (RB % NW == 0 && NB == ITERS), "transposed staging geometry");
    const int n16 = lane & 15, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const MMAD_LDS char* lds = (const MMAD_LDS char*)smem;
    uint4v rvs[EPI == GEMM_EPI_SCORE ? NB : 1];
    if constexpr (EPI == GEMM_EPI_SCORE) {
      if (ep.ref) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int rbase = (w * RBW + u / CB) * 16, cbase = (u % CB) * 32;
          rvs[u] = *(const uint4v*)((const TO*)ep.ref + (size_t)(m0 + rbase + n16) * ep.ldref + n0 +
                                    cbase + 8 * g);
        }
      } else {
#pragma unroll
        for (int u = 0; u < NB; ++u) rvs[u] = uint4v{0u, 0u, 0u, 0u};
      }
    }
    float gpart[2] = {0.f, 0.f};   // SCORE: (T0 + T1), then T2 of one 128-column group
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int rbase = (w * RBW + u / CB) * 16, cbase = (u % CB) * 32;
      const int k1 = cbase + 8 * g + q4, k2 = k1 + 4;
      const int rb2 = (rbase + 4 * p4) * 2;
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (MMAD_LDS short4v*)(lds + k1 * TCS + (rb2 ^ tsw(k1))));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (MMAD_LDS short4v*)(lds + k2 * TCS + (rb2 ^ tsw(k2))));
      const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
      const bf16x8 v8 = __builtin_shufflevector(l4, h4, 0, 1, 2, 3, 4, 5, 6, 7);
      const uint4v v = __builtin_bit_cast(uint4v, v8);
      const int row = m0 + rbase + n16;
      const int col = n0 + cbase + 8 * g;
      if (out) *(uint4v*)(out + (size_t)row * ep.ldo + col) = v;
      if constexpr (EPI == GEMM_EPI_SCORE) {
        const uint4v rv = rvs[u];
        const TO* pv = (const TO*)&v;
        const TO* pr = (const TO*)&rv;
        float wv[8];
#pragma unroll
        for (int e = 0; e < 8; e += 4) {
          const floatx4 w4 = ep.colw ? *(const floatx4*)(ep.colw + col + e) : floatx4{1.f, 1.f, 1.f, 1.f};
          wv[e] = w4[0]; wv[e + 1] = w4[1]; wv[e + 2] = w4[2]; wv[e + 3] = w4[3];
        }
        float sq = 0.f, dd[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          dd[e] = to_f32<TO>(pv[e]) - to_f32<TO>(pr[e]);
          sq = fmaf(dd[e] * dd[e], wv[e], sq);
        }
        if (ep.diff && row < ep.M) {
          float* dp = ep.diff + (size_t)row * ep.lddiff + col;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (col + e < ep.N) dp[e] = dd[e];
        }
        // the 16 chunks k = 4 (cb % 4) + g of a 128-column group combine as
        // the row-major path's butterfly (k ^ 1, k ^ 2, k ^ 4, k ^ 8):
        // lanes g ^ 1 and g ^ 2 here, then the group's blocks in registers
        sq = sum_lane_groups(sq);
        const int qb = (u % CB) & 3;
        if (qb == 0 || qb == 2) gpart[qb >> 1] = sq;
        else if (qb == 1) gpart[0] = gpart[0] + sq;
        else {
          const float tot = gpart[0] + (gpart[1] + sq);
          if (g == 0) ep.rowsq[(size_t)(col / 128) * ep.ldrow + row] = tot;
        }
      }
    }
  } else {
    // SCORE: every reference chunk loaded before the loop's stores.  ref
    // null = 0 (NAP run: sum of squared outputs); colw: per-column weights
    uint4v rvs[EPI == GEMM_EPI_SCORE ? ITERS : 1];
    if constexpr (EPI == GEMM_EPI_SCORE) {
      // one branch around the whole group (a per-chunk "ref ? load : 0"
      // became a branch per load and a wait after the first one)
      if (ep.ref) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
          const int idx = it * NT + tid;
          const int rl = idx / CPR, ch = idx % CPR;
          rvs[it] = *(const uint4v*)((const TO*)ep.ref + (size_t)(m0 + rl) * ep.ldref + n0 + ch * OEPC);
        }
      } else {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) rvs[it] = uint4v{0u, 0u, 0u, 0u};
      }
    }
    // SCORE per-column weights of this thread's columns (NAP run; 1 without)
    float wcol[EPI == GEMM_EPI_SCORE ? OEPC : 1];
    if constexpr (EPI == GEMM_EPI_SCORE && NT % CPR == 0) {
      const int col0 = n0 + (tid % CPR) * OEPC;
      if (ep.colw) {
#pragma unroll
        for (int e = 0; e < OEPC; e += 4) {
          const floatx4 w4 = *(const floatx4*)(ep.colw + col0 + e);
          wcol[e] = w4[0]; wcol[e + 1] = w4[1]; wcol[e + 2] = w4[2]; wcol[e + 3] = w4[3];
        }
      } else {
#pragma unroll
        for (int e = 0; e < OEPC; ++e) wcol[e] = 1.f;
      }
    }
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = it * NT + tid;
      const int rl = idx / CPR, ch = idx % CPR;
      const uint4v v = *(const uint4v*)(smem + rl * OSTRIDE + ch * 16);
      const int row = m0 + rl;
      const int col = n0 + ch * OEPC;
      if (out) {
        *(uint4v*)(out + (size_t)row * ep.ldo + col) = v;
      }
      if constexpr (EPI == GEMM_EPI_SCORE) {
        const uint4v rv = rvs[it];
        const TO* pv = (const TO*)&v;
        const TO* pr = (const TO*)&rv;
        float sq = 0.f;
        float dd[OEPC];
        float wv[OEPC];
        if constexpr (NT % CPR == 0) {
          // this thread's columns are the same in every iteration: loaded once
#pragma unroll
          for (int e = 0; e < OEPC; ++e) wv[e] = wcol[e];
        } else {
#pragma unroll
          for (int e = 0; e < OEPC; e += 4) {
            const floatx4 w4 = ep.colw ? *(const floatx4*)(ep.colw + col + e) : floatx4{1.f, 1.f, 1.f, 1.f};
            wv[e] = w4[0]; wv[e + 1] = w4[1]; wv[e + 2] = w4[2]; wv[e + 3] = w4[3];
          }
        }
#pragma unroll
        for (int e = 0; e < OEPC; ++e) {
          dd[e] = to_f32<TO>(pv[e]) - to_f32<TO>(pr[e]);
          sq = fmaf(dd[e] * dd[e], wv[e], sq);
        }
        if (ep.diff && row < ep.M) {
          float* dp = ep.diff + (size_t)row * ep.lddiff + col;
#pragma unroll
          for (int e = 0; e < OEPC; ++e)
            if (col + e < ep.N) dp[e] = dd[e];
        }
#pragma unroll
        for (int o = 1; o < CPR128; o <<= 1) sq += __shfl_xor(sq, o);
        if (ch % CPR128 == 0) ep.rowsq[(size_t)(col / 128) * ep.ldrow + row] = sq;
      }
    }
  }
  if constexpr (EPI == GEMM_EPI_FWD && !BIG) {
    if (ep.bn_sync) {
      // ---- fused BatchNorm(train) of this layer (layers/fc_layer.py:37-48,
      // Linear -> act -> BN): whole-batch mean / variance merged from every
      // block's Welford partials (one sequential chunk order: every block of
      // the column computes the same bits), then y = a*scale + shift from the
      // fp32 activations still in registers
      const unsigned tiles_m = (unsigned)(ntl / ep.tiles_n);
      double* s_gn = (double*)(smem + OBYTES);          // [4][BN] group merges
      double* s_gm = s_gn + 4 * BN;
      double* s_gq = s_gm + 4 * BN;
      float* s_sc = (float*)(s_gq + 4 * BN);
      float* s_sh = s_sc + BN;
      static_assert(12 * BN * 8 + 2 * BN * 4 <= XBYTES - 64, "fused-BN scratch");
      if (!col_wait(ep.bn_sync + tn, gen0, ep.bn_err, tid, bn_shw)) return;
      {
        // chunk group q (= 0..3) merges partials q, q+4, ... in order (Chan et
        // al. pairwise update); the threads of a column split the groups;
        // every partial of a group is loaded before the first use
        constexpr int NGT = NT / BN;
        const int cc = tid % BN, grp = tid / BN, col = n0 + cc;
        const int nparts = (int)tiles_m * BM / MMAD_PART_ROWS;   // a multiple of 4
        for (int q = grp; q < 4; q += NGT) {
          double n = 0.0, mean = 0.0, m2 = 0.0;
          constexpr int U = 8;
          for (int u0 = 0; u0 < nparts / 4; u0 += U) {
            float mb[U], qb[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int i = q + 4 * min(u0 + u, nparts / 4 - 1);
              mb[u] = ld_sc1(ep.part + (size_t)i * 2 * ep.ldpart + col);
              qb[u] = ld_sc1(ep.part + ((size_t)i * 2 + 1) * ep.ldpart + col);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int i = q + 4 * (u0 + u);
              int cnt = ep.M - i * MMAD_PART_ROWS;
              cnt = cnt < 0 ? 0 : (cnt > MMAD_PART_ROWS ? MMAD_PART_ROWS : cnt);
              if (u0 + u >= nparts / 4 || cnt == 0) continue;
              const double nb = (double)cnt, nn = n + nb, d = (double)mb[u] - mean;
              mean += d * (nb / nn);
              m2 += (double)qb[u] + d * d * (n * nb / nn);
              n = nn;
            }
          }
          s_gn[q * BN + cc] = n;
          s_gm[q * BN + cc] = mean;
          s_gq[q * BN + cc] = m2;
        }
      }
      __syncthreads();
      if (tid < BN) {
        const int c = n0 + tid;
        double n = 0.0, mean = 0.0, m2 = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double nb = s_gn[q * BN + tid];
          if (nb == 0.0) continue;
          const double nn = n + nb, d = s_gm[q * BN + tid] - mean;
          mean += d * (nb / nn);
          m2 += s_gq[q * BN + tid] + d * d * (n * nb / nn);
          n = nn;
        }
        const float var = n > 0.0 ? (float)(m2 / n) : 0.f;
        const float mu = (float)mean;
        float sc = 0.f, sh = 0.f;
        if (c < ep.N) {
          const float rstd = (float)(1.0 / sqrt((double)var + (double)ep.bn_eps));
          sc = bnp_g * rstd;                 // gamma / beta of column c (prefetched)
          sh = bnp_b - mu * sc;
          if (tm == 0) {
            ep.bn_save_mean[c] = mu;
            ep.bn_save_rstd[c] = rstd;
            if (ep.bn_rmean) {
              const float unb = ep.M > 1 ? var * (float)ep.M / (float)(ep.M - 1) : var;
              ep.bn_rmean[c] = (1.f - ep.bn_mom) * bnp_rm + ep.bn_mom * mu;
              ep.bn_rvar[c] = (1.f - ep.bn_mom) * bnp_rv + ep.bn_mom * unb;
            }
          }
        } else if (tm == 0) {
          ep.bn_save_mean[c] = 0.f;
          ep.bn_save_rstd[c] = 0.f;
        }
        s_sc[tid] = sc;
        s_sh[tid] = sh;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rl = wm * 16 * TM + i * 16 + 4 * g + r;
            const int cl = wn * 16 * TN + j * 16 + c;
            // from the stored (TO-rounded) a, as the backward's xhat sees it
            const float av = to_f32<TO>(from_f32<TO>(acc[i][j][r]));
            const float yv = m0 + rl < ep.M ? av * s_sc[cl] + s_sh[cl] : 0.f;
            *(TO*)(smem + rl * OSTRIDE + cl * (int)sizeof(TO)) = from_f32<TO>(yv);
          }
      __syncthreads();
      TO* yo = (TO*)ep.bn_y;
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int idx = it * NT + tid;
        const int rl = idx / CPR, ch = idx % CPR;
        const uint4v v = *(const uint4v*)(smem + rl * OSTRIDE + ch * 16);
        *(uint4v*)(yo + (size_t)(m0 + rl) * ep.ldo + n0 + ch * OEPC) = v;
      }
    }
  }
  if constexpr (EPI == GEMM_EPI_BWD_WEIGHT) {
    if (ep.sm_p) {   // with or without the weight tile's own Adam (ad_p)
      // the layer's small segment [bias | gamma | beta].  Bias: the
      // column-tile-0 blocks, one output row per thread, g = db (computed
      // above from the same partials the flat path reduces, same order).
      if (tn == 0 && tid < BM && m0 + tid < ep.sm_bNp) {
        const int n = m0 + tid;
        float g = ep.gb_src ? (n < ep.sm_bN ? db_own : 0.f) : ep.sm_g[n];
        if (ep.gb_src) ep.sm_g[n] = g;
        float pp, mm, vv;
        if constexpr (APF_OK) {
          pp = smp_p;                        // prefetched before the main loop
          mm = smp_m;
          vv = smp_v;
        } else {
          pp = ep.sm_p[n];
          mm = ep.sm_m[n];
          vv = ep.sm_v[n];
        }
        adam_elem(pp, mm, vv, g, ep.ad_w1, ep.ad_w2, ep.ad_eps, ad_step, ad_bc2);
        ep.sm_p[n] = pp;
        ep.sm_m[n] = mm;
        ep.sm_v[n] = vv;
      }
      // gamma | beta (grads already final), 4 per thread over all tiles
      int q = tile * NT + tid;
      if (smq) {
        // the first chunk was read before the main loop
        const int i4 = ep.sm_bNp + q * 4;
        floatx4 pp = smq_p, mm = smq_m, vv = smq_v;
        adam4(pp, mm, vv, smq_g, ep.ad_w1, ep.ad_w2, ep.ad_eps, ad_step, ad_bc2);
        *(floatx4*)(ep.sm_p + i4) = pp;
        *(floatx4*)(ep.sm_m + i4) = mm;
        *(floatx4*)(ep.sm_v + i4) = vv;
        q += ntl * NT;
      }
      for (; ep.sm_bNp + q * 4 < ep.sm_n; q += ntl * NT) {
        const int i4 = ep.sm_bNp + q * 4;
        const floatx4 gg = *(const floatx4*)(ep.sm_g + i4);
        floatx4 pp = *(floatx4*)(ep.sm_p + i4), mm = *(floatx4*)(ep.sm_m + i4);
        floatx4 vv = *(floatx4*)(ep.sm_v + i4);
        adam4(pp, mm, vv, gg, ep.ad_w1, ep.ad_w2, ep.ad_eps, ad_step, ad_bc2);
        *(floatx4*)(ep.sm_p + i4) = pp;
        *(floatx4*)(ep.sm_m + i4) = mm;
        *(floatx4*)(ep.sm_v + i4) = vv;
      }
    }
  }
  if constexpr (EPI == GEMM_EPI_BWD_DATA) {
    if (ep.bn_part) {
      // sum over rows of dy and dy*xhat, xhat = (a - mean)*rstd, per 64-row
      // chunk, in fp64 (torch's CPU BatchNorm backward reduces in double) and
      // in one canonical order for every tile configuration: 16-row pieces
      // summed row by row, then ((p0 + p1) + p2) + p3 per chunk.  Pieces
      // pc = grp, grp + NG, ... of this thread stay in registers; the two sums
      // go through one [PIECES][BN] fp64 LDS scratch in turn.
      constexpr int NG = NT / BN;      // thread groups per column
      constexpr int PIECES = BM / 16;  // 16-row pieces of the tile
      constexpr int PPT = (PIECES + NG - 1) / NG;   // pieces per thread
      const int cc = tid % BN, grp = tid / BN;
      const int col = n0 + cc;
      const double mu = bnp_mu, rs = bnp_rs;   // bn_mean / bn_rstd[col] (prefetched)
      const TO* an = (const TO*)ep.bn_a;
      double* scr = (double*)(smem + BM * OSTRIDE);    // [PIECES][BN]
      double ps1[PPT], ps2[PPT];
      // fused BN: this thread's a values kept for the dz pass (up to 32
      // registers; the 8-wave 256-row / 256-column tiles reload them instead)
      constexpr bool AREG = PPT <= 2;
      float areg[AREG ? PPT : 1][16];
      // this thread's a values: the ones prefetched under the K loop, or all
      // loaded here in one block (issued together, one round trip)
      TO araw[PPT][16];
      bool have_a = false;
      if constexpr (BPF_OK && PPT == B_PPT) {
        if (pfa) {
#pragma unroll
          for (int u = 0; u < PPT; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) araw[u][r] = pf_a[u][r];
          have_a = true;
        }
      }
      if (!have_a) {
#pragma unroll
        for (int u = 0; u < PPT; ++u) {
          const int pc = grp + u * NG;
          if (pc < PIECES) {
#pragma unroll
            for (int r = 0; r < 16; ++r) araw[u][r] = an[(size_t)(m0 + pc * 16 + r) * ep.ldo + col];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        const int pc = grp + u * NG;
        double s1 = 0.0, s2 = 0.0;
        if (pc < PIECES) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = pc * 16 + r;
            const double dy = to_f32<TO>(*(const TO*)(smem + rl * OSTRIDE + cc * (int)sizeof(TO)));
            const float avf = to_f32<TO>(araw[u][r]);
            if constexpr (AREG) areg[u][r] = avf;   // kept for the fused dz below
            const double av = avf;
            s1 += dy;
            s2 += dy * ((av - mu) * rs);
          }
        }
        ps1[u] = s1;
        ps2[u] = s2;
      }
#pragma unroll
      for (int which = 0; which < 2; ++which) {
#pragma unroll
        for (int u = 0; u < PPT; ++u) {
          const int pc = grp + u * NG;
          if (pc < PIECES) scr[pc * BN + cc] = which ? ps2[u] : ps1[u];
        }
        __syncthreads();
        for (int c4 = grp; c4 < BM / 64; c4 += NG) {
          double t = scr[(4 * c4) * BN + cc];
#pragma unroll
          for (int q = 1; q < 4; ++q) t += scr[(4 * c4 + q) * BN + cc];
          double* dst = ep.bn_part + (size_t)((m0 + c4 * 64) / 64) * 2 * ep.ldo + which * ep.ldo + col;
          if (ep.bn_sync) st_sc1(dst, t);   // handed to the other blocks of this column
          else *dst = t;
        }
        __syncthreads();
      }
      if (ep.bn_sync) {
        // ---- fused BatchNorm(train) + activation backward of the producer:
        // whole-batch sums from every block's partials, then
        // dz = act'(a) * gamma*rstd/M * (M dy - sum dy - xhat sum dy*xhat)
        // (fp64 bracket, as bn_bwd_apply_k) in place in the staged tile
        const unsigned tiles_m = (unsigned)(ntl / ep.tiles_n);
        double* s_g1 = scr;                               // [4][BN] group sums (scr is free here)
        double* s_g2 = (double*)(smem + OBYTES);          // [4][BN]
        double* s_t1 = s_g2 + 4 * BN;
        double* s_t2 = s_t1 + BN;
        static_assert(PIECES >= 4, "group sums need 4 x BN doubles of the piece scratch");
        static_assert(6 * BN * 8 <= XBYTES - 64, "fused-BN scratch");
        col_arrive(ep.bn_sync + tn, tiles_m, tid, bn_shw);
        if (!col_wait(ep.bn_sync + tn, gen0, ep.bn_err, tid, bn_shw)) return;
        {
          // chunk group q (= 0..3) sums partials q, q+4, ... in order; the
          // threads of a column split the groups, each group's loads in flight
          // together; then ((g0 + g1) + g2) + g3
          const int nch = (int)tiles_m * BM / 64;
          for (int q = grp; q < 4; q += NG) {
            double t1 = 0.0, t2 = 0.0;
            constexpr int U = 8;
            const int per = (nch - q + 3) / 4;          // chunks q, q+4, ... < nch
            for (int u0 = 0; u0 < per; u0 += U) {
              double p1[U], p2[U];
#pragma unroll
              for (int u = 0; u < U; ++u) {
                const int i = q + 4 * min(u0 + u, per - 1);
                p1[u] = ld_sc1(ep.bn_part + (size_t)i * 2 * ep.ldo + col);
                p2[u] = ld_sc1(ep.bn_part + ((size_t)i * 2 + 1) * ep.ldo + col);
              }
#pragma unroll
              for (int u = 0; u < U; ++u)
                if (u0 + u < per) { t1 += p1[u]; t2 += p2[u]; }
            }
            s_g1[q * BN + cc] = t1;
            s_g2[q * BN + cc] = t2;
          }
        }
        __syncthreads();
        if (tid < BN) {
          const int c = n0 + tid;
          double t1 = ((s_g1[tid] + s_g1[BN + tid]) + s_g1[2 * BN + tid]) + s_g1[3 * BN + tid];
          double t2 = ((s_g2[tid] + s_g2[BN + tid]) + s_g2[2 * BN + tid]) + s_g2[3 * BN + tid];
          if (c >= ep.N) { t1 = 0.0; t2 = 0.0; }
          if (tm == 0) {
            ep.bn_dbeta[c] = (float)t1;
            ep.bn_dgamma[c] = (float)t2;
          }
          s_t1[tid] = t1;
          s_t2[tid] = t2;
        }
        __syncthreads();
        const double t1 = s_t1[cc], t2 = s_t2[cc];
        const double cf = col < ep.N ? (double)bnp_g * rs / (double)ep.M : 0.0;
        const double Md = (double)ep.M;
        // (the piece sums go straight to the fp64 piece scratch: its group-sum
        // use above is finished)
#pragma unroll AREG ? PPT : 1
        for (int u = 0; u < PPT; ++u) {
          const int pc = grp + u * NG;
          double sz = 0.0;
          if (pc < PIECES) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = pc * 16 + r;
              TO* slot = (TO*)(smem + rl * OSTRIDE + cc * (int)sizeof(TO));
              const double dy = to_f32<TO>(*slot);
              float av;
              if constexpr (AREG) av = areg[u][r];
              else av = to_f32<TO>(an[(size_t)(m0 + rl) * ep.ldo + col]);
              const double xh = ((double)av - mu) * rs;
              const double da = cf * (Md * dy - t1 - xh * t2);
              float d = (float)(da * (double)act_grad_from_out(av, ep.bn_act, ep.slope));
              d = m0 + rl < ep.M ? d : 0.f;
              const TO dt = from_f32<TO>(d);
              *slot = dt;
              sz += (double)to_f32<TO>(dt);
            }
            scr[pc * BN + cc] = sz;
          }
        }
        __syncthreads();
        for (int c4 = grp; c4 < BM / 64; c4 += NG) {
          double t = scr[(4 * c4) * BN + cc];
#pragma unroll
          for (int q = 1; q < 4; ++q) t += scr[(4 * c4 + q) * BN + cc];
          ep.bn_dbpart[(size_t)((m0 + c4 * 64) / 64) * ep.ldo + col] = (float)t;
        }
        // coalesced store of the dz tile
        TO* dzo = (TO*)ep.bn_dz;
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
          const int idx = it * NT + tid;
          const int rl = idx / CPR, ch = idx % CPR;
          const uint4v v = *(const uint4v*)(smem + rl * OSTRIDE + ch * 16);
          *(uint4v*)(dzo + (size_t)(m0 + rl) * ep.ldo + n0 + ch * OEPC) = v;
        }
      }
    }
  }
}

template <typename T, typename TO, bool AK, bool BK_, int CFG, int EPI>
__global__ __launch_bounds__(Cfg<CFG>::NT, 1) void mmad_gemm_kernel(const T* __restrict__ A, int lda,
                                                           const T* __restrict__ B, int ldb, int K,
                                                           GemmEpi ep) {
  gemm_body<T, TO, AK, BK_, CFG, EPI>(A, lda, B, ldb, K, ep, blockIdx.x, gridDim.x, threadIdx.x);
}

// Persistent form (knob 12) of the forward-type bf16 GEMMs at large row
// counts (C5 scoring: 65,536 rows, 8 rounds of tiles): one block per resident
// slot walks the logical tiles v = blockIdx.x, + gridDim.x, ... (gridDim a
// multiple of 8, so v & 7 -- the XCD label of the tile order -- stays the
// block's own).  Per tile the body is gemm_body's, so every output bit is the
// non-persistent kernel's; what changes is that the next tile's prologue
// (LDS-DMA of its first stages) is issued right after this tile's epilogue
// stores instead of after a block retirement and a new dispatch.  Never with
// a fused BN (its column barrier needs every tile of a column resident) or a
// split (the combine's last arriver waits for its sibling slices).
template <typename T, typename TO, bool AK, bool BK_, int CFG, int EPI>
__global__ __launch_bounds__(Cfg<CFG>::NT, 1) void mmad_gemm_kernel_p(const T* __restrict__ A, int lda,
                                                             const T* __restrict__ B, int ldb, int K,
                                                             GemmEpi ep) {
  const int nt = ep.persist_tiles;
  for (int v = blockIdx.x; v < nt; v += gridDim.x) {
    // the thread index passes through an opaque move every tile, so nothing
    // derived from it is hoisted out of the tile loop (hoisted, those values
    // stay live across the whole body and the 256-row tiles spill)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    if constexpr (CFG == CFG_XST) {
      const int nx = v + (int)gridDim.x;
      gemm_body<T, TO, AK, BK_, CFG, EPI, true>(A, lda, B, ldb, K, ep, v, nt, tid, v != (int)blockIdx.x,
                                                nx < nt ? nx : -1);
    } else {
      gemm_body<T, TO, AK, BK_, CFG, EPI, true>(A, lda, B, ldb, K, ep, v, nt, tid);
    }
    __syncthreads();
  }
}

#ifdef MMAD_GEMM_B4_TU
// ---- the 4-wave 256x256 translation unit: its launcher only --------------
int mmad_gemm_b4_launch(int epi, const void* A, int lda, const void* B, int ldb, int Mp, int Np, int K,
                        const GemmEpi& ep, hipStream_t s) {
  dim3 grd((Mp / 256) * (Np / 256)), blk(256);
  auto go = [&](auto kern) {
    if (ep.done_ev || ep.start_ev)
      hipExtLaunchKernelGGL(kern, grd, blk, 0u, s, ep.start_ev, ep.done_ev, 0u, (const bf16*)A, lda,
                            (const bf16*)B, ldb, K, ep);
    else
      kern<<<grd, blk, 0, s>>>((const bf16*)A, lda, (const bf16*)B, ldb, K, ep);
  };
  if (epi == GEMM_EPI_FWD) go(mmad_gemm_kernel<bf16, bf16, true, true, CFG_B4, GEMM_EPI_FWD>);
  else if (epi == GEMM_EPI_SCORE) go(mmad_gemm_kernel<bf16, bf16, true, true, CFG_B4, GEMM_EPI_SCORE>);
  else {
    mmad_set_error("gemm: tile 8 runs the eval forward / score epilogues only");
    return MMAD_EUNSUPPORTED;
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}
#else
int mmad_gemm_b4_launch(int epi, const void* A, int lda, const void* B, int ldb, int Mp, int Np, int K,
                        const GemmEpi& ep, hipStream_t s);

// -------------------------------------------------------------------------
// host-side planning and launch
// -------------------------------------------------------------------------
static bool cfg_fits(int cfg, int Mp, int Np, int epi, int dtype) {
  if (Mp % CFG_BM[cfg] || Np % CFG_BN[cfg]) return false;
  if (is_big(cfg) && !big_ok_rt(dtype, epi)) return false;
  if (is_xst(cfg) && !(dtype == MMAD_BF16 && (epi == GEMM_EPI_FWD || epi == GEMM_EPI_SCORE))) return false;
  // the score epilogue reduces rows over 128-column groups inside one tile
  if (epi == GEMM_EPI_SCORE && CFG_BN[cfg] < 128) return false;
  return true;
}

int mmad_gemm_ntiles(int cfg, int Mp, int Np) { return (Mp / CFG_BM[cfg]) * (Np / CFG_BN[cfg]); }

int mmad_gemm_tiles(int Mp, int Np) { return (Mp / 64) * (Np / 64); }

// static choice when autotuning is off or impossible (stream capture)
template <typename Pred>
static int heuristic_cfg(int Mp, int Np, int epi, Pred allowed) {
  const int order[] = {CFG_BIG, 1, 0, 5, 4, 3};
  const int want[] = {512, 200, 200, 200, 160, 0};
  for (int i = 0; i < 6; ++i) {
    const int c = order[i];
    if (!allowed(c)) continue;
    if (mmad_gemm_ntiles(c, Mp, Np) >= want[i]) return c;
  }
  for (int c : {4, 0, 3, 5, 2, 1})
    if (allowed(c)) return c;
  (void)Mp; (void)Np; (void)epi;
  return -1;
}
static int heuristic_cfg(int Mp, int Np, int epi, int dtype) {
  return heuristic_cfg(Mp, Np, epi, [&](int c) { return cfg_fits(c, Mp, Np, epi, dtype); });
}

// group height balancing the per-XCD A-panel (gm*BM rows) and B-panel
// ((ntiles/8/gm)*BN cols) footprints
static int plan_group_m(int ntiles, int tiles_m, int BM, int BN) {
  const double per_xcd = ntiles / 8.0;
  int gm = (int)(sqrt(per_xcd * BN / BM) + 0.5);
  const int env_gm = mmad_group_override();
  if (env_gm > 0) gm = env_gm;
  return gm < 1 ? 1 : (gm > tiles_m ? tiles_m : gm);
}

// the configurations that have a persistent instantiation (the large-row tiles)
constexpr bool persist_cfg(int cfg) { return cfg == 1 || cfg == 2 || cfg == CFG_BIG || cfg == CFG_XST; }

template <typename T, typename TO, bool AK, bool BK_, int EPI>
static const void* persist_kernel(int cfg) {
  if constexpr (sizeof(T) == 2 && (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_MSE || EPI == GEMM_EPI_SCORE)) {
    switch (cfg) {
      case 1: return (const void*)mmad_gemm_kernel_p<T, TO, AK, BK_, 1, EPI>;
      case 2: return (const void*)mmad_gemm_kernel_p<T, TO, AK, BK_, 2, EPI>;
      case CFG_BIG: return (const void*)mmad_gemm_kernel_p<T, TO, AK, BK_, CFG_BIG, EPI>;
      case CFG_XST:
        if constexpr (xst_ok<T, EPI>()) return (const void*)mmad_gemm_kernel_p<T, TO, AK, BK_, CFG_XST, EPI>;
        return nullptr;
      default: return nullptr;
    }
  }
  return nullptr;
}

namespace {
std::mutex g_pcap_mu;
std::map<long, int> g_pcap;   // (device, epi, cfg) -> resident blocks of the persistent kernel
}  // namespace

static int persist_capacity(const void* fn, int epi, int cfg) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const long key = ((long)dev * 8 + epi) * 16 + cfg;
  {
    std::lock_guard<std::mutex> lk(g_pcap_mu);
    auto it = g_pcap.find(key);
    if (it != g_pcap.end()) return it->second;
  }
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, CFG_NT[cfg], 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  const int cap = per_cu > 0 && cus > 0 ? (per_cu * cus) & ~7 : 0;   // a multiple of 8 (XCD labels)
  std::lock_guard<std::mutex> lk(g_pcap_mu);
  g_pcap[key] = cap;
  return cap;
}

template <typename T, typename TO, bool AK, bool BK_, int EPI>
static int launch_tiled(const T* A, int lda, const T* B, int ldb, int Mp, int Np, int K,
                        const GemmEpi& ep_in, int cfg, hipStream_t s) {
  // CFG 7 / 8 outside their epilogues (column partials, MSE, sigmoid / tanh):
  // CFG 6, the same 256x256 tile
  if (is_xst(cfg) && !xst_ok_rt(sizeof(T) == 2 ? MMAD_BF16 : MMAD_F32, EPI, ep_in)) cfg = xst_base(cfg);
  const int BM = CFG_BM[cfg], BN = CFG_BN[cfg];
  const int tiles_m = Mp / BM, tiles_n = Np / BN, ntiles = tiles_m * tiles_n;
  GemmEpi ep = ep_in;
  ep.tiles_n = tiles_n;
  const int S = ep.splitk > 1 ? ep.splitk : 1;
  ep.group_m = plan_group_m(ntiles, tiles_m, BM, BN);
  // persistent grid: forward-type bf16 epilogues without a fused BN or a
  // split, when the tiles exceed one resident round (knob 12: any nonzero
  // value; with fewer tiles the ordinary grid is the same launch)
  const int pk = mmad_persist_override();
  if (pk != 0 && S == 1 && !ep.bn_sync && persist_cfg(cfg)) {
    const void* pfn = persist_kernel<T, TO, AK, BK_, EPI>(cfg);
    const int cap = pfn ? persist_capacity(pfn, EPI, cfg) : 0;
    if (cap > 0 && ntiles > cap) {
      ep.persist_tiles = ntiles;
      dim3 pg(cap), pb(CFG_NT[cfg]);
      auto args_go = [&](auto kern) {
        if (ep.done_ev || ep.start_ev)
          hipExtLaunchKernelGGL(kern, pg, pb, 0u, s, ep.start_ev, ep.done_ev, 0u, A, lda, B, ldb, K, ep);
        else
          kern<<<pg, pb, 0, s>>>(A, lda, B, ldb, K, ep);
      };
      if constexpr (sizeof(T) == 2 && (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_MSE || EPI == GEMM_EPI_SCORE)) {
        switch (cfg) {
          case 1: args_go(mmad_gemm_kernel_p<T, TO, AK, BK_, 1, EPI>); break;
          case 2: args_go(mmad_gemm_kernel_p<T, TO, AK, BK_, 2, EPI>); break;
          case CFG_XST:
            if constexpr (xst_ok<T, EPI>()) {
              args_go(mmad_gemm_kernel_p<T, TO, AK, BK_, CFG_XST, EPI>);
              break;
            }
            [[fallthrough]];
          default: args_go(mmad_gemm_kernel_p<T, TO, AK, BK_, CFG_BIG, EPI>); break;
        }
        MMAD_LAUNCH_CHECK();
        return MMAD_OK;
      }
    }
  }
  if (cfg == CFG_B4) {
    if constexpr (xst_ok<T, EPI>()) return mmad_gemm_b4_launch(EPI, A, lda, B, ldb, Mp, Np, K, ep, s);
  }
  dim3 grd(ntiles * S), blk(CFG_NT[cfg]);
  const size_t dyn = 0;
  // the caller's completion event rides on the launch itself (no marker packet)
  auto go = [&](auto kern) {
    if (ep.done_ev || ep.start_ev)
      hipExtLaunchKernelGGL(kern, grd, blk, (std::uint32_t)dyn, s, ep.start_ev, ep.done_ev, 0u, A, lda, B, ldb,
                            K, ep);
    else
      kern<<<grd, blk, dyn, s>>>(A, lda, B, ldb, K, ep);
  };
  switch (cfg) {
    case 0: go(mmad_gemm_kernel<T, TO, AK, BK_, 0, EPI>); break;
    case 1: go(mmad_gemm_kernel<T, TO, AK, BK_, 1, EPI>); break;
    case 2: go(mmad_gemm_kernel<T, TO, AK, BK_, 2, EPI>); break;
    case 3: go(mmad_gemm_kernel<T, TO, AK, BK_, 3, EPI>); break;
    case 4: go(mmad_gemm_kernel<T, TO, AK, BK_, 4, EPI>); break;
    case 5: go(mmad_gemm_kernel<T, TO, AK, BK_, 5, EPI>); break;
    case CFG_XST1:
      if constexpr (xst_ok<T, EPI>()) go(mmad_gemm_kernel<T, TO, AK, BK_, CFG_XST1, EPI>);
      else go(mmad_gemm_kernel<T, TO, AK, BK_, 1, EPI>);
      break;
    default:
      if constexpr (big_ok<T, EPI>()) {
        if constexpr (xst_ok<T, EPI>()) {
          if (cfg == CFG_XST) {
            go(mmad_gemm_kernel<T, TO, AK, BK_, CFG_XST, EPI>);
            break;
          }
        }
        go(mmad_gemm_kernel<T, TO, AK, BK_, CFG_BIG, EPI>);
      } else {
        mmad_set_error("gemm: tile configuration %d does not support this dtype / epilogue", cfg);
        return MMAD_EUNSUPPORTED;
      }
      break;
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

// ---- co-residency of a whole grid (the fused-BN column barrier needs it) ----
template <typename T, typename TO, bool AK, bool BK_, int EPI>
static const void* kernel_ptr(int cfg) {
  switch (cfg) {
    case 0: return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 0, EPI>;
    case 1: return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 1, EPI>;
    case 2: return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 2, EPI>;
    case 3: return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 3, EPI>;
    case 4: return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 4, EPI>;
    case 5: return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 5, EPI>;
    case CFG_XST1:
      if constexpr (xst_ok<T, EPI>()) return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, CFG_XST1, EPI>;
      return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, 1, EPI>;
    default:
      if constexpr (xst_ok<T, EPI>())
        if (cfg == CFG_XST) return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, CFG_XST, EPI>;
      if constexpr (big_ok<T, EPI>()) return (const void*)mmad_gemm_kernel<T, TO, AK, BK_, CFG_BIG, EPI>;
      return nullptr;
  }
}
static const void* kernel_for(int dtype, int epi, int cfg) {
  if (dtype == MMAD_BF16) {
    if (epi == GEMM_EPI_FWD) return kernel_ptr<bf16, bf16, true, true, GEMM_EPI_FWD>(cfg);
    if (epi == GEMM_EPI_BWD_DATA) return kernel_ptr<bf16, bf16, true, false, GEMM_EPI_BWD_DATA>(cfg);
  } else {
    if (epi == GEMM_EPI_FWD) return kernel_ptr<float, float, true, true, GEMM_EPI_FWD>(cfg);
    if (epi == GEMM_EPI_BWD_DATA) return kernel_ptr<float, float, true, false, GEMM_EPI_BWD_DATA>(cfg);
  }
  return nullptr;
}
namespace {
std::mutex g_occ_mu;
std::map<long, int> g_occ;   // (device, dtype, epi, cfg) -> resident grid capacity
}  // namespace

// blocks of (dtype, epi, cfg) that can be resident on the current device at
// once: CUs x min(occupancy API, the LDS bound); 0 if unknown
static int grid_capacity(int dtype, int epi, int cfg) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const long key = (((long)dev * 4 + dtype) * 8 + epi) * 16 + cfg;
  {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) return it->second;
  }
  const void* fn = kernel_for(dtype, epi, cfg);
  int per_cu = 0, cus = 0;
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, CFG_NT[cfg], 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  hipFuncAttributes fa{};
  if (fn && hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.sharedSizeBytes > 0) {
    const int lds_bound = (int)(163840 / fa.sharedSizeBytes);
    per_cu = per_cu < lds_bound ? per_cu : lds_bound;
  }
  (void)hipGetLastError();
  const int cap = per_cu > 0 && cus > 0 ? per_cu * cus : 0;
  std::lock_guard<std::mutex> lk(g_occ_mu);
  g_occ[key] = cap;
  return cap;
}

static bool coresident(int dtype, int epi, int cfg, int Mp, int Np) {
  return mmad_gemm_ntiles(cfg, Mp, Np) <= grid_capacity(dtype, epi, cfg);
}

bool mmad_gemm_bn_fusable(int dtype, int epi, int Mp, int Np) {
  if (epi != GEMM_EPI_FWD && epi != GEMM_EPI_BWD_DATA) return false;
  if (Mp % 128 || Np % 128 || Np / 64 > MMAD_BN_EXIT) return false;
  for (int c = 0; c < NCFG; ++c)
    if (cfg_fits(c, Mp, Np, epi, dtype) && !is_big(c) && !is_xst(c) && coresident(dtype, epi, c, Mp, Np))
      return true;
  return false;
}

static int launch_cfg(int dtype, int epi, const void* A, int lda, const void* B, int ldb, int Mp,
                      int Np, int K, const GemmEpi& ep, int cfg, hipStream_t s) {
#define MMAD_LT(T, TO, AK, BK_, EPI)                                                      \
  return launch_tiled<T, TO, AK, BK_, EPI>((const T*)A, lda, (const T*)B, ldb, Mp, Np, K, ep, cfg, s)
#define MMAD_DISPATCH_T(T)                                                               \
  switch (epi) {                                                                         \
    case GEMM_EPI_FWD: MMAD_LT(T, T, true, true, GEMM_EPI_FWD);                          \
    case GEMM_EPI_MSE: MMAD_LT(T, T, true, true, GEMM_EPI_MSE);                          \
    case GEMM_EPI_SCORE: MMAD_LT(T, T, true, true, GEMM_EPI_SCORE);                      \
    case GEMM_EPI_BWD_DATA: MMAD_LT(T, T, true, false, GEMM_EPI_BWD_DATA);               \
    case GEMM_EPI_BWD_WEIGHT: MMAD_LT(T, float, false, false, GEMM_EPI_BWD_WEIGHT);      \
    default: mmad_set_error("gemm: bad epilogue %d", epi); return MMAD_EINVAL;          \
  }
  if (dtype == MMAD_BF16) {
    MMAD_DISPATCH_T(bf16)
  } else {
    MMAD_DISPATCH_T(float)
  }
#undef MMAD_LT
#undef MMAD_DISPATCH_T
}

// ---- autotune: time every fitting tile config once per problem shape -------
namespace {
struct TuneKey {
  int dtype, epi, Mp, Np, K, bnf;
  bool operator<(const TuneKey& o) const {
    const int a[6] = {dtype, epi, Mp, Np, K, bnf}, b[6] = {o.dtype, o.epi, o.Mp, o.Np, o.K, o.bnf};
    for (int i = 0; i < 6; ++i)
      if (a[i] != b[i]) return a[i] < b[i];
    return false;
  }
};
std::mutex g_tune_mu;
std::map<TuneKey, int> g_tune;
}  // namespace

static int tune_cfg(int dtype, int epi, const void* A, int lda, const void* B, int ldb, int Mp,
                    int Np, int K, const GemmEpi& ep, hipStream_t s, int* out_cfg) {
  // the trial launches must be side-effect free beyond the outputs the real
  // launch rewrites: no fused Adam while timing
  GemmEpi et = ep;
  et.done_ev = nullptr;   // the real launch below completes the caller's event
  et.start_ev = nullptr;
  et.ad_p = nullptr;
  et.sm_p = nullptr;
  et.bn_rmean = nullptr;   // fused BN: no running-statistics update while timing
  et.bn_rvar = nullptr;
  hipEvent_t e0, e1;
  MMAD_HIP_CHECK(hipEventCreate(&e0));
  MMAD_HIP_CHECK(hipEventCreate(&e1));
  int best = -1;
  float best_ms = 1e30f;
  int rc = MMAD_OK;
  for (int c = 0; c < NCFG && rc == MMAD_OK; ++c) {
    if (!cfg_fits(c, Mp, Np, epi, dtype)) continue;
    if ((is_big(c) || is_xst(c)) && (ep.bn_sync || ep.splitk > 1)) continue;   // no fused BN / split
    if (c == CFG_B4) continue;   // the 4-wave tile: forced only (measured slower)
    if (ep.bn_sync && !coresident(dtype, epi, c, Mp, Np)) continue;
    rc = launch_cfg(dtype, epi, A, lda, B, ldb, Mp, Np, K, et, c, s);   // warm
    if (rc != MMAD_OK) break;
    float ms = 0.f;
    hipError_t e = hipEventRecord(e0, s);
    for (int r = 0; r < 3 && rc == MMAD_OK && e == hipSuccess; ++r)
      rc = launch_cfg(dtype, epi, A, lda, B, ldb, Mp, Np, K, et, c, s);
    if (rc != MMAD_OK) break;
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e != hipSuccess) {
      mmad_set_error("gemm autotune: HIP error %d (%s)", (int)e, hipGetErrorString(e));
      rc = MMAD_EHIP;
      break;
    }
    if (ms < best_ms) { best_ms = ms; best = c; }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc != MMAD_OK) return rc;
  if (best < 0) {
    mmad_set_error("gemm autotune: no tile configuration fits (Mp=%d Np=%d epi=%d)", Mp, Np, epi);
    return MMAD_EUNSUPPORTED;
  }
  *out_cfg = best;
  return MMAD_OK;
}

// split factor for a shape (1, 2, 4, 8 or 16): a function of the shape and
// the epilogue only, so every tile configuration of a shape accumulates over
// K in the same order
int mmad_gemm_splitk(int Mp, int Np, int K, int dtype, int epi) {
  const int bk = dtype == MMAD_BF16 ? 64 : 32;            // K per stage
  const int t128 = (Mp / 128) * (Np / 128);              // 128x128 output tiles
  const int t64 = (Mp / 64) * (Np / 64);                 // 64x64 output tiles
  // workspace bounds (mmad_gemm_splitk_bytes): S * t128 <= MMAD_SK_SLAB_TILES slab tiles,
  // (1 + S) control words per tile of the smallest configuration
  auto ok = [&](int S) {
    return K % (S * bk) == 0 && K / S >= 4 * bk && S * t128 <= MMAD_SK_SLAB_TILES && t64 * (1 + S) < MMAD_SK_ERR_WORD;
  };
  auto valid = [](int S) { return S == 1 || S == 2 || S == 4 || S == 8 || S == 16; };
  const int env = mmad_splitk_override();
  if (valid(env)) return ok(env) ? env : 1;
  // the exact-fp32 parity path keeps one sequential K order per output (the
  // order closest to the reference's; a different fp32 order can flip the
  // LeakyReLU branch of a pre-activation at rounding level, e.g. 5.6e-7 in
  // tests/golden/mm192.npz); split-K is the bf16 performance path's -- except,
  // behind knob 32, the fp32 dW GEMMs of large batches: a gradient feeds no
  // branch, and contracting over >= 2048 rows the narrow layers' few 64x64
  // tiles run one f32-MFMA K loop each at 1/16 of the bf16 rate
  if (dtype != MMAD_BF16) {
    const int target = mmad_splitk_dw_f32_blocks();
    if (epi != GEMM_EPI_BWD_WEIGHT || target <= 0 || K < 2048) return 1;
    int best = 1;
    for (int S = 2; S <= 16; S *= 2)
      if (ok(S) && t64 * S <= target && K / S >= 16 * bk) best = S;
    return best;
  }
  if (epi == GEMM_EPI_BWD_WEIGHT) {
    const int envw = mmad_splitk_dw_override();
    if (valid(envw)) return ok(envw) ? envw : 1;
    // dW = dz^T a contracts over the batch: the narrow layers have few
    // output tiles and a long K loop.  Split until the launch has about
    // SK_DW_BLOCKS 64x64-tile blocks, keeping >= SK_DW_MIN_STAGES K stages
    // per slice (tools/splitk_sweep.py, profiles/r02*_splitk_dw*.log)
    const int target = mmad_splitk_dw_blocks(), min_st = mmad_splitk_dw_min_stages();
    int best = 1;
    for (int S = 2; S <= 16; S *= 2)
      if (ok(S) && t64 * S <= target && K / S >= min_st * bk) best = S;
    return best;
  }
  // forward / bwd-data at the bench shapes (B=1024, widths 2048..100): the
  // in-launch combine (slab round trip + ticket) costs more than the extra
  // CUs buy back, so no split; the override keeps the others reachable
  return 1;
}

// shape-independent bound: S * Mp * Np <= MMAD_SK_SLAB_TILES * 128 * 128 slab
// floats (832: split-K 4 of c2's largest forward / bwd-data GEMMs at 128x128);
// per launch (1 + S) control words per 64x64 tile < MMAD_SK_ERR_WORD
void mmad_gemm_splitk_bytes(int Mp, int Np, size_t* slab_bytes, size_t* ctl_bytes) {
  (void)Mp;
  (void)Np;
  if (slab_bytes) *slab_bytes = (size_t)MMAD_SK_SLAB_TILES * 128 * 128 * 4;
  if (ctl_bytes) *ctl_bytes = (size_t)(MMAD_SK_ERR_WORD + 1) * 4;
}

int mmad_gemm_read_status(unsigned* ctl, hipStream_t s, const char* who) {
  if (!ctl) return MMAD_OK;
  unsigned word = 0;
  MMAD_HIP_CHECK(hipMemcpyAsync(&word, ctl + MMAD_SK_ERR_WORD, sizeof(word), hipMemcpyDeviceToHost, s));
  MMAD_HIP_CHECK(hipStreamSynchronize(s));
  if (word == 0) return MMAD_OK;
  // a slice that gave up may still have raised its flag after the combine
  // cleared it: every launch of the failed one has finished now (stream
  // synchronised), so re-zero the whole control block for the next launch
  size_t slab = 0, ctl_bytes = 0;
  mmad_gemm_splitk_bytes(0, 0, &slab, &ctl_bytes);
  MMAD_HIP_CHECK(hipMemsetAsync(ctl, 0, ctl_bytes, s));
  MMAD_HIP_CHECK(hipStreamSynchronize(s));
  mmad_set_error("%s: a split-K GEMM combine timed out waiting for a slice; its output tiles were "
                 "not written (results invalid)", who);
  return MMAD_EHIP;
}

int mmad_gemm_plan(int Mp, int Np, int K, int epi, int dtype) {
  const int env = mmad_tile_override();
  if (env >= 0 && env < NCFG && cfg_fits(env, Mp, Np, epi, dtype)) return env;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  auto it = g_tune.find(TuneKey{dtype, epi, Mp, Np, K, 0});
  return it != g_tune.end() ? it->second : heuristic_cfg(Mp, Np, epi, dtype);
}

int mmad_gemm_dispatch(int dtype, int epi, const void* A, int lda, const void* B, int ldb, int Mp,
                       int Np, int K, const GemmEpi& ep_in, hipStream_t s, int* cfg_used) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && K % 128 == 0,
                 "gemm: padded dims must be multiples of 128 (Mp=%d Np=%d K=%d)", Mp, Np, K);
  MMAD_CHECK_ARG(Mp > 0 && Np > 0 && K > 0, "gemm: empty problem");
  MMAD_CHECK_ARG(dtype == MMAD_BF16 || dtype == MMAD_F32, "gemm: bad dtype %d", dtype);
  GemmEpi ep = ep_in;
  ep.dbg = mmad_dbg_override();
  const bool bnf = ep.bn_sync != nullptr;
  MMAD_CHECK_ARG(!bnf || epi == GEMM_EPI_FWD || epi == GEMM_EPI_BWD_DATA,
                 "gemm: fused BN only for the forward / bwd-data epilogues");
  MMAD_CHECK_ARG(!bnf || Np / 64 <= MMAD_BN_EXIT, "gemm: fused BN: Np=%d too wide", Np);
  // the fused BN barrier needs one block per output tile (no split) and the
  // whole grid resident
  ep.splitk = (ep.sk_slab && ep.sk_ctl && !bnf) ? mmad_gemm_splitk(Mp, Np, K, dtype, epi) : 1;
  auto allowed = [&](int c) {
    return c >= 0 && c < NCFG && cfg_fits(c, Mp, Np, epi, dtype) &&
           ((!is_big(c) && !is_xst(c)) || ep.splitk <= 1) &&
           (!bnf || (!is_big(c) && !is_xst(c) && coresident(dtype, epi, c, Mp, Np)));
  };
  const int env = mmad_tile_override();
  const int env_epi = ep.ad_p ? mmad_tile_adam_for(Mp, Np, K) : mmad_tile_epi_override(epi);
  int cfg;
  const int force = ep.tile_force - 1;
  if (allowed(force)) {
    cfg = force;
  } else if (allowed(env_epi)) {
    cfg = env_epi;
  } else if (allowed(env)) {
    cfg = env;   // forced tile (tuning / tests); a shape it does not fit falls through
  } else {
    const TuneKey key{dtype, epi, Mp, Np, K, bnf ? 1 : 0};
    int found = -1;
    {
      std::lock_guard<std::mutex> lk(g_tune_mu);
      auto it = g_tune.find(key);
      if (it != g_tune.end()) found = it->second;
    }
    if (found >= 0) {
      cfg = found;
    } else {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(s, &cs);
      if (mmad_autotune_enabled() && cs == hipStreamCaptureStatusNone) {
        int rc = tune_cfg(dtype, epi, A, lda, B, ldb, Mp, Np, K, ep, s, &cfg);
        if (rc != MMAD_OK) return rc;
      } else {
        cfg = heuristic_cfg(Mp, Np, epi, allowed);
        if (cfg < 0) {
          mmad_set_error("gemm: no co-resident tile configuration for the fused BN epilogue "
                         "(Mp=%d Np=%d)", Mp, Np);
          return MMAD_EUNSUPPORTED;
        }
      }
      std::lock_guard<std::mutex> lk(g_tune_mu);
      g_tune[key] = cfg;
    }
  }
  if (cfg_used) *cfg_used = cfg;
  return launch_cfg(dtype, epi, A, lda, B, ldb, Mp, Np, K, ep, cfg, s);
}
#endif  // MMAD_GEMM_B4_TU
