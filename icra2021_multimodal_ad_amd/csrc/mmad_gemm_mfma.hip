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
// Tile: BM x BN = (32*MI) x (32*NI), 256 threads = 4 waves in 2x2, each wave
// (16*MI) x (16*NI) built from 16x16 MFMA tiles (bf16: v_mfma_f32_16x16x32_bf16,
// f32: v_mfma_f32_16x16x4_f32, exact f32 for the parity path).  K stage =
// 128 bytes of K per row (BK = 64 bf16 / 32 f32), register-staged global
// loads (16 B/lane), double-buffered LDS, one barrier per stage.
//
// LDS images:
//  * K-major operand: [rows][128 B], 16-byte chunk j stored at j ^ ((row>>1)&7)
//    -> the two ds_read_b64 (bf16) / one ds_read_b128 (f32) fragment reads of
//    a wave are bank-conflict free.
//  * MN-major operand: [BK][rows*esize + pad], pad = 32 B (bf16) / 16 B (f32):
//    tr-reads of 8 consecutive k-rows hit disjoint banks.
// bf16 k-slot order inside one 32-deep MFMA step: lane group g (= lane>>4)
// owns k = {4g..4g+3} U {16+4g..16+4g+3}; A and B use the same permutation,
// so the contraction is exact.
#include "mmad_common.h"
#include "mmad_gemm.h"

namespace {

// LDS images are lane-linear (global_load_lds writes wave base + lane*16), so
// every bank-conflict swizzle is applied to the per-lane SOURCE address and
// undone on the read side.  KB = bytes of K per LDS row per stage.
constexpr int MMAD_KB = 128;

template <typename T, bool KMAJ, int ROWS>
struct Img {
  static constexpr int ES = sizeof(T);
  static constexpr int KB = MMAD_KB;
  static constexpr int BK = KB / ES;                  // K per stage
  static constexpr int RB = KMAJ ? KB : ROWS * ES;    // bytes per LDS row
  static constexpr int BYTES = ROWS * KB;             // image bytes (both layouts)
  static constexpr int CPROW = RB / 16;               // 16 B chunks per LDS row
  static constexpr int CHUNKS = BYTES / 16 / 256;     // global_load_lds per thread
};

// 16-byte-chunk XOR swizzle of LDS row `r` (an involution):
//  * K-major, 128 B rows: (r>>1)&7 -> both ds_read_b64 fragment reads
//    (bf16) / the ds_read_b128 read (f32) of a wave are conflict-free;
//  * MN-major bf16, 256 B rows: (r&7)<<1; 128 B rows: ((r>>1)&3)<<1 ->
//    ds_read_b64_tr_b16 of 8 consecutive k-rows hits all 64 banks once;
//  * MN-major f32: r&7 (spreads the 4-row-apart ds_read_b32 groups).
template <typename T, bool KMAJ, int RB>
__device__ __forceinline__ int swz(int r) {
  if constexpr (KMAJ) return (r >> 1) & 7;
  else if constexpr (sizeof(T) == 2) return RB >= 256 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1);
  else return r & 7;
}

// issue one stage of one operand: global -> LDS, 16 B per lane, no registers
template <typename T, bool KMAJ, int ROWS>
__device__ __forceinline__ void issue_stage(char* img, const T* __restrict__ G, int ld, int r0,
                                            int k0, int tid, int w) {
  using I = Img<T, KMAJ, ROWS>;
  constexpr int EPC = 16 / sizeof(T);
#pragma unroll
  for (int i = 0; i < I::CHUNKS; ++i) {
    const int p = 256 * i + tid;                       // LDS position (16 B units)
    const int row = p / I::CPROW;
    const int j = (p % I::CPROW) ^ swz<T, KMAJ, I::RB>(row);
    const T* src = KMAJ ? G + (size_t)(r0 + row) * ld + k0 + j * EPC
                        : G + (size_t)(k0 + row) * ld + r0 + j * EPC;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (MMAD_LDS void*)(img + (256 * i + 64 * w) * 16), 16, 0, 0);
  }
}

// ---- bf16 fragment reads (16x16x32 MFMA operand, permuted k slots) ------
// lane group g (= lane>>4) owns k = {4g..4g+3} U {16+4g..16+4g+3} of each
// 32-deep step, in both operands, so the contraction is exact.
template <bool KMAJ, int ROWS>
__device__ __forceinline__ bf16x8 frag_bf16(const char* img, int rbase, int kk, int lane) {
  using I = Img<bf16, KMAJ, ROWS>;
  const int g = lane >> 4;
  if constexpr (KMAJ) {
    const int m = rbase + (lane & 15);
    const int f = swz<bf16, true, I::RB>(m) << 1;     // in 8-byte units
    const int c1 = (kk * 8 + g) ^ f;
    const int c2 = (kk * 8 + 4 + g) ^ f;
    bf16x4 lo = *(const bf16x4*)(img + m * I::RB + c1 * 8);
    bf16x4 hi = *(const bf16x4*)(img + m * I::RB + c2 * 8);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  } else {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int k1 = kk * 32 + 4 * g + q, k2 = k1 + 16;
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
  using I = Img<float, KMAJ, ROWS>;
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

__device__ __forceinline__ bf16x8 affine8(bf16x8 v, floatx4 s0, floatx4 s1, floatx4 t0, floatx4 t1) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = (bf16)((float)v[e] * s0[e] + t0[e]);
    v[4 + e] = (bf16)((float)v[4 + e] * s1[e] + t1[e]);
  }
  return v;
}

__device__ __forceinline__ bf16x8 affine8c(bf16x8 v, float s, float t) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] * s + t);
  return v;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void block_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int MI, int NI> struct Ring { static constexpr int NS = (MI == 2 && NI == 4) ? 5 : 4; };

}  // namespace

// -------------------------------------------------------------------------
// TR: BatchNorm normalise-on-load -- A operand (K-major, indexed by k) for the
// forward GEMMs, B operand (MN-major, indexed by n) for the dW GEMM; applied
// to the MFMA fragments right after the LDS read.
template <typename T, typename TO, bool AK, bool BK_, int MI, int NI, int EPI, bool TR>
__global__ __launch_bounds__(256, 1) void mmad_gemm_kernel(const T* __restrict__ A, int lda,
                                                            const T* __restrict__ B, int ldb, int K,
                                                            GemmEpi ep) {
  constexpr int BM = 32 * MI, BN = 32 * NI;
  using IA = Img<T, AK, BM>;
  using IB = Img<T, BK_, BN>;
  constexpr bool ATR = TR && AK;
  constexpr bool BTR = TR && !BK_;
  constexpr int NS = Ring<MI, NI>::NS;
  constexpr int SLOT = IA::BYTES + IB::BYTES + (ATR ? 4096 : 0);
  constexpr int NL = IA::CHUNKS + IB::CHUNKS + (ATR ? 1 : 0);   // vm ops per thread per stage
  constexpr int OSTRIDE = BN * (int)sizeof(TO) + 16;
  constexpr int OBYTES = BM * OSTRIDE + (EPI == GEMM_EPI_BWD_DATA ? 2 * 256 * 4 : 0);
  constexpr int LDS_BYTES = (NS * SLOT > OBYTES) ? NS * SLOT : OBYTES;
  static_assert((NS - 2) * NL <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware tile order (1-D grid).  Under round-robin dispatch, blocks with
  // equal bid % 8 share an XCD (speed only, never correctness); each such set
  // gets a contiguous range of logical tiles, and logical tiles are grouped
  // group_m M-tiles at a time, so every XCD works on a compact rectangle whose
  // A/B panels stay in its 4 MB L2.
  const int nblk = gridDim.x, bid = blockIdx.x;
  int tm, tn;
  {
    const int q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_m = nblk / ep.tiles_n;
    const int per_group = ep.group_m * ep.tiles_n;
    const int first_m = (wg / per_group) * ep.group_m;
    const int gsz = min(tiles_m - first_m, ep.group_m);
    tm = first_m + (wg % per_group) % gsz;
    tn = (wg % per_group) / gsz;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nt = K / IA::BK;

  floatx4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // B-side BatchNorm affine: one (scale, shift) per lane per n-tile, loaded
  // (and waited for) before any LDS-DMA is in flight
  float sbn[NI], tbn[NI];
  if constexpr (BTR) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wn * 16 * NI + j * 16 + (lane & 15);
      sbn[j] = ep.b_scale[n];
      tbn[j] = ep.b_shift[n];
      asm volatile("" ::"v"(sbn[j]), "v"(tbn[j]));
    }
  }

  auto issue = [&](int s) {
    char* base = smem + (s % NS) * SLOT;
    const int k0 = s * IA::BK;
    issue_stage<T, AK, BM>(base, A, lda, m0, k0, tid, w);
    issue_stage<T, BK_, BN>(base + IA::BYTES, B, ldb, n0, k0, tid, w);
    if constexpr (ATR) {
      // per-wave copy of [scale(k0..k0+BK) | shift(k0..k0+BK)] for the A-side affine
      constexpr int Q = IA::BK / 4;
      const float* src = lane < Q ? ep.a_scale + k0 + 4 * lane
                                  : (lane < 2 * Q ? ep.a_shift + k0 + 4 * (lane - Q) : ep.a_scale + k0);
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (MMAD_LDS void*)(base + IA::BYTES + IB::BYTES + w * 1024), 16,
                                       0, 0);
    }
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nt) issue(s);

  for (int t = 0; t < nt; ++t) {
    if (t + NS - 2 < nt) wait_vmcnt<(NS - 2) * NL>();
    else wait_vmcnt<0>();
    block_barrier();                       // stage t landed for every wave; slot t-1 free
    if (t + NS - 1 < nt) issue(t + NS - 1);
    const char* sa = smem + (t % NS) * SLOT;
    const char* sb = sa + IA::BYTES;
    const char* sc = sb + IB::BYTES + w * 1024;   // this wave's affine copy (ATR)
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < IA::BK / 32; ++kk) {
        bf16x8 fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = frag_bf16<AK, BM>(sa, wm * 16 * MI + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = frag_bf16<BK_, BN>(sb, wn * 16 * NI + j * 16, kk, lane);
        if constexpr (ATR) {
          const int g4 = (lane >> 4) * 4;
          const floatx4 s0 = *(const floatx4*)(sc + (kk * 32 + g4) * 4);
          const floatx4 s1 = *(const floatx4*)(sc + (kk * 32 + 16 + g4) * 4);
          const floatx4 t0 = *(const floatx4*)(sc + (IA::BK + kk * 32 + g4) * 4);
          const floatx4 t1 = *(const floatx4*)(sc + (IA::BK + kk * 32 + 16 + g4) * 4);
#pragma unroll
          for (int i = 0; i < MI; ++i) fa[i] = affine8(fa[i], s0, s1, t0, t1);
        }
        if constexpr (BTR) {
#pragma unroll
          for (int j = 0; j < NI; ++j) fb[j] = affine8c(fb[j], sbn[j], tbn[j]);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kc = 0; kc < IA::BK / 16; ++kc) {
        floatx4 fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = frag_f32<AK, BM>(sa, wm * 16 * MI + i * 16, kc, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = frag_f32<BK_, BN>(sb, wn * 16 * NI + j * 16, kc, lane);
        if constexpr (ATR) {
          const int g4 = (lane >> 4) * 4;
          const floatx4 s0 = *(const floatx4*)(sc + (kc * 16 + g4) * 4);
          const floatx4 t0 = *(const floatx4*)(sc + (IA::BK + kc * 16 + g4) * 4);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) fa[i][e] = fa[i][e] * s0[e] + t0[e];
        }
        if constexpr (BTR) {
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) fb[j][e] = fb[j][e] * sbn[j] + tbn[j];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
      }
    }
  }

  // ===================== epilogue, register phase ==========================
  const int g = lane >> 4, c = lane & 15;
  const int rw = m0 + wm * 16 * MI;  // first row of this wave
  const int cw = n0 + wn * 16 * NI;  // first col of this wave
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int col = cw + j * 16 + c;
    const bool cvalid = col < ep.N;
    float bias = 0.f, sc = 1.f, sh = 0.f;
    if (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_MSE || EPI == GEMM_EPI_SCORE) {
      if (ep.bias) bias = ep.bias[col];
      if (ep.bn_scale) { sc = ep.bn_scale[col]; sh = ep.bn_shift[col]; }
    }
    float s1[MI / 2], s2[MI / 2];
#pragma unroll
    for (int p = 0; p < MI / 2; ++p) { s1[p] = 0.f; s2[p] = 0.f; }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rw + i * 16 + 4 * g + r;
        const bool valid = cvalid && row < ep.M;
        float v = acc[i][j][r];
        if (EPI == GEMM_EPI_FWD || EPI == GEMM_EPI_SCORE) {
          v = apply_act(v + bias, ep.act, ep.slope) * sc + sh;
          v = valid ? v : 0.f;
          s1[i >> 1] += v;
        } else if (EPI == GEMM_EPI_MSE) {
          float d = 0.f;
          if (valid) d = v + bias - ep.target[(size_t)(row % ep.tmod) * ep.ldt + col];
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
      for (int p = 0; p < MI / 2; ++p) {
        float a1 = s1[p];
        a1 += __shfl_xor(a1, 16);
        a1 += __shfl_xor(a1, 32);
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
          q += __shfl_xor(q, 16);
          q += __shfl_xor(q, 32);
          if (g == 0) { part[col] = mean; part[ep.ldpart + col] = q; }
        } else if (EPI == GEMM_EPI_MSE) {
          float a2 = s2[p];
          a2 += __shfl_xor(a2, 16);
          a2 += __shfl_xor(a2, 32);
          if (g == 0) { part[col] = a1; part[ep.ldpart + col] = a2; }
        } else if (EPI == GEMM_EPI_BWD_DATA) {
          if (g == 0) part[col] = a1;
        }
      }
    }
  }

  // ===================== epilogue, LDS-staged coalesced store ===============
  __syncthreads();  // main-loop LDS no longer read
  if constexpr (EPI == GEMM_EPI_MSE) {
    if (ep.lossp) {
      // one loss partial per block: sum of d^2 = sum (dz/gscale)^2 over the tile
      float lt = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) lt += acc[i][j][r] * acc[i][j][r];
      lt = wave_sum(lt) / (ep.gscale * ep.gscale);
      float* red = (float*)smem;
      if (lane == 0) red[w] = lt;
      __syncthreads();
      if (tid == 0) ep.lossp[bid] = red[0] + red[1] + red[2] + red[3];
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 16 * MI + i * 16 + 4 * g + r;
        const int cl = wn * 16 * NI + j * 16 + c;
        *(TO*)(smem + rl * OSTRIDE + cl * (int)sizeof(TO)) = from_f32<TO>(acc[i][j][r]);
      }
  __syncthreads();
  constexpr int CPR = BN * (int)sizeof(TO) / 16;  // 16-byte chunks per output row
  constexpr int OEPC = 16 / (int)sizeof(TO);
  constexpr int ITERS = BM * CPR / 256;
  TO* out = (TO*)ep.out;
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int idx = it * 256 + tid;
    const int rl = idx / CPR, ch = idx % CPR;
    const uint4v v = *(const uint4v*)(smem + rl * OSTRIDE + ch * 16);
    const int row = m0 + rl;
    const int col = n0 + ch * OEPC;
    *(uint4v*)(out + (size_t)row * ep.ldo + col) = v;
    if constexpr (EPI == GEMM_EPI_BWD_WEIGHT) {
      if (ep.ad_p) {
        // torch.optim.Adam on this dW chunk (4 fp32), same formula as adam_k
        const size_t off = (size_t)row * ep.ldo + col;
        floatx4 gg = __builtin_bit_cast(floatx4, v);
        floatx4 pp = *(floatx4*)(ep.ad_p + off), mm = *(floatx4*)(ep.ad_m + off);
        floatx4 vv = *(floatx4*)(ep.ad_v + off);
        adam4(pp, mm, vv, gg, ep.ad_b1, ep.ad_b2, ep.ad_eps, ep.ad_step, ep.ad_bc2);
        *(floatx4*)(ep.ad_p + off) = pp;
        *(floatx4*)(ep.ad_m + off) = mm;
        *(floatx4*)(ep.ad_v + off) = vv;
        if (ep.ad_shadow) {
          bf16x4 sh;
#pragma unroll
          for (int e = 0; e < 4; ++e) sh[e] = (bf16)pp[e];
          *(bf16x4*)((bf16*)ep.ad_shadow + off) = sh;
        }
      }
    }
    if (EPI == GEMM_EPI_SCORE) {
      const TO* ref = (const TO*)ep.ref + (size_t)row * ep.ldref + col;
      const uint4v rv = *(const uint4v*)ref;
      const TO* pv = (const TO*)&v;
      const TO* pr = (const TO*)&rv;
      float sq = 0.f;
      float dd[OEPC];
#pragma unroll
      for (int e = 0; e < OEPC; ++e) {
        dd[e] = to_f32<TO>(pv[e]) - to_f32<TO>(pr[e]);
        sq += dd[e] * dd[e];
      }
      if (ep.diff && row < ep.M) {
        float* dp = ep.diff + (size_t)row * ep.lddiff + col;
#pragma unroll
        for (int e = 0; e < OEPC; ++e)
          if (col + e < ep.N) dp[e] = dd[e];
      }
#pragma unroll
      for (int o = 1; o < CPR; o <<= 1) sq += __shfl_xor(sq, o);
      if (ch == 0) ep.rowsq[(size_t)tn * ep.ldrow + row] = sq;
    }
  }
  if constexpr (EPI == GEMM_EPI_BWD_WEIGHT) {
    if (ep.ad_p && ep.sm_p) {
      // the layer's bias/gamma/beta Adam, 4 elements per thread, spread over the grid
      const int nb = nblk;
      const int b = bid;
      for (int q = b * 256 + tid; q * 4 < ep.sm_n; q += nb * 256) {
        const int i4 = q * 4;
        floatx4 gg;
        if (ep.sm_bsrc && i4 < ep.sm_bNp) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float t = 0.f;
            if (i4 + e < ep.sm_bN)
              for (int i = 0; i < ep.sm_bparts; ++i) t += ep.sm_bsrc[(size_t)i * ep.sm_bstride + i4 + e];
            gg[e] = t;
          }
          *(floatx4*)(ep.sm_g + i4) = gg;
        } else {
          gg = *(const floatx4*)(ep.sm_g + i4);
        }
        floatx4 pp = *(floatx4*)(ep.sm_p + i4), mm = *(floatx4*)(ep.sm_m + i4);
        floatx4 vv = *(floatx4*)(ep.sm_v + i4);
        adam4(pp, mm, vv, gg, ep.ad_b1, ep.ad_b2, ep.ad_eps, ep.ad_step, ep.ad_bc2);
        *(floatx4*)(ep.sm_p + i4) = pp;
        *(floatx4*)(ep.sm_m + i4) = mm;
        *(floatx4*)(ep.sm_v + i4) = vv;
      }
    }
  }
  if constexpr (EPI == GEMM_EPI_BWD_DATA) {
    if (ep.bn_part) {
      // sum over rows of dy and dy*xhat, xhat = (a - mean)*rstd, per 64-row chunk
      constexpr int NG = 256 / BN;   // thread groups per column
      constexpr int RPG = BM / NG;   // rows per group
      constexpr int GPP = RPG >= 64 ? 1 : 64 / RPG;
      const int cc = tid % BN, grp = tid / BN;
      const int col = n0 + cc;
      const float mu = ep.bn_mean[col], rs = ep.bn_rstd[col];
      const TO* an = (const TO*)ep.bn_a;
      float s1 = 0.f, s2 = 0.f;
      for (int r = 0; r < RPG; ++r) {
        const int rl = grp * RPG + r;
        const float dy = to_f32<TO>(*(const TO*)(smem + rl * OSTRIDE + cc * (int)sizeof(TO)));
        const float av = to_f32<TO>(an[(size_t)(m0 + rl) * ep.ldo + col]);
        s1 += dy;
        s2 += dy * (av - mu) * rs;
      }
      float* scr = (float*)(smem + BM * OSTRIDE);
      if constexpr (GPP == 1) {
        float* pp = ep.bn_part + (size_t)((m0 + grp * RPG) / 64) * 2 * ep.ldo;
        pp[col] = s1;
        pp[ep.ldo + col] = s2;
      } else {
        scr[grp * BN + cc] = s1;
        scr[256 + grp * BN + cc] = s2;
        __syncthreads();
        if (grp % GPP == 0) {
          for (int q = 1; q < GPP; ++q) {
            s1 += scr[(grp + q) * BN + cc];
            s2 += scr[256 + (grp + q) * BN + cc];
          }
          float* pp = ep.bn_part + (size_t)((m0 + grp * RPG) / 64) * 2 * ep.ldo;
          pp[col] = s1;
          pp[ep.ldo + col] = s2;
        }
      }
    }
  }
}

// -------------------------------------------------------------------------
// host-side launch
// -------------------------------------------------------------------------
template <typename T, typename TO, bool AK, bool BK_, int EPI, bool TR>
static int launch_tiled(const T* A, int lda, const T* B, int ldb, int Mp, int Np, int K,
                        const GemmEpi& ep_in, int tile, hipStream_t s) {
  dim3 blk(256);
  const int BM = tile == 0 ? 128 : 64, BN = tile == 2 ? 64 : 128;
  const int tiles_m = Mp / BM, tiles_n = Np / BN, nblk = tiles_m * tiles_n;
  GemmEpi ep = ep_in;
  ep.tiles_n = tiles_n;
  // group height balancing the per-XCD A-panel (gm*BM rows) and B-panel
  // ((nblk/8/gm)*BN cols) footprints
  const double per_xcd = nblk / 8.0;
  int gm = (int)(sqrt(per_xcd * BN / BM) + 0.5);
  const int env_gm = mmad_group_override();
  if (env_gm > 0) gm = env_gm;
  ep.group_m = gm < 1 ? 1 : (gm > tiles_m ? tiles_m : gm);
  dim3 grd(nblk);
  switch (tile) {
    case 0:  // 128 x 128
      mmad_gemm_kernel<T, TO, AK, BK_, 4, 4, EPI, TR><<<grd, blk, 0, s>>>(A, lda, B, ldb, K, ep);
      break;
    case 1:  // 64 x 128
      mmad_gemm_kernel<T, TO, AK, BK_, 2, 4, EPI, TR><<<grd, blk, 0, s>>>(A, lda, B, ldb, K, ep);
      break;
    default:  // 64 x 64
      mmad_gemm_kernel<T, TO, AK, BK_, 2, 2, EPI, TR><<<grd, blk, 0, s>>>(A, lda, B, ldb, K, ep);
      break;
  }
  MMAD_LAUNCH_CHECK();
  return MMAD_OK;
}

int mmad_gemm_grid_blocks(int Mp, int Np, int epi) {
  switch (mmad_pick_tile(Mp, Np, epi)) {
    case 0: return (Mp / 128) * (Np / 128);
    case 1: return (Mp / 64) * (Np / 128);
    default: return (Mp / 64) * (Np / 64);
  }
}

int mmad_pick_tile(int Mp, int Np, int epi) {
  const int env = mmad_tile_override();
  if (env >= 0) return env;
  // the score epilogue reduces rows over the tile width; keep it 128 wide
  if ((Mp / 128) * (Np / 128) >= 240) return 0;
  if (epi == GEMM_EPI_SCORE || (Mp / 64) * (Np / 128) >= 200) return 1;
  return 2;
}

int mmad_gemm_dispatch(int dtype, int epi, const void* A, int lda, const void* B, int ldb, int Mp,
                       int Np, int K, const GemmEpi& ep, hipStream_t s) {
  MMAD_CHECK_ARG(Mp % 128 == 0 && Np % 128 == 0 && K % 128 == 0,
                 "gemm: padded dims must be multiples of 128 (Mp=%d Np=%d K=%d)", Mp, Np, K);
  MMAD_CHECK_ARG(Mp > 0 && Np > 0 && K > 0, "gemm: empty problem");
  const int tile = mmad_pick_tile(Mp, Np, epi);
  if (epi == GEMM_EPI_SCORE) MMAD_CHECK_ARG(tile != 2, "score epilogue needs a 128-wide tile");
  const bool atr = ep.a_scale != nullptr, btr = ep.b_scale != nullptr;
#define MMAD_LT(T, TO, AK, BK_, EPI, TR)                                                  \
  return launch_tiled<T, TO, AK, BK_, EPI, TR>((const T*)A, lda, (const T*)B, ldb, Mp, Np, K, ep, \
                                               tile, s)
#define MMAD_DISPATCH_T(T)                                                               \
  switch (epi) {                                                                         \
    case GEMM_EPI_FWD:                                                                   \
      if (atr) MMAD_LT(T, T, true, true, GEMM_EPI_FWD, true);                            \
      MMAD_LT(T, T, true, true, GEMM_EPI_FWD, false);                                    \
    case GEMM_EPI_MSE:                                                                   \
      if (atr) MMAD_LT(T, T, true, true, GEMM_EPI_MSE, true);                            \
      MMAD_LT(T, T, true, true, GEMM_EPI_MSE, false);                                    \
    case GEMM_EPI_SCORE:                                                                 \
      MMAD_LT(T, T, true, true, GEMM_EPI_SCORE, false);                                  \
    case GEMM_EPI_BWD_DATA:                                                              \
      MMAD_LT(T, T, true, false, GEMM_EPI_BWD_DATA, false);                              \
    case GEMM_EPI_BWD_WEIGHT:                                                            \
      if (btr) MMAD_LT(T, float, false, false, GEMM_EPI_BWD_WEIGHT, true);               \
      MMAD_LT(T, float, false, false, GEMM_EPI_BWD_WEIGHT, false);                       \
    default: mmad_set_error("gemm: bad epilogue %d", epi); return MMAD_EINVAL;          \
  }
  if (dtype == MMAD_BF16) {
    MMAD_DISPATCH_T(bf16)
  } else if (dtype == MMAD_F32) {
    MMAD_DISPATCH_T(float)
  }
#undef MMAD_LT
#undef MMAD_DISPATCH_T
  mmad_set_error("gemm: bad dtype %d", dtype);
  return MMAD_EINVAL;
}
