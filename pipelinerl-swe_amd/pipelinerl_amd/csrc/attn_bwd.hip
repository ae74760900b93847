// Flash-attention backward for the trainer's packed (varlen) causal attention, gfx950, bf16,
// head dim 128.  Replaces the backward of torch's varlen flash attention (AOTriton on ROCm,
// ~150 TF at 8 x 2048 on MI355X) behind finetune/attention.py.
//
// Given Q, K, V, dO [T, H, 128] (token-major, packed sequences [cu[i], cu[i+1])), the forward's
// log-sum-exp L (natural log of sum_j exp(s * S_ij)) and delta_i = sum_d dO_id O_id:
//   P  = exp(s S - L),  dS = P (dP - delta),  S = Q K^T, dP = dO V^T
//   dV = P^T dO,  dK = s dS^T Q,  dQ = s dS K
// Two kernels, no atomics, no score matrix in HBM:
//   attn_bwd_dkdv  one workgroup = 128 keys of one (sequence, head); each wave owns 32 keys and
//                  keeps dK^T, dV^T (128 x 32 fp32 each) in accumulators while the workgroup
//                  sweeps the causal query tiles (32 rows, one swizzled LDS image per tile, read
//                  by rows and with ds_read_b64_tr_b16; the next tile is register-staged
//                  behind the current tile's MFMAs)
//   attn_bwd_dq    one workgroup = 128 queries; each wave owns 32 queries (dQ^T in accumulators)
//                  and sweeps the causal key tiles
// MFMA: v_mfma_f32_32x32x16_bf16.  Lane layouts (probed, tools/mfma_layout_probe.hip [round 1-3 tool, in git history]):
//   A[m][k]: lane l holds A[l%32][8(l/32)+i];  B[k][n]: lane l holds B[8(l/32)+i][l%32];
//   C[m][n]: lane l, reg r holds C[8(r/4)+4(l/32)+(r%4)][l%32].
// S and dP are computed with the KEY (dK/dV kernel) or the QUERY (dQ kernel) on the lane, so
// their accumulators are the B operands of the next product as they stand: the reduction index
// of that product is taken in the permuted order sigma(8h+i) = 8(i/4) + 4h + (i%4) (+16 for the
// second half), and the A operand is read transposed (ds_read_b64_tr_b16) in the same order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "prl_hip.h"

namespace prl_attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int D = 128;
constexpr int TILE = 32;   // rows per MFMA tile
constexpr int STAGE = 64;  // rows staged per barrier pair (two tiles)

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ bf16x8 ld8(const __bf16* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p)); }
__device__ __forceinline__ bf16x8 zero8() { return __builtin_bit_cast(bf16x8, u32x4{0, 0, 0, 0}); }
__device__ __forceinline__ void st4(__bf16* p, float a, float b, float c, float d) {
  bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  *reinterpret_cast<u32x2*>(p) = __builtin_bit_cast(u32x2, v);
}

// LDS tile image: 32 rows x 128 bf16 (256-B rows), 16-B chunks XOR-swizzled so that both the
// row reads (ds_read_b128, MFMA operands with the row on the lane) and the transposed reads
// (ds_read_b64_tr_b16, operands that need the tile's columns on the lane) are conflict-free
// (cdna_hip_programming.md T10, image (b)).  Byte offset of chunk ch (0..15) of row r:
__device__ __forceinline__ int toff(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 tr_read(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + off));
}
__device__ __forceinline__ bf16x8 row_read(const char* base, int r, int ch) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(base + toff(r, ch)));
}
// A operand [m = column d][k = row, sigma order] of a 32x32x16 MFMA from a tile image: d chunk dc
// (columns 32dc .. 32dc+31), k-step ks (rows 16ks ..): elements 0..3 = rows 16ks+4h+0..3,
// elements 4..7 = rows 16ks+8+4h+0..3, column 32dc + (lane & 31).  Lane 4q+p of each 16-lane
// group addresses row R+q, columns d0+4p..+3 (d0 = the group's first column).
__device__ __forceinline__ bf16x8 tr_operand(const char* base, int lane, int dc, int ks) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int h = g >> 1;
  const int ch = 4 * dc + 2 * (g & 1) + (p >> 1);
  const int r0 = 16 * ks + 4 * h + q;
  const bf16x4 a = tr_read(base, toff(r0, ch) + 8 * (p & 1));
  const bf16x4 b = tr_read(base, toff(r0 + 8, ch) + 8 * (p & 1));
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// register staging of a ROWS-row stage of X[T, H, D] (rows r0.., head h): ROWS / 16 chunks per thread
template <int ROWS>
struct StageT {
  u32x4 x[ROWS * 16 / 256];
};
typedef StageT<STAGE> Stage;
#ifndef PRL_ATTN_BSTAGE
#define PRL_ATTN_BSTAGE 64  // rows per backward stage; 32 halves the staging registers (A/B)
#endif
constexpr int BSTAGE = PRL_ATTN_BSTAGE;
template <int ROWS = STAGE>
__device__ __forceinline__ StageT<ROWS> stage_load(const __bf16* __restrict__ X, int64_t rs, int h, int r0, int r1,
                                                    int tid) {
  StageT<ROWS> st;
#pragma unroll
  for (int j = 0; j < ROWS * 16 / 256; ++j) {
    const int c = tid + 256 * j;
    const int t = r0 + (c >> 4);
    st.x[j] = t < r1 ? *reinterpret_cast<const u32x4*>(X + (int64_t)t * rs + h * D + (c & 15) * 8) : u32x4{0, 0, 0, 0};
  }
  return st;
}
template <int ROWS>
__device__ __forceinline__ void stage_store(const StageT<ROWS>& st, char* base, int tid) {
#pragma unroll
  for (int j = 0; j < ROWS * 16 / 256; ++j) {
    const int c = tid + 256 * j;
    *reinterpret_cast<u32x4*>(base + toff(c >> 4, c & 15)) = st.x[j];
  }
}

#ifndef PRL_ATTN_BUF_STAGE
#define PRL_ATTN_BUF_STAGE 1  // 0: the flat per-row-tested stage loads (A/B, tools/build_variants.py attn_flat_stage)
#endif
// The same stage through buffer loads: a wave-uniform descriptor over rows [r0, r1) of the tensor
// (base at row r0, r1 - r0 rows of rs elements), so rows past the sequence end fall outside it and
// read 0 with no per-row test, and the per-thread offsets are computed once per head (vbase = the
// thread's first chunk: row tid / 16, head h, 16-B chunk tid % 16; chunk j is 16 j rows further).
// The flat form's 64-bit address arithmetic and per-row branches took 15-19 % of the backward's
// cycles (tools/attn_clock.py [round 1-3 tool, in git history]); this form issues 8 loads and ~15 scalar instructions per stage and
// runs the backward 3-7 % and the forward 3-6 % faster (profiles/r03_attn_buf_stage_ab.jsonl).
// Spreading the 8 loads over the paired tiles' MFMAs instead of one burst after the barrier was
// measured no faster (same file): the issue cycles moved into the tiles.
// The descriptor spans at most the ROWS rows one stage reads (never the rest of the sequence): its
// byte count stays far below 2^31 at any sequence length (a whole-sequence span overflowed int32
// past ~2^31 / (rs * 2) rows, turning the bounds check off for the unmasked stages).
template <int ROWS = STAGE>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const __bf16* X, int64_t rs, int r0, int r1) {
  const int n = r1 > r0 ? (r1 - r0 < ROWS ? r1 - r0 : ROWS) : 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(X + (int64_t)r0 * rs), 0, (int)((int64_t)n * rs * 2),
                                           0x00020000);
}
__device__ __forceinline__ int stage_vbase(int64_t rs, int h, int tid) {
  return (tid >> 4) * (int)(rs * 2) + h * D * 2 + (tid & 15) * 16;
}
template <int ROWS = STAGE>
__device__ __forceinline__ StageT<ROWS> stage_load_rows(const __bf16* __restrict__ X, int64_t rs, int h, int r0,
                                                        int r1, int tid, int vbase) {
#if PRL_ATTN_BUF_STAGE
  (void)h;
  (void)tid;
  const __amdgpu_buffer_rsrc_t rsrc = rows_rsrc<ROWS>(X, rs, r0, r1);
  StageT<ROWS> st;
#pragma unroll
  for (int j = 0; j < ROWS * 16 / 256; ++j)
    st.x[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vbase + j * 16 * (int)(rs * 2), 0, 0));
  return st;
#else
  (void)vbase;
  return stage_load<ROWS>(X, rs, h, r0, r1, tid);
#endif
}

#ifndef PRL_ATTN_EXP_NOLOAD
#define PRL_ATTN_EXP_NOLOAD 0  // timing experiment only (wrong results): backward stages after the first not loaded
#endif
#ifndef PRL_ATTN_EXP_NOEXP
#define PRL_ATTN_EXP_NOEXP 0  // timing experiment only (wrong results): backward exp2 replaced by a multiply
#endif
__device__ __forceinline__ float bexp2(float x) { return PRL_ATTN_EXP_NOEXP ? x * 0.5f : __builtin_amdgcn_exp2f(x); }
#ifndef PRL_ATTN_INTERLEAVE
#define PRL_ATTN_INTERLEAVE 1  // 0: one tile at a time everywhere (A/B builds, tools/build_variants.py)
#endif
// Backward scheduling.  One wave per SIMD (dK^T and dV^T alone hold 128 accumulator registers), so
// nothing hides a tile's softmax VALU work (~7 vector instructions per MFMA) unless the wave's own
// MFMAs of ANOTHER tile sit beside it.  Away from the diagonal, tiles are processed in pairs a, b:
//   [S_a dP_a]   [S_b dP_b  |  softmax a]   [dV dK += a  |  softmax b]   [dV dK += b]
// the "|" regions are interleaved by sched_group_barrier groups (1 MFMA, its LDS reads, then
// vector work), so the matrix pipe stays busy through both softmaxes.  The accumulation order of
// every accumulator is unchanged: the results are bit-identical to one tile at a time.
#define SGB(mask, n) __builtin_amdgcn_sched_group_barrier(mask, n, 0)
constexpr int kSgMfma = 0x008, kSgValu = 0x002, kSgDsRead = 0x100;
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
#ifndef PRL_ATTN_LEAD
#define PRL_ATTN_LEAD 8  // tools/build_variants.py sweep: 0 / 1 / 3 / 6 / 8 / 12 / 16 -> 8 (6-12 within 1 %)
#endif
// NMFMA groups of (1 MFMA, NVALU vector instructions); the LDS reads run PRL_ATTN_LEAD MFMAs ahead
// of the MFMA that consumes them (NREAD reads per MFMA), so their latency is not in front of it
template <int NMFMA, int NREAD, int NVALU>
__device__ __forceinline__ void interleave() {
  constexpr int kLead = PRL_ATTN_LEAD < NMFMA ? PRL_ATTN_LEAD : NMFMA;
  SGB(kSgDsRead, NREAD * kLead);
#pragma unroll
  for (int i = 0; i < NMFMA; ++i) {
    SGB(kSgMfma, 1);
    if (i + kLead < NMFMA) SGB(kSgDsRead, NREAD);
    if (NVALU) SGB(kSgValu, NVALU);
  }
}
// a pipeline segment (dkdv_pipeline): the half softmax's 4 L / delta reads and the first PRL_ATTN_LEAD
// operand reads, then NMFMA groups of (1 MFMA, its NREAD operand reads, NVALU vector instructions)
template <int NMFMA, int NREAD, int NVALU>
__device__ __forceinline__ void interleave_seg() {
  constexpr int kLead = PRL_ATTN_LEAD < NMFMA ? PRL_ATTN_LEAD : NMFMA;
  SGB(kSgDsRead, 4 + NREAD * kLead);
#pragma unroll
  for (int i = 0; i < NMFMA; ++i) {
    SGB(kSgMfma, 1);
    if (i + kLead < NMFMA) SGB(kSgDsRead, NREAD);
    SGB(kSgValu, NVALU);
  }
}
#ifndef PRL_ATTN_CLOCK_PROBE
#define PRL_ATTN_CLOCK_PROBE 0  // diagnostic builds only (tools/build_variants.py attn_clock): per-workgroup clock stamps
#endif
#if PRL_ATTN_CLOCK_PROBE
// (shader clock, 100 MHz real time) at a workgroup's start and end, and wave 0's shader cycles per
// phase of the stage loop, into buffers of their own that nothing else reads (MI355X_MICROARCH.md,
// DVFS item 6); read by prl_attn_clock_read (tools/attn_clock.py [round 1-3 tool, in git history])
constexpr int kClockSlots = 1 << 16;
__device__ unsigned long long g_clock[4 * kClockSlots];
__device__ unsigned long long g_phase[8 * kClockSlots];
__device__ __forceinline__ void clock_stamp(int b, unsigned long long t0, unsigned long long r0) {
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && b < kClockSlots) {
    g_clock[4 * b] = t0;
    g_clock[4 * b + 1] = r0;
    g_clock[4 * b + 2] = t1;
    g_clock[4 * b + 3] = r1;
  }
}
// phases: 0 first barrier (waiting for the other waves), 1 LDS stage store + second barrier
// (incl. the wait for the stage's global loads), 2 issuing the next stage's loads, 3 paired
// tiles, 4 single (masked) tiles, 5 stages
// and, inside the paired tiles, wave 0's cycles per region of the pair schedule (regions 0-3 in
// the order of dkdv_pair / dq_pair; slot 4 counts the pairs)
__device__ unsigned long long g_pair[8 * kClockSlots];
struct PhaseClock {
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long pr[5] = {0, 0, 0, 0, 0};
  unsigned long long t = 0, tp = 0;
  __device__ __forceinline__ void start() { t = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void lap(int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    acc[i] += n - t;
    t = n;
  }
  __device__ __forceinline__ void pair_start() {
    tp = __builtin_amdgcn_s_memtime();
    pr[4]++;
  }
  __device__ __forceinline__ void pair_lap(int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    pr[i] += n - tp;
    tp = n;
  }
  __device__ __forceinline__ void store() const {
    const int b = blockIdx.x;
    if (threadIdx.x == 0 && b < kClockSlots) {
      for (int i = 0; i < 6; ++i) g_phase[8 * b + i] = acc[i];
      for (int i = 0; i < 5; ++i) g_pair[8 * b + i] = pr[i];
    }
  }
};
#define PROBE(x) x
#define PAIR_CLOCK_ARG , PhaseClock& pcl
#define PAIR_CLOCK_PASS , pc
#define PAIR_LAP(x) pcl.x
#else
#define PROBE(x)
#define PAIR_CLOCK_ARG
#define PAIR_CLOCK_PASS
#define PAIR_LAP(x)
#endif
// ---- dK / dV role: 32-query tiles against the wave's 32 keys (key on the lane) ----
__device__ __forceinline__ bool dkdv_live(int kw, int q0, int s1) {  // wave-uniform
  return !(kw >= s1 || kw > q0 + TILE - 1 || q0 >= s1);
}
// S = Q K^T and dP = dO V^T with the key on the lane.  K, V rows: PRL_ATTN_KV_LDS = 1 reads them
// from the workgroup's K / V images in LDS (kf / vf point at the wave's 32 rows there), 0 holds
// them in registers (64 VGPRs: with them the S / dP accumulators spill to AGPRs, and every
// softmax input costs a v_accvgpr_read)
#ifndef PRL_ATTN_KV_LDS
#define PRL_ATTN_KV_LDS 0  // A/B: 1 (K/V, Q/dO from LDS, 182 VGPRs) measured 8-12 % slower (profiles/r02_attn_regs_ab.jsonl)
#endif
// 2: K (Q in the dQ role) in registers, V (dO) from an LDS image of the block: 32 KiB, so two
// workgroups fit a CU (with PRL_ATTN_BWD_MINB = 2)
typedef const char* LdsRef;    // rows of a swizzled LDS image
typedef const bf16x8* RegRef;  // the lane's fragments in registers
__device__ __forceinline__ bf16x8 kv_frag(LdsRef base, int l32, int c, int hi) { return row_read(base, l32, 2 * c + hi); }
__device__ __forceinline__ bf16x8 kv_frag(RegRef f, int, int c, int) { return f[c]; }
template <typename KR, typename VR>
__device__ __forceinline__ void dkdv_scores(const char* tQ, const char* tdO, KR kf, VR vf, int l32, int hi,
                                            f32x16& S, f32x16& dP) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    S = mfma(row_read(tQ, l32, 2 * c + hi), kv_frag(kf, l32, c, hi), S);
    dP = mfma(row_read(tdO, l32, 2 * c + hi), kv_frag(vf, l32, c, hi), dP);
  }
}
// P = 2^(c2 S - L2), dS = P (dP - delta) in bf16, the 16 query rows of this lane's accumulator in
// 4 runs of 4 consecutive rows.  MASK = false when the whole tile is at or below the diagonal for
// every key of the wave: rows past the sequence end are zero-filled (zero Q, dO, L, delta) and add
// exact zeros; keys past the end only touch their own (unwritten) lanes.
template <bool MASK>
__device__ __forceinline__ void dkdv_probs(const f32x16& S, const f32x16& dP, const float* tL, const float* tDl, int q0,
                                           int key, bool kval, int s1, int hi, float c2, bf16x8* pb, bf16x8* sb) {
#pragma unroll
  for (int gg = 0; gg < 4; ++gg) {
    const f32x4 Lr = *reinterpret_cast<const f32x4*>(tL + 8 * gg + 4 * hi);
    const f32x4 Dr = *reinterpret_cast<const f32x4*>(tDl + 8 * gg + 4 * hi);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * gg + j;
      float p = bexp2(__builtin_fmaf(S[r], c2, -Lr[j]));
      if (MASK) {
        const int t = q0 + 8 * gg + 4 * hi + j;
        p = (kval && key <= t && t < s1) ? p : 0.f;
      }
      pb[r >> 3][r & 7] = (__bf16)p;
      sb[r >> 3][r & 7] = (__bf16)(p * (dP[r] - Dr[j]));
    }
  }
}
// the unmasked softmax of one half of the tile's 16 accumulator rows (HALF 0: rows 0-7 -> pb[0] / sb[0],
// HALF 1: rows 8-15 -> pb[1] / sb[1]); the same arithmetic as dkdv_probs<false>, so the two halves
// together give its results bit for bit
template <int HALF>
__device__ __forceinline__ void dkdv_probs_half(const f32x16& S, const f32x16& dP, const float* tL, const float* tDl,
                                                int hi, float c2, bf16x8* pb, bf16x8* sb) {
#pragma unroll
  for (int gg = 2 * HALF; gg < 2 * HALF + 2; ++gg) {
    const f32x4 Lr = *reinterpret_cast<const f32x4*>(tL + 8 * gg + 4 * hi);
    const f32x4 Dr = *reinterpret_cast<const f32x4*>(tDl + 8 * gg + 4 * hi);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * gg + j;
      const float p = bexp2(__builtin_fmaf(S[r], c2, -Lr[j]));
      pb[r >> 3][r & 7] = (__bf16)p;
      sb[r >> 3][r & 7] = (__bf16)(p * (dP[r] - Dr[j]));
    }
  }
}
// dV^T += dO^T P, dK^T += Q^T dS (unscaled)
__device__ __forceinline__ void dkdv_acc(const char* tQ, const char* tdO, int lane, const bf16x8* pb, const bf16x8* sb,
                                         f32x16* dKt, f32x16* dVt) {
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      dVt[dc] = mfma(tr_operand(tdO, lane, dc, ks), pb[ks], dVt[dc]);
      dKt[dc] = mfma(tr_operand(tQ, lane, dc, ks), sb[ks], dKt[dc]);
    }
}
// one tile, masked (the diagonal and ragged ends)
template <typename KR, typename VR>
__device__ __forceinline__ void dkdv_tile(const char* tQ, const char* tdO, const float* tL, const float* tDl, int q0,
                                          KR kf, VR vf, int key, bool kval, int s1, int lane,
                                          float c2, f32x16* dKt, f32x16* dVt) {
  const int hi = lane >> 5, l32 = lane & 31;
  f32x16 S = f32x16{}, dP = f32x16{};
  dkdv_scores(tQ, tdO, kf, vf, l32, hi, S, dP);
  bf16x8 pb[2], sb[2];
  dkdv_probs<true>(S, dP, tL, tDl, q0, key, kval, s1, hi, c2, pb, sb);
  dkdv_acc(tQ, tdO, lane, pb, sb, dKt, dVt);
}
// two unmasked tiles (a = the stage's first 32 rows, b = the next 32), interleaved
template <typename KR, typename VR>
__device__ __forceinline__ void dkdv_pair(const char* tQ, const char* tdO, const float* tL, const float* tDl,
                                          KR kf, VR vf, int key, bool kval, int s1, int lane,
                                          float c2, f32x16* dKt, f32x16* dVt PAIR_CLOCK_ARG) {
  const int hi = lane >> 5, l32 = lane & 31;
  const char *tQb = tQ + TILE * 256, *tdOb = tdO + TILE * 256;
  f32x16 Sa = f32x16{}, dPa = f32x16{}, Sb = f32x16{}, dPb = f32x16{};
  bf16x8 pa[2], sa[2], pb[2], sb[2];
  PAIR_LAP(pair_start());
  dkdv_scores(tQ, tdO, kf, vf, l32, hi, Sa, dPa);
  sched_fence();
  PAIR_LAP(pair_lap(0));
  dkdv_scores(tQb, tdOb, kf, vf, l32, hi, Sb, dPb);
  dkdv_probs<false>(Sa, dPa, tL, tDl, 0, key, kval, s1, hi, c2, pa, sa);
  interleave<16, 1, 8>();
  sched_fence();
  PAIR_LAP(pair_lap(1));
  dkdv_acc(tQ, tdO, lane, pa, sa, dKt, dVt);
  dkdv_probs<false>(Sb, dPb, tL + TILE, tDl + TILE, 0, key, kval, s1, hi, c2, pb, sb);
  interleave<16, 2, 8>();
  sched_fence();
  PAIR_LAP(pair_lap(2));
  dkdv_acc(tQb, tdOb, lane, pb, sb, dKt, dVt);
  PROBE(sched_fence());
  PAIR_LAP(pair_lap(3));
}

#ifndef PRL_ATTN_BWD_MINB
#define PRL_ATTN_BWD_MINB 1  // A/B: 2 = two workgroups per CU (<= 256 registers per lane)
#endif
#ifndef PRL_ATTN_PIPE
#define PRL_ATTN_PIPE 1  // 0: every stage through the two-barrier pair loop above (A/B, tools/build_variants.py attn_nopipe)
#endif
// The dK/dV role past the diagonal as one software pipeline over its 32-query tiles.  The pair loop
// above puts a tile's whole softmax (~110 vector instructions) under the 16 MFMAs of the next
// tile's S / dP, and both tiles' softmaxes under half of the pair's 64 MFMAs: those regions ran at
// 76-79 cycles per MFMA against 38-42 for the MFMA-only ones (tools/attn_clock.py [round 1-3 tool, in git history], pair regions).
// Here the MFMA stream is S/dP(t), dV/dK += (t-1), S/dP(t+1), dV/dK += t, ... and the softmax of
// tile t is split by accumulator rows into two halves, one under dV/dK += (t-1) and one under
// S/dP(t+1): every 16-MFMA segment carries half a softmax.  Tile t's stage must stay in LDS until
// dV/dK += t, which runs after the next stage's first tile, so stages rotate over three LDS slots
// and each stage needs one barrier: stage i+1 is stored (from the registers its loads filled one
// stage earlier) right after stage i's barrier, into the slot stage i-2 used, which every wave left
// before that barrier.  The accumulation order of dK^T / dV^T is the tile order, as in the pair
// loop, so results are bit-identical to it.
constexpr int kSlot = 2 * STAGE * D * 2 + 2 * STAGE * 4;  // Q image, dO image, L2, delta of one 64-row stage
static_assert(!PRL_ATTN_PIPE || (PRL_ATTN_KV_LDS == 0 && PRL_ATTN_INTERLEAVE && BSTAGE == 2 * TILE &&
                                 PRL_ATTN_BWD_MINB == 1),
              "the tile pipelines assume K / V (Q / dO) in registers, 64-row stages, paired tiles and one "
              "workgroup per CU (3 stage slots = 97.5 KiB of LDS): build those A/B variants with PRL_ATTN_PIPE=0");
__device__ __forceinline__ void pipe_store(const StageT<BSTAGE>& nq, const StageT<BSTAGE>& nd, float nl, float ndl,
                                           char* slot, int tid) {
  stage_store(nq, slot, tid);
  stage_store(nd, slot + STAGE * 256, tid);
  if (tid < BSTAGE) {
    float* f = reinterpret_cast<float*>(slot + 2 * STAGE * 256);
    f[tid] = nl;
    f[STAGE + tid] = ndl;
  }
}
__device__ __forceinline__ const float* slot_L(const char* slot) {
  return reinterpret_cast<const float*>(slot + 2 * STAGE * 256);
}
__device__ __forceinline__ const float* slot_D(const char* slot) { return slot_L(slot) + STAGE; }
// one 64-row stage of Q and dO (query head h, rows r0 .. r0 + 63) and its L2 / delta into an LDS slot by
// LDS-DMA: wave w fills rows 16w .. 16w + 15 of each image, 4 rows (1 KiB) per instruction.  The DMA
// writes lane-linearly (lane l -> byte 16 l of the instruction's 1 KiB), so the XOR swizzle of toff is
// applied on the source side: lane l reads chunk (l & 15) ^ swz(row) of its row.  Rows past the
// sequence end fall outside the buffer descriptors and land as zeros.  Waves 0 and 1 also fetch the
// 64 L2 / delta values (4 B per lane).  Completion: the __syncthreads that starts the stage's item.
typedef __attribute__((address_space(3))) void lds_void;
struct DmaJob {
  __amdgpu_buffer_rsrc_t rq, ro, rl;  // Q / dO rows r0 .. s1 - 1 of all heads; this wave's L2 (w 0) or delta (w 1)
  char* slot;                          // destination slot
  int soff;                            // the head's byte offset in a row
};
// the job for item (h, r0) into slot; valid = false: zero-size descriptors (the pieces move nothing)
__device__ __forceinline__ DmaJob make_job(const __bf16* __restrict__ q, const __bf16* __restrict__ dout,
                                           const float* __restrict__ lse2, const float* __restrict__ delta, int64_t rs,
                                           int64_t T, int h, int r0, int s1, char* slot, int w, bool valid) {
  const int r1 = valid ? s1 : r0;
  const float* src = (w == 0 ? lse2 : delta) + h * T + r0;
  const int nb = valid ? (s1 - r0 < STAGE ? s1 - r0 : STAGE) * 4 : 0;
  return DmaJob{rows_rsrc(q, rs, r0, r1), rows_rsrc(dout, rs, r0, r1),
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, nb, 0x00020000), slot, h * D * 2};
}
// the lane's byte offsets of its 16-B chunk in rows 16 w + 4 j + lane / 16 (j = 0..3) of a stage,
// the XOR swizzle applied on the source side (see stage_dma)
__device__ __forceinline__ void dma_lane_offsets(int64_t rs, int w, int lane, int* dvo) {
  const int p = lane & 15;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 16 * w + 4 * j + (lane >> 4);
    dvo[j] = r * (int)(rs * 2) + (p ^ (((r & 3) << 2) | ((r >> 2) & 3))) * 16;
  }
}
// piece k (0..8) of a job: 0-3 Q rows, 4-7 dO rows (1 KiB each), 8 the 64 L2 / delta values (waves 0, 1)
template <int K>
__device__ __forceinline__ void dma_piece(const DmaJob& j, const int* dvo, int w, int lane) {
  if constexpr (K < 4) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(j.rq, (lds_void*)(j.slot + 1024 * (4 * w + K)), 16, dvo[K], j.soff, 0, 0);
  } else if constexpr (K < 8) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(j.ro, (lds_void*)(j.slot + STAGE * 256 + 1024 * (4 * w + K - 4)), 16,
                                             dvo[K - 4], j.soff, 0, 0);
  } else {
    if (w < 2)  // wave-uniform
      __builtin_amdgcn_raw_ptr_buffer_load_lds(j.rl, (lds_void*)(j.slot + 2 * STAGE * 256 + w * STAGE * 4), 4,
                                               lane * 4, 0, 0, 0);
  }
}
// one 64-row stage of Q and dO (query head h, rows r0 .. r0 + 63) and its L2 / delta into an LDS slot
// by LDS-DMA: wave w fills rows 16w .. 16w + 15 of each image, 4 rows (1 KiB) per instruction.  The
// DMA writes lane-linearly (lane l -> byte 16 l of the instruction's 1 KiB), so the XOR swizzle of
// toff is applied on the source side: lane l reads chunk (l & 15) ^ swz(row) of its row.  Rows past
// the sequence end fall outside the buffer descriptors and land as zeros.  Completion: the
// __syncthreads that starts the stage's item.
__device__ __forceinline__ void stage_dma(const DmaJob& j, const int* dvo, int w, int lane) {
  dma_piece<0>(j, dvo, w, lane);
  dma_piece<1>(j, dvo, w, lane);
  dma_piece<2>(j, dvo, w, lane);
  dma_piece<3>(j, dvo, w, lane);
  dma_piece<4>(j, dvo, w, lane);
  dma_piece<5>(j, dvo, w, lane);
  dma_piece<6>(j, dvo, w, lane);
  dma_piece<7>(j, dvo, w, lane);
  dma_piece<8>(j, dvo, w, lane);
}

#ifndef PRL_ATTN_PIPE_SCHED
#define PRL_ATTN_PIPE_SCHED 1  // 0: the pipeline's segments scheduled by sched_group_barrier patterns (A/B)
#endif
#ifndef PRL_ATTN_PIPE_LEAD
#define PRL_ATTN_PIPE_LEAD 4  // MFMA operands read this many MFMAs ahead in the explicit schedule
#endif
// One pipelined stage (64 MFMAs) with every instruction placed by hand: gap g = MFMA g, the LDS
// reads of MFMA g + LEAD's operand and gap g's share of a softmax half, then a scheduling fence, so
// the compiler keeps the order (the sched_group_barrier patterns above left the vector work in
// clumps).  Segments of 16 gaps: S/dP(a) | dV/dK += previous b | S/dP(b) | dV/dK += a, carrying the
// softmax halves: previous b rows 8-15 | a rows 0-7 | a rows 8-15 | b rows 0-7.  In a segment, local
// gap t = 0 reads the half's L2 / delta rows, t = 2..9 forms p = 2^(c2 S - L2) of element t - 2 and
// t = 8..15 dS = p (dP - delta) of element t - 8, packing element pairs to bf16 (the arithmetic of
// dkdv_probs).  MFMA operands: S/dP segments: row reads (Q even, dO odd gaps, chunk 2 (t/2) + hi);
// dV/dK segments: transposed reads of dO (even) / Q (odd), d-chunk t / 4, k-step (t / 2) & 1 -- the
// order of dkdv_scores / dkdv_acc, so the accumulation order and the results are the pair loop's.
// PREV = false: the head's first pipelined stage (no previous tile b: no segment-1 vector work, no
// segment-2 MFMAs).  Every index below is a constant once the gap loop is unrolled.
struct PipeTile {
  const char *q, *o;   // the 32-row tile's Q and dO images in LDS
  const float *L, *D;  // its 32 L2 / delta values
};
__device__ __forceinline__ bf16x8 pipe_operand(int g, const PipeTile& pbt, const PipeTile& a, const PipeTile& b,
                                               int lane) {
  const int seg = g >> 4, t = g & 15;
  if (seg == 0 || seg == 2) {
    const PipeTile& x = seg == 0 ? a : b;
    return row_read((t & 1) ? x.o : x.q, lane & 31, 2 * (t >> 1) + (lane >> 5));
  }
  const PipeTile& y = seg == 1 ? pbt : a;
  return tr_operand((t & 1) ? y.q : y.o, lane, t >> 2, (t >> 1) & 1);
}
template <bool PREV>
struct PipeIter {
  static constexpr int LEAD = PRL_ATTN_PIPE_LEAD;
  static constexpr bool live(int g) { return PREV || (g >> 4) != 1; }  // MFMA g exists
  const PipeTile &pbt, &a, &b;
  const bf16x8 *kf, *vf;
  int lane, hi;
  float c2;
  f32x16 &Sa, &dPa, &Sb, &dPb;
  bf16x8 *pa, *sa, *pb, *sb;
  f32x16 *dKt, *dVt;
  bf16x8 ring[LEAD];
  f32x4 Lr[2], Dr[2];
  float pv[8];

  template <int G>
  __device__ __forceinline__ void gap() {
    constexpr int seg = G >> 4, t = G & 15;
    // 1. MFMA G
    if constexpr (live(G)) {
      const bf16x8 op = ring[G % LEAD];
      if constexpr (seg == 0 || seg == 2) {
        f32x16& S = seg == 0 ? Sa : Sb;
        f32x16& dP = seg == 0 ? dPa : dPb;
        if constexpr (t == 0) S = mfma(op, kf[0], f32x16{});
        else if constexpr (t == 1) dP = mfma(op, vf[0], f32x16{});
        else if constexpr (t & 1) dP = mfma(op, vf[t >> 1], dP);
        else S = mfma(op, kf[t >> 1], S);
      } else {
        const bf16x8* pp = seg == 1 ? pb : pa;
        const bf16x8* ss = seg == 1 ? sb : sa;
        constexpr int dc = t >> 2, ks = (t >> 1) & 1;
        if constexpr (t & 1) dKt[dc] = mfma(op, ss[ks], dKt[dc]);
        else dVt[dc] = mfma(op, pp[ks], dVt[dc]);
      }
    }
    // 2. the operand of MFMA G + LEAD
    if constexpr (G + LEAD < 64 && live(G + LEAD)) ring[(G + LEAD) % LEAD] = operand<G + LEAD>();
    // 3. this gap's share of the segment's softmax half
    if constexpr (PREV || seg != 0) {
      const f32x16& S = (seg == 0 || seg == 3) ? Sb : Sa;
      const f32x16& dP = (seg == 0 || seg == 3) ? dPb : dPa;
      const PipeTile& st = seg == 0 ? pbt : (seg == 3 ? b : a);
      constexpr int half = (seg == 0 || seg == 2) ? 1 : 0;
      bf16x8* pd = (seg == 0 || seg == 3) ? pb : pa;
      bf16x8* sd = (seg == 0 || seg == 3) ? sb : sa;
      if constexpr (t == 0) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          Lr[u] = *reinterpret_cast<const f32x4*>(st.L + 8 * (2 * half + u) + 4 * hi);
          Dr[u] = *reinterpret_cast<const f32x4*>(st.D + 8 * (2 * half + u) + 4 * hi);
        }
      }
      if constexpr (t >= 2 && t < 10) {  // p of element e: accumulator row 8 half + e
        constexpr int e = t - 2;
        pv[e] = bexp2(__builtin_fmaf(S[8 * half + e], c2, -Lr[e >> 2][e & 3]));
      }
      if constexpr (t >= 8) {  // dS of element e
        constexpr int e = t - 8;
        pd[half][e] = (__bf16)pv[e];
        sd[half][e] = (__bf16)(pv[e] * (dP[8 * half + e] - Dr[e >> 2][e & 3]));
      }
    }
    sched_fence();
  }
  template <int G>
  __device__ __forceinline__ bf16x8 operand() const {
    constexpr int seg = G >> 4, t = G & 15;
    if constexpr (seg == 0 || seg == 2) {
      const PipeTile& x = seg == 0 ? a : b;
      return row_read((t & 1) ? x.o : x.q, lane & 31, 2 * (t >> 1) + hi);
    } else {
      const PipeTile& y = seg == 1 ? pbt : a;
      return tr_operand((t & 1) ? y.q : y.o, lane, t >> 2, (t >> 1) & 1);
    }
  }
  template <int... G>
  __device__ __forceinline__ void prime(std::integer_sequence<int, G...>) {
    ((live(G) ? (void)(ring[G] = operand<G>()) : (void)0), ...);
  }
  template <int... G>
  __device__ __forceinline__ void run(std::integer_sequence<int, G...>) {
    (gap<G>(), ...);
  }
};
template <bool PREV>
__device__ __forceinline__ void dkdv_iter(const PipeTile& pbt, const PipeTile& a, const PipeTile& b,
                                          const bf16x8* kf, const bf16x8* vf, int lane, float c2, f32x16& Sa,
                                          f32x16& dPa, f32x16& Sb, f32x16& dPb, bf16x8* pa, bf16x8* sa, bf16x8* pb,
                                          bf16x8* sb, f32x16* dKt, f32x16* dVt) {
  PipeIter<PREV> it{pbt, a, b, kf, vf, lane, lane >> 5, c2, Sa, dPa, Sb, dPb, pa, sa, pb, sb, dKt, dVt, {}, {}, {}, {}};
  it.prime(std::make_integer_sequence<int, PipeIter<PREV>::LEAD>{});
  it.run(std::make_integer_sequence<int, 64>{});
}

// items: int32 triplets (seq_start, seq_end, block_start), block = 128 keys (dkdv) / queries (dq).
// GQA: k / v / dk / dv have Hkv heads, q / dout / dq have H = rep * Hkv; the dK/dV role of kv head
// g sweeps the query heads g*rep .. g*rep+rep-1 (all of its group), so dK / dV are complete sums
// in registers with no atomics.
// h0 .. h1-1: the query heads this workgroup sweeps (all of the group, or a part of it for a split
// heavy key block); part != null: write the unscaled fp32 accumulators there ([2][128][128],
// dK then dV, row = key - kb) for attn_bwd_dkdv_reduce instead of bf16 dk / dv.
__device__ __forceinline__ void attn_bwd_dkdv(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                              const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                              const float* __restrict__ lse2, const float* __restrict__ delta,
                                              int s1, int kb, int h0, int h1, __bf16* __restrict__ dk,
                                              __bf16* __restrict__ dv, float* __restrict__ part, int64_t T, int H,
                                              int Hkv, float c2, float scale, int g, char* sQ, char* sdO, float* sL,
                                              float* sDl, char* sKV, char* sPipe) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, hi = lane >> 5, l32 = lane & 31;
  const int64_t rsq = (int64_t)H * D, rsk = (int64_t)Hkv * D;
  const int rep = H / Hkv;
  const int kw = kb + 32 * w;
  const int key = kw + l32;
  const bool kval = key < s1;
#if PRL_ATTN_KV_LDS == 1
  {  // the block's 128 K and V rows into two swizzled images (visible after the loop's first barriers)
    const Stage k0 = stage_load(k, rsk, g, kb, s1, tid), k1 = stage_load(k, rsk, g, kb + STAGE, s1, tid);
    const Stage v0 = stage_load(v, rsk, g, kb, s1, tid), v1 = stage_load(v, rsk, g, kb + STAGE, s1, tid);
    stage_store(k0, sKV, tid);
    stage_store(k1, sKV + STAGE * 256, tid);
    stage_store(v0, sKV + 128 * 256, tid);
    stage_store(v1, sKV + 128 * 256 + STAGE * 256, tid);
  }
  const LdsRef kf = sKV + 32 * w * 256, vf = sKV + 128 * 256 + 32 * w * 256;
#elif PRL_ATTN_KV_LDS == 2
  {  // the block's 128 V rows into a swizzled image (visible after the loop's first barriers)
    const Stage v0 = stage_load(v, rsk, g, kb, s1, tid), v1 = stage_load(v, rsk, g, kb + STAGE, s1, tid);
    stage_store(v0, sKV, tid);
    stage_store(v1, sKV + STAGE * 256, tid);
  }
  bf16x8 kf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) kf[c] = kval ? ld8(k + (int64_t)key * rsk + g * D + 16 * c + 8 * hi) : zero8();
  const LdsRef vf = sKV + 32 * w * 256;
#else
  bf16x8 kf[8], vf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    kf[c] = kval ? ld8(k + (int64_t)key * rsk + g * D + 16 * c + 8 * hi) : zero8();
    vf[c] = kval ? ld8(v + (int64_t)key * rsk + g * D + 16 * c + 8 * hi) : zero8();
  }
#endif
  f32x16 dKt[4], dVt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dKt[i] = f32x16{};
    dVt[i] = f32x16{};
  }
  PROBE(PhaseClock pc);
#if PRL_ATTN_PIPE
  {
    // the sequence of (query head, 64-row stage) items; item m lands in LDS slot m % 3 by LDS-DMA
    // issued right after item m - 1's barrier (one stage ahead, no staging registers, no LDS store
    // pass), and the barrier that starts item m (its __syncthreads waits for the DMA) is the only
    // one per stage.  Stages 0 and 1 of a head hold the diagonal: the pair / masked-tile code;
    // stages from 2 on: the pipeline, drained at the head's last stage.
    const int nst = (s1 - kb + BSTAGE - 1) / BSTAGE;
    PROBE(PhaseClock& pcl = pc);
    const int wu = __builtin_amdgcn_readfirstlane(w);  // provably wave-uniform: descriptors and LDS bases in SGPRs
    int dvo[4];
    dma_lane_offsets(rsq, wu, lane, dvo);
    stage_dma(make_job(q, dout, lse2, delta, rsq, T, h0, kb, s1, sPipe, wu, true), dvo, wu, lane);
    int cs = 0;
    // start item (h, i): wait for it, then refill the slot two items back with the next item
    // (issuing the 9 pieces one every 7 MFMAs of the schedule instead measured slower: 4543 vs 4337
    // cycles per stage; each piece holds the wave ~100 cycles wherever it is issued)
    auto begin_item = [&](int h, int i) -> char* {
      const int ns = cs == 2 ? 0 : cs + 1;
      PROBE(pc.start(); pc.acc[5]++);
      // the LDS-DMA of item (h, i) done (hipcc's wait before the barrier does not always count the
      // DMA: one loop's barrier had none, and dK went wrong), then every wave's
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // item (h, i) is in slot cs; every wave is done with the slot ns held
      PROBE(pc.lap(0));
      const int hn = i + 1 < nst ? h : h + 1, in = i + 1 < nst ? i + 1 : 0;
      stage_dma(make_job(q, dout, lse2, delta, rsq, T, hn, kb + in * BSTAGE, s1, sPipe + ns * kSlot, wu,
                         hn < h1 && !PRL_ATTN_EXP_NOLOAD),
                dvo, wu, lane);
      sched_fence();
      PROBE(pc.lap(2));
      char* const cur = sPipe + cs * kSlot;
      cs = ns;
      return cur;
    };
#pragma unroll 1
    for (int h = h0; h < h1; ++h) {
#pragma unroll 1
      for (int i = 0; i < 2 && i < nst; ++i) {  // the diagonal stages
        const char* const cur = begin_item(h, i);
        const char *cq = cur, *co = cur + STAGE * 256;
        const float *cL = slot_L(cur), *cD = slot_D(cur);
        const int q00 = kb + i * BSTAGE;
        if (PRL_ATTN_INTERLEAVE && kw < s1 && q00 >= kw + TILE - 1 && q00 + TILE < s1) {  // wave-uniform
          dkdv_pair(cq, co, cL, cD, kf, vf, key, kval, s1, lane, c2, dKt, dVt PAIR_CLOCK_PASS);
        } else {
#pragma unroll 1
          for (int half = 0; half < BSTAGE / TILE; ++half) {
            const int q0 = q00 + TILE * half;
            if (!dkdv_live(kw, q0, s1)) continue;  // wave-uniform
            dkdv_tile(cq + half * TILE * 256, co + half * TILE * 256, cL + half * TILE, cD + half * TILE, q0, kf, vf,
                      key, kval, s1, lane, c2, dKt, dVt);
          }
        }
        PROBE(pc.lap(4));
      }
      if (nst <= 2) continue;
      // stages 2 .. nst - 1: every row is past every key of the block (no masks)
      f32x16 Sa, dPa, Sb, dPb;
      bf16x8 pa[2], sa[2], pb[2], sb[2];
#if PRL_ATTN_PIPE_SCHED
      auto tiles = [](const char* cur, PipeTile& ta, PipeTile& tb) {
        ta = PipeTile{cur, cur + STAGE * 256, slot_L(cur), slot_D(cur)};
        tb = PipeTile{cur + TILE * 256, cur + STAGE * 256 + TILE * 256, slot_L(cur) + TILE, slot_D(cur) + TILE};
      };
      PipeTile ta, tb, prevb;
      tiles(begin_item(h, 2), ta, tb);
      PAIR_LAP(pair_start());
      dkdv_iter<false>(ta, ta, tb, kf, vf, lane, c2, Sa, dPa, Sb, dPb, pa, sa, pb, sb, dKt, dVt);
      PAIR_LAP(pair_lap(3));
      PROBE(pc.lap(3));
      prevb = tb;
#pragma unroll 1
      for (int i = 3; i < nst; ++i) {
        tiles(begin_item(h, i), ta, tb);
        PAIR_LAP(pair_start());
        dkdv_iter<true>(prevb, ta, tb, kf, vf, lane, c2, Sa, dPa, Sb, dPb, pa, sa, pb, sb, dKt, dVt);
        PAIR_LAP(pair_lap(3));
        PROBE(pc.lap(3));
        prevb = tb;
      }
      // drain: the head's last tile b
      dkdv_probs_half<1>(Sb, dPb, prevb.L, prevb.D, hi, c2, pb, sb);
      sched_fence();
      dkdv_acc(prevb.q, prevb.o, lane, pb, sb, dKt, dVt);
      sched_fence();
#else
      const char* cur = begin_item(h, 2);
      const char *cq = cur, *co = cur + STAGE * 256;
      const float *cL = slot_L(cur), *cD = slot_D(cur);
      Sa = f32x16{};
      dPa = f32x16{};
      dkdv_scores(cq, co, kf, vf, l32, hi, Sa, dPa);
      sched_fence();
      dkdv_probs_half<0>(Sa, dPa, cL, cD, hi, c2, pa, sa);
      sched_fence();
#pragma unroll 1
      for (int i = 2;; ++i) {
        PAIR_LAP(pair_start());
        if (i > 2) {
          const char *pq = cq, *po = co;
          const float *pL = cL, *pD = cD;
          cur = begin_item(h, i);
          cq = cur;
          co = cur + STAGE * 256;
          cL = slot_L(cur);
          cD = slot_D(cur);
          PAIR_LAP(pair_start());
          // S / dP of tile a | the previous tile b's softmax, rows 8-15
          dkdv_probs_half<1>(Sb, dPb, pL + TILE, pD + TILE, hi, c2, pb, sb);
          Sa = f32x16{};
          dPa = f32x16{};
          dkdv_scores(cq, co, kf, vf, l32, hi, Sa, dPa);
          interleave_seg<16, 1, 4>();
          sched_fence();
          PAIR_LAP(pair_lap(0));
          // dV / dK += the previous tile b | tile a's softmax, rows 0-7
          dkdv_probs_half<0>(Sa, dPa, cL, cD, hi, c2, pa, sa);
          dkdv_acc(pq + TILE * 256, po + TILE * 256, lane, pb, sb, dKt, dVt);
          interleave_seg<16, 2, 4>();
          sched_fence();
          PAIR_LAP(pair_lap(1));
        }
        // S / dP of tile b | tile a's softmax, rows 8-15
        dkdv_probs_half<1>(Sa, dPa, cL, cD, hi, c2, pa, sa);
        Sb = f32x16{};
        dPb = f32x16{};
        dkdv_scores(cq + TILE * 256, co + TILE * 256, kf, vf, l32, hi, Sb, dPb);
        interleave_seg<16, 1, 4>();
        sched_fence();
        PAIR_LAP(pair_lap(2));
        // dV / dK += tile a | tile b's softmax, rows 0-7
        dkdv_probs_half<0>(Sb, dPb, cL + TILE, cD + TILE, hi, c2, pb, sb);
        dkdv_acc(cq, co, lane, pa, sa, dKt, dVt);
        interleave_seg<16, 2, 4>();
        sched_fence();
        PAIR_LAP(pair_lap(3));
        PROBE(pc.lap(3));
        if (i + 1 == nst) break;
      }
      // drain: the head's last tile b
      dkdv_probs_half<1>(Sb, dPb, cL + TILE, cD + TILE, hi, c2, pb, sb);
      sched_fence();
      dkdv_acc(cq + TILE * 256, co + TILE * 256, lane, pb, sb, dKt, dVt);
      sched_fence();
#endif
    }
  }
#else
#pragma unroll 1
  for (int h = h0; h < h1; ++h) {
  const int vb = stage_vbase(rsq, h, tid);
  StageT<BSTAGE> nq = stage_load_rows<BSTAGE>(q, rsq, h, kb, s1, tid, vb),
                 nd = stage_load_rows<BSTAGE>(dout, rsq, h, kb, s1, tid, vb);
  float nl = 0.f, ndl = 0.f;
  if (tid < BSTAGE && kb + tid < s1) {
    nl = lse2[(int64_t)h * T + kb + tid];
    ndl = delta[(int64_t)h * T + kb + tid];
  }
  for (int q00 = kb; q00 < s1; q00 += BSTAGE) {
    PROBE(pc.start(); pc.acc[5]++);
    __syncthreads();  // every wave is done with the previous stage
    PROBE(pc.lap(0));
    stage_store(nq, sQ, tid);
    stage_store(nd, sdO, tid);
    if (tid < BSTAGE) {
      sL[tid] = nl;
      sDl[tid] = ndl;
    }
    __syncthreads();
    PROBE(pc.lap(1));
    const int qn = q00 + BSTAGE;  // prefetch the next stage behind this stage's MFMAs
    if (qn < s1 && !PRL_ATTN_EXP_NOLOAD) {
      nq = stage_load_rows<BSTAGE>(q, rsq, h, qn, s1, tid, vb);
      nd = stage_load_rows<BSTAGE>(dout, rsq, h, qn, s1, tid, vb);
      if (tid < BSTAGE && qn + tid < s1) {
        nl = lse2[(int64_t)h * T + qn + tid];
        ndl = delta[(int64_t)h * T + qn + tid];
      }
    }
    PROBE(pc.lap(2));
    if (PRL_ATTN_INTERLEAVE && BSTAGE == 2 * TILE && kw < s1 && q00 >= kw + TILE - 1 && q00 + TILE < s1) {  // wave-uniform
      dkdv_pair(sQ, sdO, sL, sDl, kf, vf, key, kval, s1, lane, c2, dKt, dVt PAIR_CLOCK_PASS);
      PROBE(pc.lap(3));
      continue;
    }
#pragma unroll 1
    for (int half = 0; half < BSTAGE / TILE; ++half) {
      const int q0 = q00 + TILE * half;
      if (!dkdv_live(kw, q0, s1)) continue;  // wave-uniform
      dkdv_tile(sQ + half * TILE * 256, sdO + half * TILE * 256, sL + half * TILE, sDl + half * TILE, q0, kf, vf, key,
                kval, s1, lane, c2, dKt, dVt);
    }
    PROBE(pc.lap(4));
  }
  }
#endif
  PROBE(pc.store());
  if (!kval) return;
  if (part) {
    float* pk = part + (int64_t)(key - kb) * D;
    float* pv = pk + 128 * D;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d0 = 32 * dc + 8 * gg + 4 * hi;
        *reinterpret_cast<f32x4*>(pk + d0) = f32x4{dKt[dc][4 * gg], dKt[dc][4 * gg + 1], dKt[dc][4 * gg + 2],
                                                   dKt[dc][4 * gg + 3]};
        *reinterpret_cast<f32x4*>(pv + d0) = f32x4{dVt[dc][4 * gg], dVt[dc][4 * gg + 1], dVt[dc][4 * gg + 2],
                                                   dVt[dc][4 * gg + 3]};
      }
    return;
  }
  __bf16* dkr = dk + (int64_t)key * rsk + g * D;
  __bf16* dvr = dv + (int64_t)key * rsk + g * D;
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * dc + 8 * g + 4 * hi;
      st4(dkr + d0, scale * dKt[dc][4 * g], scale * dKt[dc][4 * g + 1], scale * dKt[dc][4 * g + 2],
          scale * dKt[dc][4 * g + 3]);
      st4(dvr + d0, dVt[dc][4 * g], dVt[dc][4 * g + 1], dVt[dc][4 * g + 2], dVt[dc][4 * g + 3]);
    }
}

// ---- dQ role: 32-key tiles against the wave's 32 queries (query on the lane) ----
__device__ __forceinline__ bool dq_live(int qw, int k0, int s1, int kend) {  // wave-uniform
  return !(qw >= s1 || k0 > qw + TILE - 1 || k0 >= kend);
}
template <typename KR, typename VR>
__device__ __forceinline__ void dq_scores(const char* tK, const char* tV, KR qf, VR of, int l32, int hi,
                                          f32x16& St, f32x16& dPt) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    St = mfma(row_read(tK, l32, 2 * c + hi), kv_frag(qf, l32, c, hi), St);
    dPt = mfma(row_read(tV, l32, 2 * c + hi), kv_frag(of, l32, c, hi), dPt);
  }
}
// dS^T in bf16.  MASK = false when every key of the tile is at or below every query of the wave
// and inside the sequence (a key past the end has S = 0 and would give 2^(-L2), unbounded).
template <bool MASK>
__device__ __forceinline__ void dq_probs(const f32x16& St, const f32x16& dPt, int k0, int qq, bool qval, int s1, int hi,
                                         float c2, float lq, float dq_delta, bf16x8* sb) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float p = bexp2(__builtin_fmaf(St[r], c2, -lq));
    if (MASK) {
      const int kj = k0 + 8 * (r >> 2) + 4 * hi + (r & 3);
      p = (qval && kj <= qq && kj < s1) ? p : 0.f;
    }
    sb[r >> 3][r & 7] = (__bf16)(p * (dPt[r] - dq_delta));
  }
}
__device__ __forceinline__ void dq_acc(const char* tK, int lane, const bf16x8* sb, f32x16* dQt) {
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) dQt[dc] = mfma(tr_operand(tK, lane, dc, ks), sb[ks], dQt[dc]);
}
// one tile, masked
template <typename KR, typename VR>
__device__ __forceinline__ void dq_tile(const char* tK, const char* tV, int k0, KR qf, VR of,
                                        int qq, bool qval, int s1, int lane, float c2, float lq, float dq_delta,
                                        f32x16* dQt) {
  const int hi = lane >> 5, l32 = lane & 31;
  f32x16 St = f32x16{}, dPt = f32x16{};
  dq_scores(tK, tV, qf, of, l32, hi, St, dPt);
  bf16x8 sb[2];
  dq_probs<true>(St, dPt, k0, qq, qval, s1, hi, c2, lq, dq_delta, sb);
  dq_acc(tK, lane, sb, dQt);
}
// two unmasked tiles, interleaved as in dkdv_pair
template <typename KR, typename VR>
__device__ __forceinline__ void dq_pair(const char* tK, const char* tV, KR qf, VR of, int qq,
                                        bool qval, int s1, int lane, float c2, float lq, float dq_delta, f32x16* dQt
                                        PAIR_CLOCK_ARG) {
  const int hi = lane >> 5, l32 = lane & 31;
  const char *tKb = tK + TILE * 256, *tVb = tV + TILE * 256;
  f32x16 Sa = f32x16{}, dPa = f32x16{}, Sb = f32x16{}, dPb = f32x16{};
  bf16x8 sa[2], sb[2];
  PAIR_LAP(pair_start());
  dq_scores(tK, tV, qf, of, l32, hi, Sa, dPa);
  sched_fence();
  PAIR_LAP(pair_lap(0));
  dq_scores(tKb, tVb, qf, of, l32, hi, Sb, dPb);
  dq_probs<false>(Sa, dPa, 0, qq, qval, s1, hi, c2, lq, dq_delta, sa);
  interleave<16, 1, 5>();
  sched_fence();
  PAIR_LAP(pair_lap(1));
  dq_acc(tK, lane, sa, dQt);
  dq_probs<false>(Sb, dPb, 0, qq, qval, s1, hi, c2, lq, dq_delta, sb);
  interleave<8, 2, 10>();
  sched_fence();
  PAIR_LAP(pair_lap(2));
  dq_acc(tKb, lane, sb, dQt);
  PROBE(sched_fence());
  PAIR_LAP(pair_lap(3));
}

#if PRL_ATTN_PIPE
// The dQ role's stages below the diagonal as the same kind of pipeline as the dK/dV role's: per 64-key
// stage (tiles a, b) the MFMA stream S/dP(a) 16 | dQ += previous b 8 | S/dP(b) 16 | dQ += a 8, and
// each tile's softmax (16 elements: p = 2^(c2 S - L2), dS = p (dP - delta), L2 and delta per lane)
// spread over the 24 MFMAs between its S/dP and its dQ product: tile a over gaps 16-39, tile b over
// gaps 40-47 and the next stage's 0-15.  The 32 half-operations (p of an element, dS of an element:
// p0 p1 s0 p2 s1 ... p15 s14 s15) go to window gap (3 j) / 4.  The order of the dQ accumulation is
// the pair loop's (dq_acc), so the results are its bit for bit.
template <int J>
struct DqOp {  // half-operation J of a tile's softmax: kind 0 = p of element e, 1 = dS of element e
  static constexpr int kind = J == 0 ? 0 : (J == 31 ? 1 : ((J & 1) ? 0 : 1));
  static constexpr int e = J == 0 ? 0 : (J == 31 ? 15 : ((J & 1) ? (J + 1) / 2 : J / 2 - 1));
};
template <bool PREV>
struct DqIter {
  static constexpr int LEAD = PRL_ATTN_PIPE_LEAD;
  static constexpr bool live(int g) { return PREV || g < 16 || g >= 24; }  // MFMA g exists
  const char *kpb, *ka, *va, *kb, *vb;  // tile images: previous b's K; a's and b's K and V
  const bf16x8 *qf, *of;
  int lane, hi;
  float c2, lq, dlt;
  f32x16 &Sa, &dPa, &Sb, &dPb;
  bf16x8 *sa, *sb;
  float* pv;  // p of tile b's elements carried over the stage seam
  f32x16* dQt;
  bf16x8 ring[LEAD];
  float pa[16];

  template <int G>
  __device__ __forceinline__ bf16x8 operand() const {
    if constexpr (G < 16 || (G >= 24 && G < 40)) {
      constexpr int t = G < 16 ? G : G - 24;
      return row_read((t & 1) ? (G < 16 ? va : vb) : (G < 16 ? ka : kb), lane & 31, 2 * (t >> 1) + hi);
    } else {
      constexpr int t = G < 24 ? G - 16 : G - 40;
      return tr_operand(G < 24 ? kpb : ka, lane, t >> 1, t & 1);
    }
  }
  // half-op J of the softmax of S / dP into p / dst
  template <int J>
  __device__ __forceinline__ void sm_op(const f32x16& S, const f32x16& dP, float* p, bf16x8* dst) {
    constexpr int e = DqOp<J>::e;
    if constexpr (DqOp<J>::kind == 0) p[e] = bexp2(__builtin_fmaf(S[e], c2, -lq));
    else dst[e >> 3][e & 7] = (__bf16)(p[e] * (dP[e] - dlt));
  }
  // the half-ops whose window gap (3 j / 4) is U: tile a's window starts at gap 16, tile b's at 40
  template <int U, int J = 0>
  __device__ __forceinline__ void sm_gap(const f32x16& S, const f32x16& dP, float* p, bf16x8* dst) {
    if constexpr (J < 32) {
      if constexpr ((3 * J) / 4 == U) sm_op<J>(S, dP, p, dst);
      sm_gap<U, J + 1>(S, dP, p, dst);
    }
  }
  template <int G>
  __device__ __forceinline__ void gap() {
    if constexpr (live(G)) {
      const bf16x8 op = ring[G % LEAD];
      if constexpr (G < 16 || (G >= 24 && G < 40)) {
        constexpr int t = G < 16 ? G : G - 24;
        f32x16& S = G < 16 ? Sa : Sb;
        f32x16& dP = G < 16 ? dPa : dPb;
        if constexpr (t == 0) S = mfma(op, qf[0], f32x16{});
        else if constexpr (t == 1) dP = mfma(op, of[0], f32x16{});
        else if constexpr (t & 1) dP = mfma(op, of[t >> 1], dP);
        else S = mfma(op, qf[t >> 1], S);
      } else {
        constexpr int t = G < 24 ? G - 16 : G - 40;
        dQt[t >> 1] = mfma(op, (G < 24 ? sb : sa)[t & 1], dQt[t >> 1]);
      }
    }
    if constexpr (G + LEAD < 48 && live(G + LEAD)) ring[(G + LEAD) % LEAD] = operand<G + LEAD>();
    if constexpr (G < 16) {  // the previous tile b's window gaps 8 .. 23
      if constexpr (PREV) sm_gap<G + 8>(Sb, dPb, pv, sb);
    } else if constexpr (G < 40) {  // tile a's window gaps 0 .. 23
      sm_gap<G - 16>(Sa, dPa, pa, sa);
    } else {  // tile b's window gaps 0 .. 7
      sm_gap<G - 40>(Sb, dPb, pv, sb);
    }
    sched_fence();
  }
  template <int... G>
  __device__ __forceinline__ void prime(std::integer_sequence<int, G...>) {
    ((live(G) ? (void)(ring[G] = operand<G>()) : (void)0), ...);
  }
  template <int... G>
  __device__ __forceinline__ void run(std::integer_sequence<int, G...>) {
    (gap<G>(), ...);
  }
  // the last tile b of the pipeline: the rest of its softmax (window gaps 8 .. 23), then dQ += b
  template <int... U>
  __device__ __forceinline__ void drain_sm(std::integer_sequence<int, U...>) {
    (sm_gap<U + 8>(Sb, dPb, pv, sb), ...);
  }
};
template <bool PREV>
__device__ __forceinline__ void dq_iter(const char* kpb, const char* ka, const char* va, const char* kb,
                                        const char* vb, const bf16x8* qf, const bf16x8* of, int lane, float c2,
                                        float lq, float dlt, f32x16& Sa, f32x16& dPa, f32x16& Sb, f32x16& dPb,
                                        bf16x8* sa, bf16x8* sb, float* pv, f32x16* dQt) {
  DqIter<PREV> it{kpb, ka, va, kb, vb, qf, of, lane, lane >> 5, c2, lq, dlt, Sa, dPa, Sb, dPb, sa, sb, pv, dQt, {}, {}};
  it.prime(std::make_integer_sequence<int, DqIter<PREV>::LEAD>{});
  it.run(std::make_integer_sequence<int, 48>{});
}
__device__ __forceinline__ void dq_drain(const char* kpb, const bf16x8* qf, const bf16x8* of, int lane, float c2,
                                         float lq, float dlt, f32x16& Sb, f32x16& dPb, bf16x8* sb, float* pv,
                                         f32x16* dQt) {
  f32x16 dummy;
  DqIter<true> it{kpb, kpb, kpb, kpb, kpb, qf, of, lane, lane >> 5, c2, lq, dlt, dummy, dummy, Sb, dPb, sb, sb, pv,
                  dQt, {}, {}};
  it.drain_sm(std::make_integer_sequence<int, 16>{});
  sched_fence();
  dq_acc(kpb, lane, sb, dQt);
}
// one 64-key stage of K and V (kv head g, keys r0 .. r0 + 63) into an LDS slot by LDS-DMA, as stage_dma
__device__ __forceinline__ void stage_dma_kv(const __bf16* __restrict__ k, const __bf16* __restrict__ v, int64_t rs,
                                             int g, int r0, int r1, char* slot, const int* dvo, int w) {
  const __amdgpu_buffer_rsrc_t rk = rows_rsrc(k, rs, r0, r1);
  const DmaJob j{rk, rows_rsrc(v, rs, r0, r1), rk, slot, g * D * 2};  // (rl unused: no piece 8)
  dma_piece<0>(j, dvo, w, 0);
  dma_piece<1>(j, dvo, w, 0);
  dma_piece<2>(j, dvo, w, 0);
  dma_piece<3>(j, dvo, w, 0);
  dma_piece<4>(j, dvo, w, 0);
  dma_piece<5>(j, dvo, w, 0);
  dma_piece<6>(j, dvo, w, 0);
  dma_piece<7>(j, dvo, w, 0);
}
#endif
__device__ __forceinline__ void attn_bwd_dq(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                   const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                   const float* __restrict__ lse2, const float* __restrict__ delta,
                                                   const int32_t* __restrict__ items, __bf16* __restrict__ dq,
                                                   int64_t T, int H, int Hkv, float c2, float scale, int it, int h,
                                                   char* sK, char* sV, char* sQO) {
  const int tid = threadIdx.x;
  const int s0 = items[3 * it], s1 = items[3 * it + 1], qb = items[3 * it + 2];
  const int lane = tid & 63, w = tid >> 6, hi = lane >> 5, l32 = lane & 31;
  const int64_t rs = (int64_t)H * D, rsk = (int64_t)Hkv * D;
  const int g = h / (H / Hkv);  // this query head's kv head
  const int qw = qb + 32 * w;
  const int qq = qw + l32;
  const bool qval = qq < s1;
#if PRL_ATTN_KV_LDS == 1
  {  // the block's 128 Q and dO rows into two swizzled images (visible after the loop's barriers)
    const Stage q0 = stage_load(q, rs, h, qb, s1, tid), q1 = stage_load(q, rs, h, qb + STAGE, s1, tid);
    const Stage o0 = stage_load(dout, rs, h, qb, s1, tid), o1 = stage_load(dout, rs, h, qb + STAGE, s1, tid);
    stage_store(q0, sQO, tid);
    stage_store(q1, sQO + STAGE * 256, tid);
    stage_store(o0, sQO + 128 * 256, tid);
    stage_store(o1, sQO + 128 * 256 + STAGE * 256, tid);
  }
  const LdsRef qf = sQO + 32 * w * 256, of = sQO + 128 * 256 + 32 * w * 256;
#elif PRL_ATTN_KV_LDS == 2
  {  // the block's 128 dO rows into a swizzled image (visible after the loop's barriers)
    const Stage o0 = stage_load(dout, rs, h, qb, s1, tid), o1 = stage_load(dout, rs, h, qb + STAGE, s1, tid);
    stage_store(o0, sQO, tid);
    stage_store(o1, sQO + STAGE * 256, tid);
  }
  bf16x8 qf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) qf[c] = qval ? ld8(q + (int64_t)qq * rs + h * D + 16 * c + 8 * hi) : zero8();
  const LdsRef of = sQO + 32 * w * 256;
#else
  bf16x8 qf[8], of[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    qf[c] = qval ? ld8(q + (int64_t)qq * rs + h * D + 16 * c + 8 * hi) : zero8();
    of[c] = qval ? ld8(dout + (int64_t)qq * rs + h * D + 16 * c + 8 * hi) : zero8();
  }
#endif
  const float lq = qval ? lse2[(int64_t)h * T + qq] : 0.f;
  const float dq_delta = qval ? delta[(int64_t)h * T + qq] : 0.f;
  f32x16 dQt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dQt[i] = f32x16{};
  const int kend = (qb + 128 < s1 ? qb + 128 : s1);  // causal: keys <= the block's last query
  PROBE(PhaseClock pc);
#if PRL_ATTN_PIPE
  {
    // key stage m = keys s0 + 64 m in LDS slot m % 3 by LDS-DMA one stage ahead, one barrier per stage
    // (as the dK/dV role); stages before the block's first query (m < np) are below the diagonal
    // for every wave: the pipeline; the last two: the pair / masked-tile code
    const int wu = __builtin_amdgcn_readfirstlane(w);
    int dvo[4];
    dma_lane_offsets(rsk, wu, lane, dvo);
    const int nk = (kend - s0 + BSTAGE - 1) / BSTAGE, np = (qb - s0) / BSTAGE;
    stage_dma_kv(k, v, rsk, g, s0, s1, sQO, dvo, wu);
    int cs = 0;
    auto begin_item = [&](int m) -> char* {
      const int ns = cs == 2 ? 0 : cs + 1;
      PROBE(pc.start(); pc.acc[5]++);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this stage's LDS-DMA (see the dK/dV role)
      __syncthreads();
      PROBE(pc.lap(0));
      if (m + 1 < nk && !PRL_ATTN_EXP_NOLOAD)
        stage_dma_kv(k, v, rsk, g, s0 + (m + 1) * BSTAGE, s1, sQO + ns * kSlot, dvo, wu);
      sched_fence();
      PROBE(pc.lap(2));
      char* const cur = sQO + cs * kSlot;
      cs = ns;
      return cur;
    };
    if (np > 0) {
      f32x16 Sa, dPa, Sb, dPb;
      bf16x8 sa[2], sb[2];
      float pv[16];
      const char* cur = begin_item(0);
      dq_iter<false>(cur, cur, cur + STAGE * 256, cur + TILE * 256, cur + STAGE * 256 + TILE * 256, qf, of, lane, c2,
                     lq, dq_delta, Sa, dPa, Sb, dPb, sa, sb, pv, dQt);
      PROBE(pc.lap(3));
#pragma unroll 1
      for (int m = 1; m < np; ++m) {
        const char* kpb = cur + TILE * 256;
        cur = begin_item(m);
        dq_iter<true>(kpb, cur, cur + STAGE * 256, cur + TILE * 256, cur + STAGE * 256 + TILE * 256, qf, of, lane,
                      c2, lq, dq_delta, Sa, dPa, Sb, dPb, sa, sb, pv, dQt);
        PROBE(pc.lap(3));
      }
      dq_drain(cur + TILE * 256, qf, of, lane, c2, lq, dq_delta, Sb, dPb, sb, pv, dQt);
    }
#pragma unroll 1
    for (int m = np; m < nk; ++m) {  // the diagonal stages
      const char* const cur = begin_item(m);
      const char *tK = cur, *tV = cur + STAGE * 256;
      const int k00 = s0 + m * BSTAGE;
      if (PRL_ATTN_INTERLEAVE && qw < s1 && k00 + BSTAGE - 1 <= qw && k00 + BSTAGE <= s1) {  // wave-uniform
        dq_pair(tK, tV, qf, of, qq, qval, s1, lane, c2, lq, dq_delta, dQt PAIR_CLOCK_PASS);
      } else {
#pragma unroll 1
        for (int half = 0; half < BSTAGE / TILE; ++half) {
          const int k0 = k00 + TILE * half;
          if (!dq_live(qw, k0, s1, kend)) continue;  // wave-uniform
          dq_tile(tK + half * TILE * 256, tV + half * TILE * 256, k0, qf, of, qq, qval, s1, lane, c2, lq, dq_delta,
                  dQt);
        }
      }
      PROBE(pc.lap(4));
    }
  }
#else
  const int vb = stage_vbase(rsk, g, tid);
  StageT<BSTAGE> nk = stage_load_rows<BSTAGE>(k, rsk, g, s0, s1, tid, vb),
                 nv = stage_load_rows<BSTAGE>(v, rsk, g, s0, s1, tid, vb);
  for (int k00 = s0; k00 < kend; k00 += BSTAGE) {
    PROBE(pc.start(); pc.acc[5]++);
    __syncthreads();
    PROBE(pc.lap(0));
    stage_store(nk, sK, tid);
    stage_store(nv, sV, tid);
    __syncthreads();
    PROBE(pc.lap(1));
    if (k00 + BSTAGE < kend && !PRL_ATTN_EXP_NOLOAD) {
      nk = stage_load_rows<BSTAGE>(k, rsk, g, k00 + BSTAGE, s1, tid, vb);
      nv = stage_load_rows<BSTAGE>(v, rsk, g, k00 + BSTAGE, s1, tid, vb);
    }
    PROBE(pc.lap(2));
    if (PRL_ATTN_INTERLEAVE && BSTAGE == 2 * TILE && qw < s1 && k00 + BSTAGE - 1 <= qw && k00 + BSTAGE <= s1) {  // wave-uniform
      dq_pair(sK, sV, qf, of, qq, qval, s1, lane, c2, lq, dq_delta, dQt PAIR_CLOCK_PASS);
      PROBE(pc.lap(3));
      continue;
    }
#pragma unroll 1
    for (int half = 0; half < BSTAGE / TILE; ++half) {
      const int k0 = k00 + TILE * half;
      if (!dq_live(qw, k0, s1, kend)) continue;  // wave-uniform
      dq_tile(sK + half * TILE * 256, sV + half * TILE * 256, k0, qf, of, qq, qval, s1, lane, c2, lq, dq_delta, dQt);
    }
    PROBE(pc.lap(4));
  }
#endif
  PROBE(pc.store());
  if (!qval) return;
  __bf16* dqr = dq + (int64_t)qq * rs + h * D;
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 32 * dc + 8 * g + 4 * hi;
      st4(dqr + d0, scale * dQt[dc][4 * g], scale * dQt[dc][4 * g + 1], scale * dQt[dc][4 * g + 2],
          scale * dQt[dc][4 * g + 3]);
    }
}

#ifndef PRL_ATTN_XCD
#define PRL_ATTN_XCD 1  // A/B (tools/build_variants.py attn_xcd_off): fwd 28/4 heads 0.343 -> 0.318 ms at 8 x 2048
#endif
// XCD-aware order of the query-block workgroups (forward, dQ role).  Workgroups are dealt round-
// robin over the 8 XCDs (blocks b and b + 8 share an L2), so the `rep` query heads of one kv group
// (consecutive logical blocks, reading the same K / V stages) would land on `rep` different L2s.
// Remap: physical block b (x = b % 8, s = b / 8) runs logical group j = (s / G) * 8 + x, member
// s % G, so a group's G blocks share an XCD while consecutive groups still go to different XCDs
// (the heaviest-first item order is kept across the chip).  Bijective on [0, N - N % (8 G));
// the tail keeps the identity.
__device__ __forceinline__ int xcd_group_remap(int b, int n, int G) {
  if (!PRL_ATTN_XCD || G <= 1) return b;
  const int main = n - n % (8 * G);
  if (b >= main) return b;
  const int x = b & 7, sl = b >> 3;
  return ((sl / G) * 8 + x) * G + sl % G;
}

// One launch for both roles: workgroups [0, n_split) are the parts of split heavy dK/dV work
// (split units: int32 (seq_start, seq_end, block_start, kv head, h0, h1, slot), each writing fp32
// partials to parts + slot * 2 * 128 * 128), [n_split, n_split + n_kv * Hkv) compute dK/dV of a
// (key block, kv head) over the whole query-head group, the rest dQ of a (query block, query
// head), so the lighter dQ workgroups fill the causal tail.
__global__ __launch_bounds__(256, PRL_ATTN_BWD_MINB) void attn_bwd_fused(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                      const __bf16* __restrict__ v, const __bf16* __restrict__ dout,
                                                      const float* __restrict__ lse2, const float* __restrict__ delta,
                                                      const int32_t* __restrict__ kv_items, int n_kv,
                                                      const int32_t* __restrict__ q_items, __bf16* __restrict__ dq,
                                                      __bf16* __restrict__ dk, __bf16* __restrict__ dv, int64_t T,
                                                      int H, int Hkv, float c2, float scale,
                                                      const int32_t* __restrict__ split_units, int n_split,
                                                      float* __restrict__ parts) {
#if PRL_ATTN_PIPE
  // three stage slots for the dK/dV role; the dQ role's K / V stage uses the first 32 KiB (at the
  // bottom of LDS: its reads keep 16-bit immediate offsets; at slot 2 the dQ role ran 4-10 % slower)
  __shared__ __attribute__((aligned(16))) char sPipe[3 * kSlot];
  char* const s0 = sPipe;
  char* const s1 = s0 + STAGE * D * 2;
  float* const sL = reinterpret_cast<float*>(s0 + 2 * STAGE * D * 2);
  float* const sDl = sL + STAGE;
#else
  __shared__ __attribute__((aligned(16))) char s0[STAGE * D * 2], s1[STAGE * D * 2];
  __shared__ __attribute__((aligned(16))) float sL[STAGE], sDl[STAGE];
  char* const sPipe = nullptr;
#endif
#if PRL_ATTN_KV_LDS
  // K and V (mode 2: V) images of the key block; the dQ role's Q and dO (dO)
  __shared__ __attribute__((aligned(16))) char sKV[(PRL_ATTN_KV_LDS == 1 ? 2 : 1) * 128 * D * 2];
#else
  char* sKV = nullptr;
#endif
  const int b = blockIdx.x;
  const int rep = H / Hkv;
#if PRL_ATTN_CLOCK_PROBE
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (b < n_split) {
    const int32_t* u = split_units + 7 * b;
    attn_bwd_dkdv(q, k, v, dout, lse2, delta, u[1], u[2], u[4], u[5], dk, dv, parts + (int64_t)u[6] * 2 * 128 * D, T,
                  H, Hkv, c2, scale, u[3], s0, s1, sL, sDl, sKV, sPipe);
  } else if (b < n_split + n_kv * Hkv) {
    const int it = (b - n_split) / Hkv, g = (b - n_split) % Hkv;
    attn_bwd_dkdv(q, k, v, dout, lse2, delta, kv_items[3 * it + 1], kv_items[3 * it + 2], g * rep, (g + 1) * rep, dk,
                  dv, nullptr, T, H, Hkv, c2, scale, g, s0, s1, sL, sDl, sKV, sPipe);
  } else {
    const int nd = n_split + n_kv * Hkv;
    const int lq = xcd_group_remap(b - nd, (int)gridDim.x - nd, rep);
    attn_bwd_dq(q, k, v, dout, lse2, delta, q_items, dq, T, H, Hkv, c2, scale, lq / H, lq % H, s0, s1,
                PRL_ATTN_PIPE ? sPipe : sKV);
  }
#if PRL_ATTN_CLOCK_PROBE
  clock_stamp(b, t0, r0);
#endif
}

// dK / dV of split key blocks: the parts' fp32 partials summed in part order (deterministic),
// dK scaled, rounded to bf16.  groups: int32 (seq_end, block_start, kv head, first slot, parts);
// one thread per (key, 8 head-dim columns), 16 keys per 256-thread workgroup.
__global__ __launch_bounds__(256) void attn_bwd_dkdv_reduce(const float* __restrict__ parts,
                                                            const int32_t* __restrict__ groups,
                                                            __bf16* __restrict__ dk, __bf16* __restrict__ dv, int Hkv,
                                                            float scale) {
  const int gi = blockIdx.x >> 3;  // 8 workgroups x 16 keys per 128-key block
  const int32_t* gr = groups + 5 * gi;
  const int s1 = gr[0], kb = gr[1], g = gr[2], slot0 = gr[3], np = gr[4];
  const int r = ((blockIdx.x & 7) << 4) + (threadIdx.x >> 4), c8 = (threadIdx.x & 15) * 8;
  const int key = kb + r;
  if (key >= s1) return;
  float ak[8] = {}, av[8] = {};
  for (int p = 0; p < np; ++p) {
    const float* pk = parts + (int64_t)(slot0 + p) * 2 * 128 * D + (int64_t)r * D + c8;
    const f32x4 k0 = *reinterpret_cast<const f32x4*>(pk), k1 = *reinterpret_cast<const f32x4*>(pk + 4);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(pk + 128 * D), v1 = *reinterpret_cast<const f32x4*>(pk + 128 * D + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ak[j] += k0[j];
      ak[4 + j] += k1[j];
      av[j] += v0[j];
      av[4 + j] += v1[j];
    }
  }
  const int64_t o = (int64_t)key * Hkv * D + (int64_t)g * D + c8;
  st4(dk + o, scale * ak[0], scale * ak[1], scale * ak[2], scale * ak[3]);
  st4(dk + o + 4, scale * ak[4], scale * ak[5], scale * ak[6], scale * ak[7]);
  st4(dv + o, av[0], av[1], av[2], av[3]);
  st4(dv + o + 4, av[4], av[5], av[6], av[7]);
}

// Forward (same structure as the dQ role): one workgroup = 128 queries of one query head, each
// wave owns 32 queries with the query on the MFMA lane; per 32-key tile S^T = K Q^T, an online
// base-2 softmax per query (lane) with a lazy rescale of the output accumulators (only when the
// running max grows by more than 8), O^T += V^T P with V^T read transposed from the tile image.
// Writes O [T, H, 128] bf16 and lse2[h][t] = log2 sum_j 2^(c2 S_tj) (the backward's input).
constexpr float kRescale = 8.0f;
#ifndef PRL_ATTN_FWD_MINB
#define PRL_ATTN_FWD_MINB 2  // 2 workgroups per CU = 2 waves per SIMD: one wave's softmax under the other's MFMAs
#endif
// one 32-key tile of the forward: S^T = K Q^T, online softmax update of (m, l, O^T), O^T += V^T P.
// MASK: masked scores become -1e30 (p = 0 once m is finite: the first tile of a sequence always
// holds key s0, visible to every query)
template <bool MASK>
__device__ __forceinline__ void fwd_tile(const char* tK, const char* tV, int k0, const bf16x8* qf, int qq, bool qval,
                                         int s1, int lane, float c2, float& m, float& l, f32x16* Ot) {
  const int hi = lane >> 5, l32 = lane & 31;
  f32x16 St = f32x16{};
#pragma unroll
  for (int c = 0; c < 8; ++c) St = mfma(row_read(tK, l32, 2 * c + hi), qf[c], St);
  if (MASK) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kj = k0 + 8 * (r >> 2) + 4 * hi + (r & 3);
      if (!(qval && kj <= qq && kj < s1)) St[r] = -1e30f;
    }
  }
  float tmax = St[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, St[r]);
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c2;  // the other half of this query's keys; c2 > 0
  if (tmax > m + kRescale) {  // lazy rebase, per lane
    const float f = fexp2(m - tmax);
    l *= f;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
#pragma unroll
      for (int r = 0; r < 16; ++r) Ot[dc][r] *= f;
    m = tmax;
  }
  bf16x8 pb[2];
  float ps = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = fexp2(__builtin_fmaf(St[r], c2, -m));
    ps += p;
    pb[r >> 3][r & 7] = (__bf16)p;
  }
  l += ps + __shfl_xor(ps, 32, 64);
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) Ot[dc] = mfma(tr_operand(tV, lane, dc, ks), pb[ks], Ot[dc]);
}

#ifndef PRL_ATTN_FWD_DMA
#define PRL_ATTN_FWD_DMA 1
#endif
#if PRL_ATTN_FWD_DMA && !PRL_ATTN_PIPE
#error "PRL_ATTN_FWD_DMA uses the pipeline's LDS-DMA stage loads (PRL_ATTN_PIPE)"
#endif
#ifndef PRL_ATTN_FWD_PAIR
#define PRL_ATTN_FWD_PAIR 1
#endif
#ifndef PRL_ATTN_FWD_PAIR_SPREAD
#define PRL_ATTN_FWD_PAIR_SPREAD 1  // tile b's softmax spread over tile a's P.V MFMAs (A/B: 0)
#endif
// both 32-key tiles of a stage every key of which is visible to every query of the wave: S of both
// tiles (16 MFMAs back to back), one running-max / lazy-rescale decision over the 64 keys (one
// cross-half exchange instead of two), then both tiles' P and O^T += V^T P (16 MFMAs).  Same
// arithmetic per element as fwd_tile; the rescale points can differ (decided per 64 keys), so the
// results match the per-tile form to rounding, not bit for bit.
__device__ __forceinline__ void fwd_pair(const char* tK, const char* tV, const bf16x8* qf, int lane, float c2, float& m,
                                         float& l, f32x16* Ot) {
  const int hi = lane >> 5, l32 = lane & 31;
  f32x16 Sa = f32x16{}, Sb = f32x16{};
#pragma unroll
  for (int c = 0; c < 8; ++c) Sa = mfma(row_read(tK, l32, 2 * c + hi), qf[c], Sa);
#pragma unroll
  for (int c = 0; c < 8; ++c) Sb = mfma(row_read(tK + TILE * 256, l32, 2 * c + hi), qf[c], Sb);
  // the max of the 32 scores by v_max3_f32 (fmaxf put a canonicalizing v_max beside almost every
  // max of MFMA results: 54 instructions for 31 maxima)
  float tmax = fmaxf(Sa[0], Sb[0]);
#pragma unroll
  for (int r = 1; r < 16; ++r) asm("v_max3_f32 %0, %1, %2, %3" : "=v"(tmax) : "v"(tmax), "v"(Sa[r]), "v"(Sb[r]));
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c2;
  if (tmax > m + kRescale) {
    const float f = fexp2(m - tmax);
    l *= f;
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
#pragma unroll
      for (int r = 0; r < 16; ++r) Ot[dc][r] *= f;
    m = tmax;
  }
  bf16x8 pa[2], pb[2];
  float ps = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = fexp2(__builtin_fmaf(Sa[r], c2, -m));
    ps += p;
    pa[r >> 3][r & 7] = (__bf16)p;
  }
#if PRL_ATTN_FWD_PAIR_SPREAD
  // tile b's probabilities two elements per gap of tile a's P.V MFMAs (the V operand read two MFMAs
  // ahead), fenced per gap so the compiler keeps the spread; same operations and summation order
  float pbv[16];
  bf16x8 ring[2] = {tr_operand(tV, lane, 0, 0), tr_operand(tV, lane, 0, 1)};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bf16x8 op = ring[i & 1];
    if (i + 2 < 16) {
      const int j = i + 2;
      ring[i & 1] = tr_operand(tV + (j >> 3) * TILE * 256, lane, (j & 7) >> 1, j & 1);
    }
    if (i < 8) {
      Ot[i >> 1] = mfma(op, pa[i & 1], Ot[i >> 1]);
#pragma unroll
      for (int e = 2 * i; e < 2 * i + 2; ++e) pbv[e] = fexp2(__builtin_fmaf(Sb[e], c2, -m));
      pb[i >> 2][(2 * i) & 7] = (__bf16)pbv[2 * i];
      pb[i >> 2][(2 * i + 1) & 7] = (__bf16)pbv[2 * i + 1];
    } else {
      if (i == 8) {
#pragma unroll
        for (int e = 0; e < 16; ++e) ps += pbv[e];
      }
      Ot[(i - 8) >> 1] = mfma(op, pb[i & 1], Ot[(i - 8) >> 1]);
    }
    sched_fence();
  }
  l += ps + __shfl_xor(ps, 32, 64);
#else
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = fexp2(__builtin_fmaf(Sb[r], c2, -m));
    ps += p;
    pb[r >> 3][r & 7] = (__bf16)p;
  }
  l += ps + __shfl_xor(ps, 32, 64);
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) Ot[dc] = mfma(tr_operand(tV, lane, dc, ks), pa[ks], Ot[dc]);
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) Ot[dc] = mfma(tr_operand(tV + TILE * 256, lane, dc, ks), pb[ks], Ot[dc]);
#endif
}

__global__ __launch_bounds__(256, PRL_ATTN_FWD_MINB) void attn_fwd(const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                                                const __bf16* __restrict__ v, const int32_t* __restrict__ items,
                                                __bf16* __restrict__ out, float* __restrict__ lse2, int64_t T, int H,
                                                int Hkv, float c2) {
#if PRL_ATTN_FWD_DMA
  // two K/V stage slots (64 KiB per workgroup, two workgroups per CU) filled by LDS-DMA one stage
  // ahead: one barrier per stage, no staging registers, no store pass.  Two separate arrays and a
  // loop unrolled by two, so every stage reads one array while the next stage's DMA writes the other
  // and the compiler can tell them apart (with one runtime-indexed array it waited for the in-flight
  // DMA, vmcnt(0), before the stage's first transposed read).
  __shared__ __attribute__((aligned(16))) char sKVa[2 * STAGE * D * 2], sKVb[2 * STAGE * D * 2];
#else
  __shared__ __attribute__((aligned(16))) char sK[STAGE * D * 2], sV[STAGE * D * 2];
#endif
  const int tid = threadIdx.x;
  const int lb = xcd_group_remap(blockIdx.x, gridDim.x, H / Hkv);
  const int it = lb / H, h = lb % H;
  const int s0 = items[3 * it], s1 = items[3 * it + 1], qb = items[3 * it + 2];
  const int lane = tid & 63, w = tid >> 6, hi = lane >> 5, l32 = lane & 31;
  const int64_t rs = (int64_t)H * D, rsk = (int64_t)Hkv * D;
  const int g = h / (H / Hkv);
  const int qw = qb + 32 * w;
  const int qq = qw + l32;
  const bool qval = qq < s1;
  bf16x8 qf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) qf[c] = qval ? ld8(q + (int64_t)qq * rs + h * D + 16 * c + 8 * hi) : zero8();
  f32x16 Ot[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) Ot[i] = f32x16{};
  float m = -1e30f, l = 0.f;  // running max (base-2 units) and sum for query qq
  const int kend = (qb + 128 < s1 ? qb + 128 : s1);
  // the stage's two 32-key tiles (keys k00 .. k00 + 63) from the K / V images in LDS
  auto tiles = [&](int k00, const char* sK, const char* sV) {
    if (PRL_ATTN_FWD_PAIR && qw < s1 && k00 + STAGE - 1 <= qw && k00 + STAGE <= s1) {  // wave-uniform
      fwd_pair(sK, sV, qf, lane, c2, m, l, Ot);
      return;
    }
#pragma unroll
    for (int half = 0; half < STAGE / TILE; ++half) {
      const int k0 = k00 + TILE * half;
      if (qw >= s1 || k0 > qw + TILE - 1 || k0 >= kend) continue;  // wave-uniform
      // every key of the tile visible to every query of the wave: the unmasked body (all but the
      // diagonal tile of each wave); wave-uniform, two separate code paths
      if (k0 + TILE - 1 <= qw && k0 + TILE <= s1)
        fwd_tile<false>(sK + half * TILE * 256, sV + half * TILE * 256, k0, qf, qq, qval, s1, lane, c2, m, l, Ot);
      else
        fwd_tile<true>(sK + half * TILE * 256, sV + half * TILE * 256, k0, qf, qq, qval, s1, lane, c2, m, l, Ot);
    }
  };
#if PRL_ATTN_FWD_DMA
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int dvo[4];
  dma_lane_offsets(rsk, wu, lane, dvo);
  stage_dma_kv(k, v, rsk, g, s0, s1, sKVa, dvo, wu);
  auto stage = [&](int k00, const char* cur, char* nxt) {
    // this wave's DMA of the stage landed (vmcnt), then every wave's (barrier); every wave is also
    // done with the other array's stage, which the next DMA overwrites
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (k00 + STAGE < kend) stage_dma_kv(k, v, rsk, g, k00 + STAGE, s1, nxt, dvo, wu);
    sched_fence();
    tiles(k00, cur, cur + STAGE * D * 2);
  };
  for (int k00 = s0; k00 < kend; k00 += 2 * STAGE) {
    stage(k00, sKVa, sKVb);
    if (k00 + STAGE < kend) stage(k00 + STAGE, sKVb, sKVa);
  }
#else
  const int vb = stage_vbase(rsk, g, tid);
  Stage nk = stage_load_rows(k, rsk, g, s0, s1, tid, vb), nv = stage_load_rows(v, rsk, g, s0, s1, tid, vb);
  for (int k00 = s0; k00 < kend; k00 += STAGE) {
    __syncthreads();
    stage_store(nk, sK, tid);
    stage_store(nv, sV, tid);
    __syncthreads();
    if (k00 + STAGE < kend) {
      nk = stage_load_rows(k, rsk, g, k00 + STAGE, s1, tid, vb);
      nv = stage_load_rows(v, rsk, g, k00 + STAGE, s1, tid, vb);
    }
    tiles(k00, sK, sV);
  }
#endif
  if (!qval) return;
  const float inv = 1.0f / l;
  __bf16* orow = out + (int64_t)qq * rs + h * D;
#pragma unroll
  for (int dc = 0; dc < 4; ++dc)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int d0 = 32 * dc + 8 * gg + 4 * hi;
      st4(orow + d0, Ot[dc][4 * gg] * inv, Ot[dc][4 * gg + 1] * inv, Ot[dc][4 * gg + 2] * inv,
          Ot[dc][4 * gg + 3] * inv);
    }
  if (hi == 0) lse2[(int64_t)h * T + qq] = m + __builtin_log2f(l);
}

// delta[h][t] = sum_d O dO (fp32) for the HIP forward's [H][T] lse2 (no layout conversion)
__global__ __launch_bounds__(256) void attn_bwd_delta(const __bf16* __restrict__ out, const __bf16* __restrict__ dout,
                                                      float* __restrict__ delta, int64_t T, int H) {
  const int sub = threadIdx.x & 15;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const bool live = row < T * H;
  float s = 0.f;
  if (live) {
    const bf16x8 o = ld8(out + row * D + 8 * sub), g = ld8(dout + row * D + 8 * sub);
#pragma unroll
    for (int i = 0; i < 8; ++i) s = __builtin_fmaf((float)o[i], (float)g[i], s);
  }
#pragma unroll
  for (int m = 8; m > 0; m >>= 1) s += __shfl_xor(s, m, 16);
  if (live && sub == 0) {
    const int64_t t = row / H;
    delta[(int64_t)(row - t * H) * T + t] = s;
  }
}

// delta[h][t] = sum_d O dO (fp32);  lse2[h][t] = L * log2(e), with L in torch's varlen layout
// [nseq][H][lse_len] (row of sequence b starting at token cu[b]).  One wave per (t, h).
__global__ __launch_bounds__(256) void attn_bwd_pre(const __bf16* __restrict__ out, const __bf16* __restrict__ dout,
                                                    const float* __restrict__ lse, const int32_t* __restrict__ cu,
                                                    int nseq, int64_t lse_len, float* __restrict__ lse2,
                                                    float* __restrict__ delta, int64_t T, int H) {
  // 16 lanes per (t, h) row of 128 elements: 8 per lane, 16 rows per workgroup
  const int sub = threadIdx.x & 15;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const bool live = row < T * H;
  float s = 0.f;
  if (live) {
    const bf16x8 o = ld8(out + row * D + 8 * sub), g = ld8(dout + row * D + 8 * sub);
#pragma unroll
    for (int i = 0; i < 8; ++i) s = __builtin_fmaf((float)o[i], (float)g[i], s);
  }
#pragma unroll
  for (int m = 8; m > 0; m >>= 1) s += __shfl_xor(s, m, 16);
  if (live && sub == 0) {
    const int64_t t = row / H;
    const int h = (int)(row - t * H);
    int lo = 0, hi = nseq - 1;  // last b with cu[b] <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (cu[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int64_t off = t - cu[lo];
    delta[(int64_t)h * T + t] = s;
    lse2[(int64_t)h * T + t] = off < lse_len ? lse[((int64_t)lo * H + h) * lse_len + off] * 1.4426950408889634f : 0.f;
  }
}

}  // namespace prl_attn

using namespace prl_attn;

extern "C" {

int prl_attn_bwd_preprocess(const void* out, const void* dout, const float* lse, const int32_t* cu_seqlens,
                            int32_t nseq, int64_t lse_len, float* lse2, float* delta, int64_t tokens, int32_t heads,
                            int32_t head_dim, void* stream) {
  if (!out || !dout || !lse || !cu_seqlens || !lse2 || !delta || tokens < 0 || heads <= 0 || nseq <= 0 ||
      lse_len <= 0)
    return PRL_E_INVALID;
  if (head_dim != D) return PRL_E_UNSUPPORTED;
  if (tokens == 0) return PRL_OK;
  const int64_t rows = tokens * heads;
  hipLaunchKernelGGL(attn_bwd_pre, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (const __bf16*)out, (const __bf16*)dout, lse, cu_seqlens, (int)nseq, lse_len, lse2, delta, tokens,
                     (int)heads);
  return (int)hipGetLastError();
}

int prl_attn_fwd(const void* q, const void* k, const void* v, const int32_t* q_items, int32_t n_q_items, void* out,
                 float* lse2, int64_t tokens, int32_t heads, int32_t kv_heads, int32_t head_dim, float scale,
                 void* stream) {
  if (!q || !k || !v || !out || !lse2 || tokens < 0 || heads <= 0 || kv_heads <= 0 || heads % kv_heads ||
      n_q_items < 0 || (n_q_items && !q_items))
    return PRL_E_INVALID;
  if (head_dim != D) return PRL_E_UNSUPPORTED;
  const int64_t blocks = (int64_t)n_q_items * heads;
  if (blocks > 0x7FFFFFFF) return PRL_E_UNSUPPORTED;
  if (blocks == 0) return PRL_OK;
  hipLaunchKernelGGL(attn_fwd, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, q_items, (__bf16*)out, lse2, tokens,
                     (int)heads, (int)kv_heads, scale * 1.4426950408889634f);
  return (int)hipGetLastError();
}

int prl_attn_bwd_delta(const void* out, const void* dout, float* delta, int64_t tokens, int32_t heads,
                       int32_t head_dim, void* stream) {
  if (!out || !dout || !delta || tokens < 0 || heads <= 0) return PRL_E_INVALID;
  if (head_dim != D) return PRL_E_UNSUPPORTED;
  if (tokens == 0) return PRL_OK;
  const int64_t rows = tokens * heads;
  hipLaunchKernelGGL(attn_bwd_delta, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), (const __bf16*)out, (const __bf16*)dout, delta, tokens,
                     (int)heads);
  return (int)hipGetLastError();
}

static int attn_bwd_launch(const void* q, const void* k, const void* v, const void* dout, const float* lse2,
                           const float* delta, const int32_t* kv_items, int32_t n_kv_items, const int32_t* q_items,
                           int32_t n_q_items, const int32_t* split_units, int32_t n_split,
                           const int32_t* split_groups, int32_t n_groups, float* parts, void* dq, void* dk, void* dv,
                           int64_t tokens, int32_t heads, int32_t kv_heads, int32_t head_dim, float scale,
                           void* stream) {
  if (!q || !k || !v || !dout || !lse2 || !delta || !dq || !dk || !dv || tokens < 0 || heads <= 0 || kv_heads <= 0 ||
      heads % kv_heads || n_kv_items < 0 || n_q_items < 0 || (n_kv_items && !kv_items) || (n_q_items && !q_items) ||
      n_split < 0 || n_groups < 0 || (n_split && (!split_units || !parts)) || (n_groups && (!split_groups || !parts)))
    return PRL_E_INVALID;
  if (head_dim != D) return PRL_E_UNSUPPORTED;
  const int64_t blocks = (int64_t)n_split + (int64_t)n_kv_items * kv_heads + (int64_t)n_q_items * heads;
  if (blocks > 0x7FFFFFFF || (int64_t)n_groups * 8 > 0x7FFFFFFF) return PRL_E_UNSUPPORTED;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float c2 = scale * 1.4426950408889634f;
  if (blocks > 0) {
    hipLaunchKernelGGL(attn_bwd_fused, dim3((unsigned)blocks), dim3(256), 0, s, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, (const __bf16*)dout, lse2, delta, kv_items, (int)n_kv_items, q_items,
                       (__bf16*)dq, (__bf16*)dk, (__bf16*)dv, tokens, (int)heads, (int)kv_heads, c2, scale,
                       split_units, (int)n_split, parts);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  if (n_groups > 0) {
    hipLaunchKernelGGL(attn_bwd_dkdv_reduce, dim3((unsigned)(8 * n_groups)), dim3(256), 0, s, parts, split_groups,
                       (__bf16*)dk, (__bf16*)dv, (int)kv_heads, scale);
    return (int)hipGetLastError();
  }
  return PRL_OK;
}

int prl_attn_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse2, const float* delta,
                 const int32_t* kv_items, int32_t n_kv_items, const int32_t* q_items, int32_t n_q_items, void* dq,
                 void* dk, void* dv, int64_t tokens, int32_t heads, int32_t kv_heads, int32_t head_dim, float scale,
                 void* stream) {
  return attn_bwd_launch(q, k, v, dout, lse2, delta, kv_items, n_kv_items, q_items, n_q_items, nullptr, 0, nullptr, 0,
                         nullptr, dq, dk, dv, tokens, heads, kv_heads, head_dim, scale, stream);
}

int prl_attn_bwd_split(const void* q, const void* k, const void* v, const void* dout, const float* lse2,
                       const float* delta, const int32_t* kv_items, int32_t n_kv_items, const int32_t* q_items,
                       int32_t n_q_items, const int32_t* split_units, int32_t n_split, const int32_t* split_groups,
                       int32_t n_groups, float* parts, void* dq, void* dk, void* dv, int64_t tokens, int32_t heads,
                       int32_t kv_heads, int32_t head_dim, float scale, void* stream) {
  return attn_bwd_launch(q, k, v, dout, lse2, delta, kv_items, n_kv_items, q_items, n_q_items, split_units, n_split,
                         split_groups, n_groups, parts, dq, dk, dv, tokens, heads, kv_heads, head_dim, scale, stream);
}

#if PRL_ATTN_CLOCK_PROBE
// diagnostic builds only: the stamps of the last attn_bwd_fused launch, 4 x n u64
int prl_attn_clock_read(unsigned long long* host, int32_t n) {
  if (!host || n < 0 || n > kClockSlots) return PRL_E_INVALID;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_clock), sizeof(unsigned long long) * 4 * (size_t)n, 0,
                                  hipMemcpyDeviceToHost);
}
int prl_attn_phase_read(unsigned long long* host, int32_t n) {
  if (!host || n < 0 || n > kClockSlots) return PRL_E_INVALID;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 8 * (size_t)n, 0,
                                  hipMemcpyDeviceToHost);
}
int prl_attn_pair_read(unsigned long long* host, int32_t n) {
  if (!host || n < 0 || n > kClockSlots) return PRL_E_INVALID;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair), sizeof(unsigned long long) * 8 * (size_t)n, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

}  // extern "C"
