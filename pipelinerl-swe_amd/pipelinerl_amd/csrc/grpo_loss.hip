// Fused GRPO loss head for MI355X (gfx950).  HBM-bound: one read of the [rows x V] logits,
// one write of dlogits, ~45 B of per-token side data.  No MFMA.
//
// Reference: pipelinerl/finetune/rl/__init__.py:199-366 (ATen op chain over [1, T, V]) and
// its autograd backward.  Kernels:
//   grpo_fwd_resident<NV>  bf16 logits, V % 8 == 0 (Qwen2.5: V = 151936 / 152064).
//       Persistent grid, one 1024-thread workgroup per CU, one vocab row per iteration; rows after
//       a workgroup's first are claimed from a counter in the caller's workspace (KArgs.row_ctr).
//       The whole row (V*2 B = 297 KiB) is held in VGPRs (NV x 16 B per lane), so the
//       gradient pass re-reads nothing.  Read / write phases: the row's dlogits stores retire,
//       then the whole next row (~300 KiB per CU) is loaded at once, so a CU never mixes HBM
//       reads and writes (3-4 % faster than loading vector k of row r+grid right behind the
//       store of vector k of row r; the phased schedule below).
//       Row reduction: per-lane online (max, sum 2^y, sum 2^y y) with lazy rebase, wave
//       shuffles, then one LDS exchange (double-buffered by row parity: one barrier/row).
//   grpo_fwd_pair_f32<NV>  fp32 logits: each row over a pair of workgroups (one half each, in
//       VGPRs), one tagged partial exchange per row, rows claimed by the pair's leader.
//   grpo_fwd_hybrid_f32<NR, NL> fp32 rows past the pair kernel's range: 75 % of the row on chip.
//   grpo_fwd_stream<T,VEC> any dtype / V: same math, row re-read for the gradient pass.
//   grpo_bwd_stream<T,VEC> gradient-only pass from the saved per-row coefficients.
//   grpo_stats_partial     the ~38 masked statistics of rl/__init__.py:315-375 and the
//                          value-head gradient, from the per-row outputs (light: ~60 B/row)
//   grpo_finalize          deterministic fold of the per-workgroup statistic partials.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "grpo_common.h"
#include "prl_hip.h"

namespace prl {

// Combine the per-wave states in LDS: global max first, then one accumulation pass (one
// exp2 per wave, short live ranges).  A NaN max anywhere poisons the row.
template <int NW>
__device__ __forceinline__ Lse block_combine(const float (*red)[3], float c) {
  float M = red[0][0];
  bool bad = M != M;
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    const float m = red[w][0];
    M = fmaxf(M, m);
    bad |= m != m;
  }
  float S = 0.f, W = 0.f;
#pragma unroll 4
  for (int w = 0; w < NW; ++w) {
    const float d = (red[w][0] - M) * c;
    const float f = fexp2(d);
    const float sw = red[w][1];
    S = __builtin_fmaf(sw, f, S);
    W = __builtin_fmaf(f, __builtin_fmaf(sw, d, red[w][2]), W);
  }
  if (bad) S = __builtin_nanf("");
  return Lse{M, S, W};
}

// per-row epilogue shared by the forward kernels: every lane computes the (uniform) token
// values and gradient coefficients; `writer` stores the per-row outputs.
__device__ __forceinline__ TokGrad row_epilogue(const KArgs& a, int64_t q, const TokIn& tin, float lp,
                                                float H, float lse, float m, float l2s, bool writer) {
  const TokVals v = token_values(a, tin, lp, H);
  const TokGrad g = token_grad(a, v);
  if (writer) {
    a.o_lp[q] = lp;
    a.o_ent[q] = H;
    a.o_lse[q] = lse;
    a.o_max[q] = m;
    a.o_l2s[q] = l2s;
    a.o_tok[q] = v.tl;
    a.o_glp[q] = g.g_lp;
    a.o_gh[q] = g.g_h;
  }
  return g;
}

// the rows' token inputs through the scalar cache (round 3; the vector-load form is retired)
using RowLd = SclLd;

// the target logit of a row, read through the scalar cache as the aligned dword holding it (no
// 16-bit scalar load on gfx950; rows of the streaming kernels may start 2-B aligned); j must be a
// valid column.  The dword can reach 2 B past the tensor's last element (odd V, last row), never
// past the 4-B-aligned granule holding it, so never into an unmapped page.
__device__ __forceinline__ float row_logit_scl(const uint16_t* row, int64_t j) {
  const uintptr_t ad = reinterpret_cast<uintptr_t>(row + j);
  const uint32_t w = SclLd::ld(reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3), 0);
  return __uint_as_float((ad & 2) ? (w & 0xffff0000u) : (w << 16));
}
__device__ __forceinline__ float row_logit_scl(const float* row, int64_t j) { return SclLd::ld(row, j); }
__device__ __forceinline__ float row_logit(const uint16_t* row, int64_t j) {
  return row_logit_scl(row, j);
}
__device__ __forceinline__ float row_logit(const float* row, int64_t j) {
  return row_logit_scl(row, j);
}

// Pin scalar-loaded row inputs to this point of the program: the scheduler otherwise sinks the
// s_loads to their first use after the row reduction and waits for them in front of the barrier.
// Here (the row's vector loads just issued) the wait costs nothing: pass 1 waits for the row anyway.
__device__ __forceinline__ void pin_sgpr(TokIn& t, float& x) {
  asm volatile("" : "+s"(t.label), "+s"(t.reward), "+s"(t.ref), "+s"(t.old), "+s"(t.gt), "+s"(t.ovf),
                 "+s"(t.advsrc), "+s"(x));
}

// buffer descriptor over one row (wave-uniform inputs only); out-of-range lanes read 0 and
// their stores are dropped by the hardware bounds check
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
// cache policy of the row stream (aux bits of buffer_load/store on gfx950: 1 = sc0, 2 = nt,
// 16 = sc1).  The logits and dlogits are touched once per launch; the build can override for A/B
// experiments.  Stores are nt sc1 (round 3): an sc1 store drops its line from the XCD's L2 instead
// of keeping it dirty there, so the dlogits stream does not evict through L2 write-backs; alternated
// on two boxes, 7.11 -> 6.97 and 7.40 -> 7.35 ms per C2 launch against nt alone (sc1 without nt,
// and sc0 sc1, were slower; the load policy made no difference: profiles/r03_loss_cache_policy_ab.jsonl).
#ifndef PRL_LOAD_AUX
#define PRL_LOAD_AUX 2
#endif
#ifndef PRL_STORE_AUX
#define PRL_STORE_AUX 18
#endif
constexpr int kLoadAux = PRL_LOAD_AUX;
constexpr int kStoreAux = PRL_STORE_AUX;
constexpr uint32_t kPadBf16x2 = 0xF1CAF1CAu;  // two bf16 -1.0e30: contributes 2^-huge = 0

// A 16-byte buffer store reads its data VGPRs after it issues.  A VALU write of one of those
// registers in the next issue slot replaced the stored data on MI355X (NV = 24 phased schedule:
// dword 1 of vectors 2 / 4 / 6 in lanes 12-15 of each 16 held the unpacked float of the next
// vector's logit; tools/nv24_probe.py).  LLVM inserts the wait state only for stores
// with no register in soffset, and these stores take the vector's row offset in an SGPR soffset,
// so it emitted none.  The store is therefore fenced: nothing is scheduled across the two
// barriers, and s_nop 1 gives the store two wait states before its data registers are reused
// (tools/isa_store_hazard_scan.py checks the built ISA: tests/test_isa_hazards_cpu.py).
#ifndef PRL_STORE_FENCE
#define PRL_STORE_FENCE 1
#endif
__device__ __forceinline__ void store_row_b128(u32x4 o, __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, o), rs,
                                         voff, soff, kStoreAux);
#if PRL_STORE_FENCE
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1");
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// The phased schedule (round 2): a row's stores retire (vmcnt(0)) before the next row's loads are
// issued, so this CU never mixes reads and writes: 7.50 -> 7.24 ms per C2 launch on one box
// (profiles/r02_loss_phase_ab.jsonl; the same schedule on a plain 20 GB copy:
// profiles/r02_phased_copy.jsonl).  Rows above kPhasedMaxNV keep the round-1 interleaved schedule
// (the next row's vector k loaded right behind the store of vector k).
// The phased schedule keeps pass 2's gradient vectors and the row in registers at once: above
// NV = 20 (V > 163 840) it spills row vectors to scratch, so rows that large keep the interleaved
// schedule.  (Its round-2 wrong dlogits at NV = 24 were the store-data hazard fenced in
// store_row_b128 below; both schedules are correct at every NV since.)  Qwen2.5's vocabularies are
// NV = 19, covered by tests/test_grpo_edge_gpu.py::test_multi_row_per_workgroup.
#ifndef PRL_PHASED_MAX_NV
#define PRL_PHASED_MAX_NV 20
#endif
constexpr int kPhasedMaxNV = PRL_PHASED_MAX_NV;
// Order in which the persistent grid visits the rows: iteration i processes row perm(i) (7.40 vs
// 7.46 ms per C2 launch against the identity, same box): the rows in flight at any moment are scattered over the whole [rows x V]
// tensor (i * P mod n, P a prime > n, so a bijection) instead of one contiguous ~76 MB window;
// per-row outputs are written per row, so results are bit-identical either way.
__device__ __forceinline__ int64_t perm_row(int64_t i, int64_t n) {
  return (int64_t)(((uint64_t)i * 2654435761ull) % (uint64_t)n);
}

// The exponent arguments on element pairs (packed FP32 ops): pass 1 y = (x - m) c with two
// partial sums per lane; pass 2 t = (x - M) c + k with a per-row constant k, and without an entropy
// term d = sign(alpha) 2^((x - M) c + log2|alpha| - log2 S): alpha folded into the exponent, its
// sign applied to the packed bf16 result, no multiply.  x - M stays an exact subtraction (x c - M c
// would lose |M c| ulp-scale accuracy at large logits: the scale-2000 edge test).  Results agree with
// the other kernels' scalar forms within the fp32 rounding of the exponent's argument (round 5).

// Pass 1's online state on element pairs: (max, pairwise sums of 2^y and 2^y y).
struct Lse2 {
  float m;
  f32x2 s, w;
};
template <int N>
__device__ __forceinline__ void lse2_add(Lse2& st, const float (&x)[N], float c) {
  float vm = x[0];
#pragma unroll
  for (int j = 1; j < N; ++j) vm = fmaxf(vm, x[j]);
  if ((vm - st.m) * c > kRescaleSlack) {  // lse_rebase on both halves
    const float d = (st.m - vm) * c;
    const float f = fexp2(d);
    st.w = f * (st.s * d + st.w);
    st.s = st.s * f;
    st.m = vm;
  }
  const f32x2 cc = {c, c}, mm = {st.m, st.m};
#pragma unroll
  for (int j = 0; j < N; j += 2) {
    const f32x2 xv = {x[j], x[j + 1]};
    const f32x2 y = (xv - mm) * cc;
    const f32x2 e = {fexp2(y.x), fexp2(y.y)};
    st.s += e;
    st.w = e * y + st.w;
  }
  if (vm != vm) st.m = __builtin_nanf("");  // a NaN logit poisons the state
}

template <int NV>
__global__ __launch_bounds__(1024) void grpo_fwd_resident(KArgs a) {
  constexpr int BLOCK = 1024, NW = BLOCK / 64;
  constexpr int VSTRIDE = BLOCK * 16;  // bytes between a lane's consecutive vectors
  // the phased schedule; with it the target column's extra g_lp/temperature term is written by the
  // owner lane after the row's stores retired, instead of 8 selects per vector in every lane (190
  // v_cndmask per row and wave in the ISA)
  constexpr bool kPhased = NV <= kPhasedMaxNV;
#ifdef PRL_COPY_CEILING
  constexpr bool kCopyCeiling = true;
#else
  constexpr bool kCopyCeiling = false;
#endif
#ifdef PRL_NO_PASS1
  // measurement only (with PRL_COPY_CEILING): pass 1's statistics skipped too — wrong results,
  // the schedule's pure data movement
  constexpr bool kNoPass1 = true;
#else
  constexpr bool kNoPass1 = false;
#endif
  __shared__ float red[2][NW][3];
  __shared__ int64_t next_q[2];  // the workgroup's next row, by row parity (published at the row's barrier)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t nrows = fwd_rows(a);
  const int nvec = (int)(a.V >> 3);
  const int64_t row_bytes = a.V * 2;
  const float c = kLog2e / a.temperature;
  const float inv_t = 1.0f / a.temperature;
  const uint16_t* __restrict__ lg = static_cast<const uint16_t*>(a.logits);
  uint16_t* __restrict__ dl = static_cast<uint16_t*>(a.dlogits);
  const int voff = tid * 16;
  const bool last_ok = (NV - 1) * BLOCK + tid < nvec;  // only vector NV-1 can be partial

  u32x4 buf[NV];
  int64_t q = blockIdx.x;
  if (q < nrows) {
    int64_t lrow, tok, qo;
    map_row(a, perm_row(q, nrows), lrow, tok, qo);
    const auto rs = row_rsrc(lg + lrow * a.ld, row_bytes);
#pragma unroll
    for (int k = 0; k < NV; ++k)
      buf[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * VSTRIDE, kLoadAux));
  }
  int par = 0;
  int64_t qn = q + gridDim.x;
  for (; q < nrows; q = qn, par ^= 1) {
    // Dynamic rows (a.row_ctr): the workgroup claims its next row now, while this row's loads are
    // in flight (one vector atomic by one thread; its latency hides behind the row's loads), and
    // publishes it at the row's barrier.  A workgroup that starts late — its CU held by another
    // queue's kernel (an RCCL channel, a side-stream kernel) — then takes fewer rows instead of
    // finishing a full static share after everyone else.  Rows are independent, so the results do
    // not depend on which workgroup computes which row.
    uint32_t claim = 0;
    if (a.row_ctr && tid == 0) claim = atomicAdd(a.row_ctr, 1u);
    // The row's token inputs and its target logit come through the scalar cache while the row's
    // vector loads are in flight: nothing here waits for them, and the epilogue after the
    // barrier finds its inputs in SGPRs (with vector loads this was a chain of four waits per
    // row, each for every load outstanding on the CU).
    int64_t lrow, tok, qo;
    map_row<RowLd>(a, perm_row(q, nrows), lrow, tok, qo);
    const int64_t tid_raw = RowLd::ld(a.input_ids, tok);
    TokIn tin = tok_in<RowLd>(a, tok);
    const bool bad_id = (uint64_t)tid_raw >= (uint64_t)a.V;
    const int64_t tgt = bad_id ? -1 : tid_raw;  // -1: never matches a column below
    float xr = row_logit(lg + lrow * a.ld, bad_id ? 0 : tid_raw);
    pin_sgpr(tin, xr);  // issue (and land) them here, not in front of the barrier
    const float xt = bad_id ? __builtin_nanf("") : xr;

    // ---- pass 1: row statistics from registers
    Lse st;
    Lse2 st2 = {kEmptyMax, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      u32x4 v = buf[k];
      if (k == NV - 1 && !last_ok) v = u32x4{kPadBf16x2, kPadBf16x2, kPadBf16x2, kPadBf16x2};
      float x[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = bf_lo(v[j]);
        x[2 * j + 1] = bf_hi(v[j]);
      }
      if constexpr (kNoPass1) {
        st2.s.x += x[0];  // keeps the loads' consumers (one add per vector)
      } else {
        lse2_add<8>(st2, x, c);
      }
    }
    st = Lse{st2.m, st2.s.x + st2.s.y, st2.w.x + st2.w.y};
    st = wave_reduce_lse(st, c);
    if (lane == 0) {  // (the wave index as an SGPR: a VGPR copy was the kernel's one scratch reload per row)
      const int wu = __builtin_amdgcn_readfirstlane(wid);
      red[par][wu][0] = st.m;
      red[par][wu][1] = st.s;
      red[par][wu][2] = st.w;
    }
    if (tid == 0) next_q[par] = a.row_ctr ? (int64_t)gridDim.x + (int64_t)claim : q + gridDim.x;
    __syncthreads();
    {  // wave-uniform in SGPRs: the next row's scalar loads and buffer descriptors are built from it
      const int64_t v = next_q[par];
      qn = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v));
    }
    const Lse tot = block_combine<NW>(red[par], c);
    const float l2s = log2f(tot.s);
    const float M = tot.m;
    const float lse = M * inv_t + kLn2 * l2s;
    const float H = kLn2 * (l2s - tot.w / tot.s);
    const float lp = (xt - M) * inv_t - kLn2 * l2s;
    const TokGrad core = row_epilogue(a, qo, tin, lp, H, lse, M, l2s, tid == 0);
    // Make the packed row opaque here so the compiler re-unpacks it in pass 2 instead of
    // keeping pass 1's unpacked floats alive (8 instead of 4 VGPRs per vector -> spills).
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(buf[k]));

    // ---- pass 2: gradient from registers; the next row streams into the freed registers
    const bool has_next = qn < nrows;
    int64_t nlrow = lrow;
    if (has_next) {
      int64_t nt, nq;
      map_row<RowLd>(a, perm_row(qn, nrows), nlrow, nt, nq);
    }
    const auto rn = row_rsrc(lg + nlrow * a.ld, has_next ? row_bytes : 0);
    if (a.write_grad) {
      const auto ws = row_rsrc(dl + lrow * a.ld, row_bytes);
      const float alpha = -(core.g_lp + core.g_h * H) * inv_t;
      const float beta = -core.g_h * kLn2 * inv_t;
      const float gadd = core.g_lp * inv_t;
      // folded forms: t = (x - M) c + k2 (k2 = -log2 S); without an entropy term
      // d = sign(alpha) 2^((x - M) c + k1), k1 = log2|alpha| - log2 S (alpha = 0: -inf, d = 0)
      const float k2 = -l2s;
      const float k1 = log2f(fabsf(alpha)) - l2s;
      const uint32_t sgn2 = alpha < 0.f ? 0x80008000u : 0u;
      const int tv = tgt < 0 ? -1 : (int)(tgt >> 3);
      const int te = (int)(tgt & 7);
      const int kt = tv < 0 ? -1 : tv / BLOCK;
      const int lt = tv - (kt < 0 ? 0 : kt) * BLOCK;
      const bool zero_row = (core.g_lp == 0.f && core.g_h == 0.f);
      // The row's stores, in one of three forms chosen per row (wave-uniform, so each form is its
      // own unrolled loop): kMode 0 a zero row, 1 no entropy term (beta == 0: the reference's default
      // entropy_bonus 0, one packed FMA fewer per element pair), 2 the general form.  Forms 1 and 2
      // agree bit for bit where beta == 0 but for the sign of a zero.
      auto row_pass = [&](auto mode) {
        constexpr int kMode = decltype(mode)::value;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          u32x4 o;
          if constexpr (kCopyCeiling) {  // structural ceiling experiment: same traffic and schedule, no gradient math
            o = buf[k];
          } else if constexpr (kMode == 0) {
            o = u32x4{0u, 0u, 0u, 0u};
          } else {
            // opaque per form, so the unpack shared by forms 1 and 2 is not hoisted above the
            // form branch (8 instead of 4 live VGPRs per vector: spills)
            u32x4 v = buf[k];
            asm volatile("" : "+v"(v));
            const f32x2 cc = {c, c}, mm = {M, M}, kk = {kMode == 1 ? k1 : k2, kMode == 1 ? k1 : k2};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const f32x2 xv = {bf_lo(v[j]), bf_hi(v[j])};
              const f32x2 t = (xv - mm) * cc + kk;
              const f32x2 p = {fexp2(t.x), fexp2(t.y)};
              if constexpr (kMode == 1) {
                o[j] = pack_bf16x2(p.x, p.y) ^ sgn2;
              } else {
                const f32x2 g = t * f32x2{beta, beta} + f32x2{alpha, alpha};
                const f32x2 dd = p * g;
                o[j] = pack_bf16x2(dd.x, dd.y);
              }
            }
          }
          store_row_b128(o, ws, voff, k * VSTRIDE);
        }
      };
      if constexpr (!kPhased) {
        // interleaved schedule (NV > 20): one form (three forms spill there), the next row's
        // vector k loaded right behind the store of vector k
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          u32x4 o;
          if (zero_row) {
            o = u32x4{0u, 0u, 0u, 0u};
          } else {
            float d[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float x0 = bf_lo(buf[k][j]), x1 = bf_hi(buf[k][j]);
              const float t0 = __builtin_fmaf(x0 - M, c, -l2s), t1 = __builtin_fmaf(x1 - M, c, -l2s);
              const float p0 = fexp2(t0), p1 = fexp2(t1);
              d[2 * j] = p0 * __builtin_fmaf(beta, t0, alpha);
              d[2 * j + 1] = p1 * __builtin_fmaf(beta, t1, alpha);
            }
            if (k == kt && tid == lt) {
#pragma unroll
              for (int j = 0; j < 8; ++j) d[j] += (j == te) ? gadd : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(d[2 * j], d[2 * j + 1]);
          }
          store_row_b128(o, ws, voff, k * VSTRIDE);
          buf[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rn, voff, k * VSTRIDE, kLoadAux));
        }
      } else if (zero_row)
        row_pass(std::integral_constant<int, 0>{});
      else if (beta == 0.f)
        row_pass(std::integral_constant<int, 1>{});
      else
        row_pass(std::integral_constant<int, 2>{});
      if constexpr (kPhased) {
        // the whole row's stores retire before the next row's loads start (the phased schedule)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // the target column's g_lp term, by its one owner lane after the row's stores retired
        // (so this 2-B store lands after the 16-B store of the same bytes): the same operations
        // as the vector loop on the same bf16 value, rounded the same way (no contraction)
        if (tid == lt && !zero_row) {
          float dm;
          if (beta == 0.f) {
            const float pt = fexp2(__builtin_fmaf(xt - M, c, k1));
            dm = alpha < 0.f ? -pt : pt;
          } else {
            const float tt = __builtin_fmaf(xt - M, c, k2);
            dm = __fmul_rn(fexp2(tt), __builtin_fmaf(tt, beta, alpha));
          }
          dl[lrow * a.ld + tgt] = f_to_bf(__fadd_rn(dm, gadd));
        }
        if (has_next) {
#pragma unroll
          for (int k = 0; k < NV; ++k)
            buf[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rn, voff, k * VSTRIDE, kLoadAux));
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k)
        buf[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rn, voff, k * VSTRIDE, kLoadAux));
    }
  }
}

// ---------------------------------------------------------------------------------------
// generic streaming path: T = float (PRL_F32) or uint16_t (bf16); VEC elements per access
// a 16-B store into a wave-uniform row through a buffer descriptor (soffset 0: the hardware wait
// state for the store data is emitted), with the resident kernel's cache policy
__device__ __forceinline__ void store_row16(void* row, int64_t gv, u32x4 o) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, o), rs,
                                         (int)(gv * 16), 0, kStoreAux);
}
template <typename T, int VEC>
struct RowIO;
template <>
struct RowIO<uint16_t, 8> {
  static __device__ __forceinline__ void load(const uint16_t* row, int64_t gv, float (&x)[8]) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row) + gv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = bf_lo(v[j]);
      x[2 * j + 1] = bf_hi(v[j]);
    }
  }
  static __device__ __forceinline__ void store(uint16_t* row, int64_t gv, const float (&d)[8]) {
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(d[2 * j], d[2 * j + 1]);
    store_row16(row, gv, o);
  }
};
template <>
struct RowIO<float, 4> {
  static __device__ __forceinline__ void load(const float* row, int64_t gv, float (&x)[4]) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row) + gv);
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = v[j];
  }
  static __device__ __forceinline__ void store(float* row, int64_t gv, const float (&d)[4]) {
    f32x4 o = {d[0], d[1], d[2], d[3]};
    store_row16(row, gv, __builtin_bit_cast(u32x4, o));
  }
};
template <>
struct RowIO<uint16_t, 1> {
  static __device__ __forceinline__ void load(const uint16_t* row, int64_t gv, float (&x)[1]) { x[0] = bf_to_f(row[gv]); }
  static __device__ __forceinline__ void store(uint16_t* row, int64_t gv, const float (&d)[1]) { row[gv] = f_to_bf(d[0]); }
};
template <>
struct RowIO<float, 1> {
  static __device__ __forceinline__ void load(const float* row, int64_t gv, float (&x)[1]) { x[0] = row[gv]; }
  static __device__ __forceinline__ void store(float* row, int64_t gv, const float (&d)[1]) { row[gv] = d[0]; }
};


// gradient of one vector: d_j = p_j (alpha + beta t_j) (+ gadd at the target column)
template <int VEC>
__device__ __forceinline__ void grad_vec(const float (&x)[VEC], float (&d)[VEC], float c, float M,
                                         float l2s, float alpha, float beta, int64_t base, int64_t tgt,
                                         float gadd) {
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const float t = __builtin_fmaf(x[j] - M, c, -l2s);
    d[j] = fexp2(t) * __builtin_fmaf(beta, t, alpha);
    if (base + j == tgt) d[j] += gadd;
  }
}

#ifndef PRL_STREAM_F32_U
#define PRL_STREAM_F32_U 4
#endif
#ifndef PRL_STREAM_F32_WG_PER_CU
#define PRL_STREAM_F32_WG_PER_CU 1
#endif
// BLOCK threads per row, U vectors per thread in flight per loop step.  The fp32 form (rows of
// 594 KiB do not fit the register file) runs 1024-thread workgroups, one per CU, 4 vectors per
// thread: 64 KiB of loads in flight per CU, and only ~#CUs rows (~150 MB) between a row's first
// read and its re-read, so the gradient pass's re-read is served by the 256 MiB Infinity Cache.
template <typename T, int VEC, int BLOCK = 256, int U = 1>
__global__ __launch_bounds__(BLOCK) void grpo_fwd_stream(KArgs a) {
  constexpr int NW = BLOCK / 64;
  __shared__ float red[2][NW][3];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t nrows = fwd_rows(a);
  const int64_t nvec = a.V / VEC;
  const float c = kLog2e / a.temperature;
  const float inv_t = 1.0f / a.temperature;
  const T* lg = static_cast<const T*>(a.logits);
  T* dl = static_cast<T*>(a.dlogits);
  int par = 0;
  for (int64_t i = blockIdx.x; i < nrows; i += gridDim.x, par ^= 1) {
    int64_t lrow, tok, q;
    map_row<RowLd>(a, i, lrow, tok, q);
    const T* row = lg + lrow * a.ld;
    const int64_t tid_raw = RowLd::ld(a.input_ids, tok);
    const TokIn tin = tok_in<RowLd>(a, tok);
    const bool bad_id = (uint64_t)tid_raw >= (uint64_t)a.V;
    const int64_t tgt = bad_id ? -1 : tid_raw;
    const float xr = row_logit(row, bad_id ? 0 : tid_raw);
    const float xt = bad_id ? __builtin_nanf("") : xr;
    Lse st = lse_empty();
    int64_t gv = tid;
    for (; gv + (U - 1) * BLOCK < nvec; gv += U * BLOCK) {
      float x[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) RowIO<T, VEC>::load(row, gv + u * BLOCK, x[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) lse_add<VEC>(st, x[u], c);
    }
    for (; gv < nvec; gv += BLOCK) {
      float x[VEC];
      RowIO<T, VEC>::load(row, gv, x);
      lse_add<VEC>(st, x, c);
    }
    st = wave_reduce_lse(st, c);
    if (lane == 0) {
      red[par][wid][0] = st.m;
      red[par][wid][1] = st.s;
      red[par][wid][2] = st.w;
    }
    __syncthreads();
    const Lse tot = block_combine<NW>(red[par], c);
    const float l2s = log2f(tot.s);
    const float M = tot.m;
    const float lse = M * inv_t + kLn2 * l2s;
    const float H = kLn2 * (l2s - tot.w / tot.s);
    const float lp = (xt - M) * inv_t - kLn2 * l2s;
    const TokGrad core = row_epilogue(a, q, tin, lp, H, lse, M, l2s, tid == 0);
    if (a.write_grad) {
      T* drow = dl + lrow * a.ld;
      const float alpha = -(core.g_lp + core.g_h * H) * inv_t;
      const float beta = -core.g_h * kLn2 * inv_t;
      const float gadd = core.g_lp * inv_t;
      const bool zero_row = (core.g_lp == 0.f && core.g_h == 0.f);
      int64_t g2 = tid;
      for (; g2 + (U - 1) * BLOCK < nvec; g2 += U * BLOCK) {
        float d[U][VEC];
        if (zero_row) {
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < VEC; ++j) d[u][j] = 0.f;
        } else {
          float x[U][VEC];
#pragma unroll
          for (int u = 0; u < U; ++u) RowIO<T, VEC>::load(row, g2 + u * BLOCK, x[u]);
#pragma unroll
          for (int u = 0; u < U; ++u)
            grad_vec<VEC>(x[u], d[u], c, M, l2s, alpha, beta, (g2 + u * BLOCK) * VEC, tgt, gadd);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) RowIO<T, VEC>::store(drow, g2 + u * BLOCK, d[u]);
      }
      for (; g2 < nvec; g2 += BLOCK) {
        float d[VEC];
        if (zero_row) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) d[j] = 0.f;
        } else {
          float x[VEC];
          RowIO<T, VEC>::load(row, g2, x);
          grad_vec<VEC>(x, d, c, M, l2s, alpha, beta, g2 * VEC, tgt, gadd);
        }
        RowIO<T, VEC>::store(drow, g2, d);
      }
    }
  }
}

// fp32 rows (Accelerate's mixed precision upcasts the logits, finetune_loop.py:381-385): a row
// (594 KiB at V = 151 936) does not fit one CU's registers, and grpo_fwd_stream's gradient pass
// re-reads it — from HBM, mostly: 74.0 GB fetched per C2 launch for 39.8 GB of logits
// (profiles/r04_fp32_pmc.json).  This kernel keeps NR vectors per lane in registers and NL in LDS
// (NL x 16 KiB of the CU's 160 KiB; 75 % of a Qwen2.5 row at NR = 19, NL = 9) and re-reads only the
// tail.  Each lane writes and reads only its own LDS slots, so the slab needs no barrier; one
// workgroup per CU (the slab), rows strided over the grid as grpo_fwd_stream.
#ifndef PRL_HYB_NR
#define PRL_HYB_NR 19
#endif
#ifndef PRL_HYB_NL
#define PRL_HYB_NL 9
#endif
#ifndef PRL_HYB_U1
#define PRL_HYB_U1 2
#endif
constexpr int kHybNR = PRL_HYB_NR, kHybNL = PRL_HYB_NL;
typedef __attribute__((address_space(3))) void lds_void_t;
// d = p (alpha + beta t) (+ gadd at the target column) of one fp32 vector, stored at voff + soff of
// the dlogits row.  ``hit``: this lane's vector holds the target, at element ``jt`` (uniform).  The
// offsets come as one per-lane VGPR plus a wave-uniform SGPR, and the target test as a row-uniform
// vector index against a per-row lane flag (target_lane): per-vector lane addresses — or a
// per-vector ``lane column + k * 4096`` to compare the target with — are loop invariants the
// compiler hoists out of the row loop, one VGPR per resident vector (what spilled the first version,
// and, as 18 reloads per row from scratch, the round-5 pair kernel: ~9 GB of extra reads per C2
// launch).  The store is store_row_b128 (fenced: SGPR soffset, see its comment).
__device__ __forceinline__ void hyb_store(__amdgpu_buffer_rsrc_t ws, int voff, int soff, bool hit, int jt, f32x4 x,
                                         bool zero_row, float c, float M, float l2s, float alpha, float beta,
                                         float gadd) {
  f32x4 d = {0.f, 0.f, 0.f, 0.f};
  if (!zero_row) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = __builtin_fmaf(x[j] - M, c, -l2s);
      d[j] = fexp2(t) * __builtin_fmaf(beta, t, alpha);
      if (hit && j == jt) d[j] += gadd;
    }
  }
  store_row_b128(__builtin_bit_cast(u32x4, d), ws, voff, soff);
}
// A row's target relative to a resident block's first column, trel (uniform; < 0: none): it sits in
// the block's vector trel >> 12 (1024 lanes x 4 columns), lane (trel >> 2) & 1023, element trel & 3.
struct TargetPos {
  int kt;     // vector index (negative: none)
  int jt;     // element
  bool lane;  // this lane owns it
};
__device__ __forceinline__ TargetPos target_pos(int trel, int tid) {
  TargetPos t;
  t.kt = trel < 0 ? -1 : (trel >> 12);
  t.jt = trel & 3;
  t.lane = ((trel >> 2) & 1023) == tid;
  return t;
}
template <int NR, int NL>
__global__ __launch_bounds__(1024) void grpo_fwd_hybrid_f32(KArgs a) {
  constexpr int BLOCK = 1024, NW = BLOCK / 64, U = 4;  // pass 2's tail vectors in flight
  constexpr int U1 = PRL_HYB_U1;  // the tail's vectors in flight in pass 1, beside the NR resident ones
  constexpr int VSTRIDE = BLOCK * 16;  // bytes between a lane's consecutive vectors
  __shared__ f32x4 slab[NL > 0 ? NL : 1][BLOCK];
  __shared__ float red[2][NW][3];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t nrows = fwd_rows(a);
  const int nvec = (int)(a.V >> 2);  // the host guarantees nvec >= (NR + NL) * BLOCK
  const float c = kLog2e / a.temperature;
  const float inv_t = 1.0f / a.temperature;
  const float* lg = static_cast<const float*>(a.logits);
  float* dl = static_cast<float*>(a.dlogits);
  const int voff = tid * 16;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  f32x4 buf[NR];
  // a row's resident part: the LDS share by LDS-DMA (no registers: wave w's 64 lanes fill
  // slab[k][64 w ..], 1 KiB per instruction), then the register share
  auto load_resident = [&](const __amdgpu_buffer_rsrc_t& r) {
#pragma unroll
    for (int k = 0; k < NL; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(&slab[k][wu * 64]), 16, voff, (NR + k) * VSTRIDE, 0,
                                               kLoadAux);
#pragma unroll
    for (int k = 0; k < NR; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, k * VSTRIDE, kLoadAux));
  };
  auto row_of_iter = [&](int64_t it) {
    int64_t lr, tk, qq;
    map_row<RowLd>(a, it, lr, tk, qq);
    return row_rsrc(lg + lr * a.ld, a.V * 4);
  };
  if (blockIdx.x < nrows) load_resident(row_of_iter(blockIdx.x));
  int par = 0;
  for (int64_t i = blockIdx.x; i < nrows; i += gridDim.x, par ^= 1) {
    int64_t lrow, tok, q;
    map_row<RowLd>(a, i, lrow, tok, q);
    const float* row = lg + lrow * a.ld;
    const auto rs = row_rsrc(row, a.V * 4);
    const bool has_next = i + gridDim.x < nrows;
    const int64_t tid_raw = RowLd::ld(a.input_ids, tok);
    const TokIn tin = tok_in<RowLd>(a, tok);
    const bool bad_id = (uint64_t)tid_raw >= (uint64_t)a.V;
    const int tgt = bad_id ? -1 : (int)tid_raw;
    const float xr = row_logit(row, bad_id ? 0 : tid_raw);
    const float xt = bad_id ? __builtin_nanf("") : xr;
    Lse st = lse_empty();
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const float x[4] = {buf[k][0], buf[k][1], buf[k][2], buf[k][3]};
      lse_add<4>(st, x, c);
    }
    // this lane's DMA pieces landed (issued before the register loads, which have all returned by
    // now; the explicit wait also orders the LDS reads after the DMA for the compiler)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const f32x4 v = slab[k][tid];
      const float x[4] = {v[0], v[1], v[2], v[3]};
      lse_add<4>(st, x, c);
    }
    constexpr int kTail0 = (NR + NL) * BLOCK;
    int gv = kTail0 + tid;
    for (; gv + (U1 - 1) * BLOCK < nvec; gv += U1 * BLOCK) {
      float x[U1][4];
#pragma unroll
      for (int u = 0; u < U1; ++u) RowIO<float, 4>::load(row, gv + u * BLOCK, x[u]);
#pragma unroll
      for (int u = 0; u < U1; ++u) lse_add<4>(st, x[u], c);
    }
    for (; gv < nvec; gv += BLOCK) {
      float x[4];
      RowIO<float, 4>::load(row, gv, x);
      lse_add<4>(st, x, c);
    }
    st = wave_reduce_lse(st, c);
    if (lane == 0) {
      red[par][wid][0] = st.m;
      red[par][wid][1] = st.s;
      red[par][wid][2] = st.w;
    }
    __syncthreads();
    const Lse tot = block_combine<NW>(red[par], c);
    const float l2s = log2f(tot.s);
    const float M = tot.m;
    const float lse = M * inv_t + kLn2 * l2s;
    const float H = kLn2 * (l2s - tot.w / tot.s);
    const float lp = (xt - M) * inv_t - kLn2 * l2s;
    const TokGrad core = row_epilogue(a, q, tin, lp, H, lse, M, l2s, tid == 0);
    // opaque here, so nothing pass 1 derived from the row stays live into pass 2
#pragma unroll
    for (int k = 0; k < NR; ++k) asm volatile("" : "+v"(buf[k]));
    if (a.write_grad) {
      const auto ws = row_rsrc(dl + lrow * a.ld, a.V * 4);
      const float alpha = -(core.g_lp + core.g_h * H) * inv_t;
      const float beta = -core.g_h * kLn2 * inv_t;
      const float gadd = core.g_lp * inv_t;
      const bool zero_row = (core.g_lp == 0.f && core.g_h == 0.f);
      const TargetPos tp = target_pos(tgt, tid);
#pragma unroll
      for (int k = 0; k < NR; ++k)
        hyb_store(ws, voff, k * VSTRIDE, tp.lane && k == tp.kt, tp.jt, buf[k], zero_row, c, M, l2s, alpha, beta, gadd);
#pragma unroll
      for (int k = 0; k < NL; ++k)
        hyb_store(ws, voff, (NR + k) * VSTRIDE, tp.lane && NR + k == tp.kt, tp.jt, slab[k][tid], zero_row, c, M, l2s,
                  alpha, beta, gadd);
      const int vt = tgt < 0 ? -1 : (tgt >> 2);  // the target's vector (tail: per-lane compare)
      int g2 = kTail0 + tid;
      for (; g2 + (U - 1) * BLOCK < nvec; g2 += U * BLOCK) {
        f32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          x[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, g2 * 16, u * VSTRIDE, kLoadAux));
#pragma unroll
        for (int u = 0; u < U; ++u)
          hyb_store(ws, g2 * 16, u * VSTRIDE, g2 + u * BLOCK == vt, tp.jt, x[u], zero_row, c, M, l2s, alpha, beta,
                    gadd);
      }
      for (; g2 < nvec; g2 += BLOCK) {
        const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, g2 * 16, 0, kLoadAux));
        hyb_store(ws, g2 * 16, 0, g2 == vt, tp.jt, x, zero_row, c, M, l2s, alpha, beta, gadd);
      }
    }
    // the next row's DMA overwrites this lane's slab slots only after its own reads above (same
    // lane, program order: the LDS reads retire before the next row's DMA is issued)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (has_next) load_resident(row_of_iter(i + gridDim.x));
  }
}

// fp32 rows, fully resident: each row is split over a PAIR of workgroups (one per CU), each holding
// its half-row (297 KiB at V = 151 936: NV = 19 vectors per lane, as the bf16 kernel holds a whole
// bf16 row) in VGPRs, so no byte of the row is read twice.  The two halves exchange their partial
// (max, sum 2^y, sum 2^y y) once per row through a 16-B tagged granule in global memory — one sc1
// store of {m, s, w, tag} by one lane, sc1 polls by the partner's lane 0 (the data-tagged hand-off
// of MI355X_MICROARCH.md's price list, handoff-1to1) — and both combine the two partials in half
// order, so both hold bit-identical row statistics.  Pairs are blocks b and b ^ 8 (one XCD under the
// round-robin placement: speed only).
//
// Rows are claimed (round 6), so a pair whose CUs are held by another queue's kernel (an RCCL
// channel, a side-stream kernel) takes fewer rows instead of finishing a static share after everyone
// else: the LEADER (half 0) claims the pair's next row from a counter at the top of each row (its
// latency hides behind the row's loads) and publishes it in the pair's claim granule {row, 0, tag}
// right before its partial; the PARTNER loads that granule after the exchange and uses it after its
// gradient pass (by then it has landed), so the claim costs the pair no wait.  Every wait is
// bounded: a half whose partner has not published within PairArgs::spin_ticks of the realtime clock
// (100 MHz) goes SOLO for the rest of the launch — it computes the partner's partial from HBM (the
// same loads and arithmetic in the same order: the same bits), writes the partner half's gradient
// streamed from HBM too, claims its own rows, and marks its own partial slots with kSoloTag so a
// partner that arrives later goes SOLO at its next exchange instead of waiting.  A row two halves
// both finish is written twice with the same bits.  A pair that starts after the rows are claimed
// exits at its first claim.  Slots and the counter are zeroed by the host before each launch.
struct PairArgs {
  uint32_t* slots;      // [pairs] x kPairSlotStride: partials {m, s, w, tag} [2 halves][2 parities], claims {row lo, row hi, 0, tag} [2 parities]
  uint32_t* row_ctr;    // rows claimed so far
  int64_t slot_bytes;   // bytes of the slot array (its buffer descriptor's range)
  int64_t spin_ticks;   // realtime ticks a half waits for its partner before going SOLO
  uint32_t* fallbacks;  // rows whose other half a SOLO half streamed (one vector atomic each)
};
#ifndef PRL_PAIR_SPIN_TICKS
#define PRL_PAIR_SPIN_TICKS 20000  // 200 us
#endif
constexpr int kPairMinNV = 8, kPairMaxNV = 19;  // above 19 the registers spill (hybrid kernel there)
constexpr int kSc1 = 16;  // aux bit of buffer_load / buffer_store: sc1 (bypass the CU's L1; write through)
constexpr int kPairSlotStride = 96;
// The pair kernel visits rows in claim order: perm_row's 64-bit modulo kept two loop invariants
// (the row count as floats) and a loop-carried value in registers the kernel does not have, so
// they went to scratch and back every row (2.7 % extra writes; through perm_row 12.66 / 12.85 vs
// 13.05 / 13.30 ms per C2 launch, alternated on one box)
__device__ __forceinline__ int64_t pair_row(int64_t i, int64_t) { return i; }
constexpr uint32_t kSoloTag = 0xFFFFFFFFu;  // a partial slot's tag once its half went SOLO

__device__ __forceinline__ u32x4 load_slot(__amdgpu_buffer_rsrc_t slots, int off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(slots, off, 0, kSc1));
}
__device__ __forceinline__ void store_slot(__amdgpu_buffer_rsrc_t slots, int off, u32x4 g) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, g), slots,
                                         off, 0, kSc1);
}
// One lane: poll the granule at `off` (first look already in v) with sc1 loads until it carries
// `tag`, or kSoloTag, or a tag past `tag` (its writer is ahead), or spin_ticks of the realtime clock
// have passed (no wait when spin_ticks is 0).  The clock is read once per 8 polls (a tight clock loop
// delays other kernels' starts; flat_pack.hip paced_read_kernel), s_sleep between polls.
__device__ __forceinline__ u32x4 poll_slot(__amdgpu_buffer_rsrc_t slots, int off, uint32_t tag, int64_t spin_ticks,
                                           u32x4 v) {
  auto waiting = [&](const u32x4& x) { return x[3] != tag && x[3] != kSoloTag && (int32_t)(x[3] - tag) < 0; };
  if (waiting(v) && spin_ticks > 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool more = true;
    while (more) {
#pragma unroll 1
      for (int k = 0; k < 8 && waiting(v); ++k) {
        __builtin_amdgcn_s_sleep(2);
        asm volatile("" ::: "memory");  // a fresh load every turn
        v = load_slot(slots, off);
      }
      more = waiting(v) && (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks;
    }
  }
  return v;
}

// the (m, s, w) state of a half row: its NV vectors per lane from registers (FROM_REGS) or streamed
// from HBM in the same order, then the wave and block reductions.  The same code computes both, so a
// half's own partial and the one a SOLO half computes for its partner are the same bits.
template <int NV, bool FROM_REGS>
__device__ __forceinline__ Lse half_state(const f32x4 (&buf)[NV], __amdgpu_buffer_rsrc_t rs, int voff, bool last_ok,
                                          float c, float (*red)[3], int lane, int wid) {
  constexpr int BLOCK = 1024, NW = BLOCK / 64, VSTRIDE = BLOCK * 16;
  const f32x4 pad = {kEmptyMax, kEmptyMax, kEmptyMax, kEmptyMax};
  Lse st = lse_empty();
  if constexpr (FROM_REGS) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const f32x4 v = (k == NV - 1 && !last_ok) ? pad : buf[k];
      const float x[4] = {v[0], v[1], v[2], v[3]};
      lse_add<4>(st, x, c);
    }
  } else {
    constexpr int U = 2;  // few extra registers beside the resident half (this is the rare path)
#pragma unroll
    for (int k0 = 0; k0 < NV; k0 += U) {
      f32x4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k0 + u < NV) t[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (k0 + u) * VSTRIDE, kLoadAux));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u < NV) {
          const f32x4 v = (k0 + u == NV - 1 && !last_ok) ? pad : t[u];
          const float x[4] = {v[0], v[1], v[2], v[3]};
          lse_add<4>(st, x, c);
        }
      }
    }
  }
  st = wave_reduce_lse(st, c);
  if (lane == 0) {
    red[wid][0] = st.m;
    red[wid][1] = st.s;
    red[wid][2] = st.w;
  }
  __syncthreads();
  return block_combine<NW>(red, c);
}

// the same from the lane's byte offset voff = 16 x its thread index
__device__ __forceinline__ TargetPos target_pos_v(int trel, int voff) {
  TargetPos t;
  t.kt = trel < 0 ? -1 : (trel >> 12);
  t.jt = trel & 3;
  t.lane = ((trel << 2) & (1023 << 4)) == voff;
  return t;
}
// a SOLO half's gradient pass over the OTHER half of its row, streamed from HBM (rare path)
template <int NV>
__device__ __forceinline__ void half_grad_stream(__amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t ws, int voff,
                                                 TargetPos tp, bool zero_row, float c, float M, float l2s, float alpha, float beta,
                                                 float gadd) {
  constexpr int BLOCK = 1024, VSTRIDE = BLOCK * 16, U = 2;
#pragma unroll
  for (int k0 = 0; k0 < NV; k0 += U) {
    f32x4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u < NV) t[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (k0 + u) * VSTRIDE, kLoadAux));
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u < NV) hyb_store(ws, voff, (k0 + u) * VSTRIDE, tp.lane && k0 + u == tp.kt, tp.jt, t[u], zero_row, c, M, l2s,
                                 alpha, beta, gadd);
  }
}

template <int NV>
__global__ __launch_bounds__(1024) void grpo_fwd_pair_f32(KArgs a, PairArgs pa) {
  constexpr int BLOCK = 1024, NW = BLOCK / 64, VSTRIDE = BLOCK * 16;
  __shared__ float red[2][NW][3];
  __shared__ float red2[NW][3];   // the other half's partial, when this half computes it
  __shared__ uint32_t xch[2][4];  // the partner's published partial and whether it arrived
  __shared__ int64_t next_row[2]; // the row after this one (by parity)
  __shared__ int solo_sh;         // this half went SOLO
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x;
  const int h = (b >> 3) & 1;                          // which half of the row (0: the leader)
  const int64_t p = (int64_t)(b >> 4) * 8 + (b & 7);   // pair: blocks b and b ^ 8 (the host launches a multiple of 16)
  const int64_t nrows = fwd_rows(a);
  const int nvec = (int)(a.V >> 2);
  const int n0 = (nvec + 1) >> 1;                      // half 0: vectors [0, n0), half 1: [n0, nvec)
  const int nmine = h ? nvec - n0 : n0, npart = h ? n0 : nvec - n0;
  const int64_t off_mine = h ? (int64_t)n0 * 16 : 0, off_part = h ? 0 : (int64_t)n0 * 16;
  const int col0 = h ? n0 * 4 : 0, col0_part = h ? 0 : n0 * 4;  // first column of each half
  const float c = kLog2e / a.temperature;
  const float inv_t = 1.0f / a.temperature;
  const float* lg = static_cast<const float*>(a.logits);
  float* dl = static_cast<float*>(a.dlogits);
  const int voff = tid * 16;
  const bool last_ok = (NV - 1) * BLOCK + tid < nmine;  // only vector NV-1 can be partial
  const bool last_ok_part = (NV - 1) * BLOCK + tid < npart;
  const auto slots = __builtin_amdgcn_make_buffer_rsrc(pa.slots, 0, (int)pa.slot_bytes, 0x00020000);
  const int pbase = (int)p * kPairSlotStride;
  auto part_off = [&](int half, int par) { return pbase + (half * 2 + par) * 16; };
  auto claim_off = [&](int par) { return pbase + 64 + par * 16; };
  f32x4 buf[NV];
  auto half_rsrc = [&](int64_t lrow, int64_t off, int n) {
    return row_rsrc(reinterpret_cast<const char*>(lg + lrow * a.ld) + off, (int64_t)n * 16);
  };
  auto load_half = [&](int64_t row) {
    int64_t lrow, tok, qo;
    map_row<RowLd>(a, pair_row(row, nrows), lrow, tok, qo);
    const auto rs = half_rsrc(lrow, off_mine, nmine);
#pragma unroll
    for (int k = 0; k < NV; ++k)
      buf[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * VSTRIDE, kLoadAux));
  };
  // lane 0 of a half going SOLO: mark both of its partial slots so the partner stops waiting on it
  auto mark_solo = [&]() {
    const u32x4 g = {0u, 0u, 0u, kSoloTag};
    store_slot(slots, part_off(h, 0), g);
    store_slot(slots, part_off(h, 1), g);
  };
  auto uniform64 = [](int64_t v) {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v));
  };

  // ---- the first row: the leader claims it, the partner follows (or goes SOLO after spin_ticks)
  if (tid == 0) {
    int solo = 0;
    int64_t r;
    if (h == 0) {
      r = (int64_t)atomicAdd(pa.row_ctr, 1u);
      store_slot(slots, claim_off(0), u32x4{(uint32_t)r, (uint32_t)(r >> 32), 0u, 1u});
    } else {
      const u32x4 v = poll_slot(slots, claim_off(0), 1u, pa.spin_ticks, load_slot(slots, claim_off(0)));
      if (v[3] == 1u) {
        r = (int64_t)(((uint64_t)v[1] << 32) | v[0]);
      } else {
        solo = 1;
        mark_solo();
        r = (int64_t)atomicAdd(pa.row_ctr, 1u);
      }
    }
    next_row[1] = r;
    solo_sh = solo;
  }
  __syncthreads();
  int64_t i = uniform64(next_row[1]);
  bool solo = __builtin_amdgcn_readfirstlane(solo_sh) != 0;
  if (i < nrows) load_half(i);
  for (uint32_t it = 0; i < nrows; ++it) {
    const int par = (int)(it & 1);
    const uint32_t tag = it + 1;
    // this lane's identity, opaque per row: what derives from it (wave, lane, lane-0 flag, the
    // target test) is recomputed here instead of hoisted out of the loop into registers the kernel
    // does not have (they went to scratch and back every row)
    int vo = voff;
    asm volatile("" : "+v"(vo));
    const int lane_r = (vo >> 4) & 63, wid_r = vo >> 10;
    const bool t0 = vo == 0;
    // the next row's claim (leader or SOLO): one vector atomic, its latency behind the row's loads
    uint32_t claim = 0;
    if (t0 && (h == 0 || solo)) claim = atomicAdd(pa.row_ctr, 1u);
    int64_t lrow, tok, qo;
    map_row<RowLd>(a, pair_row(i, nrows), lrow, tok, qo);
    const int64_t tid_raw = RowLd::ld(a.input_ids, tok);
    TokIn tin = tok_in<RowLd>(a, tok);
    const bool bad_id = (uint64_t)tid_raw >= (uint64_t)a.V;
    const int64_t tgt = bad_id ? -1 : tid_raw;
    float xr = row_logit(lg + lrow * a.ld, bad_id ? 0 : tid_raw);
    pin_sgpr(tin, xr);
    const float xt = bad_id ? __builtin_nanf("") : xr;

    // ---- pass 1: this half's state from registers, published for the partner (with the claim)
    const Lse mine = half_state<NV, true>(buf, slots, voff, last_ok, c, red[par], lane_r, wid_r);  // (rsrc unused)
    if (t0) {
      int arrived = 0;
      if (!solo) {
        if (h == 0) store_slot(slots, claim_off(par ^ 1), u32x4{claim, 0u, 0u, tag + 1});
        store_slot(slots, part_off(h, par), u32x4{__float_as_uint(mine.m), __float_as_uint(mine.s), __float_as_uint(mine.w), tag});
        const u32x4 v = poll_slot(slots, part_off(h ^ 1, par), tag, pa.spin_ticks, load_slot(slots, part_off(h ^ 1, par)));
        arrived = v[3] == tag;
        xch[par][0] = v[0];
        xch[par][1] = v[1];
        xch[par][2] = v[2];
        if (!arrived) mark_solo();  // the partner is late or SOLO: this half goes SOLO
      }
      xch[par][3] = (uint32_t)arrived;
      if (h == 0 || solo) next_row[par] = (int64_t)claim;  // (a partner that just went SOLO claims after pass 2)
    }
    __syncthreads();
    const bool paired = __builtin_amdgcn_readfirstlane((int)xch[par][3]) != 0;
    const bool was_solo = solo;
    solo = !paired;
    Lse part;
    if (paired) {
      part = Lse{__uint_as_float(xch[par][0]), __uint_as_float(xch[par][1]), __uint_as_float(xch[par][2])};
    } else {  // SOLO: the other half's partial from HBM (block-uniform branch)
      part = half_state<NV, false>(buf, half_rsrc(lrow, off_part, npart), voff, last_ok_part, c, red2, lane_r, wid_r);
      if (t0) atomicAdd(pa.fallbacks, 1u);
    }
    const Lse tot = h == 0 ? lse_combine(mine, part, c) : lse_combine(part, mine, c);
    const float l2s = log2f(tot.s);
    const float M = tot.m;
    const float lse = M * inv_t + kLn2 * l2s;
    const float H = kLn2 * (l2s - tot.w / tot.s);
    const float lp = (xt - M) * inv_t - kLn2 * l2s;
    const TokGrad core = row_epilogue(a, qo, tin, lp, H, lse, M, l2s, (h == 0 || solo) && t0);
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(buf[k]));

    // ---- pass 2: this half's gradient from registers (SOLO: the other half's streamed), then the
    // next row (stores retired) — the partner learns it from the claim granule, loaded behind its
    // stores (the load's latency hides in their drain; nothing holds it through the pass)
    if (a.write_grad) {
      const auto ws = row_rsrc(reinterpret_cast<char*>(dl + lrow * a.ld) + off_mine, (int64_t)nmine * 16);
      const float alpha = -(core.g_lp + core.g_h * H) * inv_t;
      const float beta = -core.g_h * kLn2 * inv_t;
      const float gadd = core.g_lp * inv_t;
      const bool zero_row = (core.g_lp == 0.f && core.g_h == 0.f);
      const TargetPos tp = target_pos_v((int)(tgt < 0 ? -1 : tgt - col0), vo);  // (other half: trel < 0)
#pragma unroll
      for (int k = 0; k < NV; ++k)
        hyb_store(ws, voff, k * VSTRIDE, tp.lane && k == tp.kt, tp.jt, buf[k], zero_row, c, M, l2s, alpha, beta, gadd);
      if (solo) {
        const auto wo = row_rsrc(reinterpret_cast<char*>(dl + lrow * a.ld) + off_part, (int64_t)npart * 16);
        const TargetPos tq = target_pos_v((int)(tgt < 0 ? -1 : tgt - col0_part), vo);
        half_grad_stream<NV>(half_rsrc(lrow, off_part, npart), wo, voff, tq, zero_row, c, M, l2s, alpha, beta, gadd);
      }
    }
    const bool follow = h == 1 && !was_solo;  // the partner (block-uniform): its next row from the claim granule
    u32x4 cv = {0u, 0u, 0u, 0u};
    if (follow && !solo && t0) cv = load_slot(slots, claim_off(par ^ 1));
    if (a.write_grad) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (follow) {
      if (t0) {
        int64_t r;
        const u32x4 v = solo ? cv : poll_slot(slots, claim_off(par ^ 1), tag + 1, pa.spin_ticks, cv);
        if (!solo && v[3] == tag + 1) {
          r = (int64_t)(((uint64_t)v[1] << 32) | v[0]);
        } else {
          if (!solo) mark_solo();
          solo_sh = 1;
          r = (int64_t)atomicAdd(pa.row_ctr, 1u);
        }
        next_row[par] = r;
        if (solo) solo_sh = 1;  // (redundant, but without it the allocator spills a row vector: checked in the ISA)
      }
      __syncthreads();
      solo = solo || __builtin_amdgcn_readfirstlane(solo_sh) != 0;
    }
    i = uniform64(next_row[par]);
    if (i < nrows) load_half(i);
  }
}

// gradient pass from saved per-row coefficients for the upstream gradient *up (device);
// skip_if_one: dlogits already holds the gradient for *up == grad_scale (fused forward)
template <typename T, int VEC>
__global__ __launch_bounds__(256) void grpo_bwd_stream(KArgs a, const float* max_in, const float* l2s_in,
                                                       const float* ent_in, const float* glp_in,
                                                       const float* gh_in, const float* up,
                                                       int skip_if_one) {
  constexpr int BLOCK = 256;
  // g_lp / g_h were saved at a.gscale (the loss scale the forward assumed): the upstream
  // gradient is applied relative to it, and an upstream equal to it needs no pass at all
  const float up_abs = up ? *up : 1.0f;
  if (skip_if_one && up_abs == a.gscale) return;
  const float scale = up_abs / a.gscale;
  const int tid = threadIdx.x;
  const int64_t nrows = a.B * (a.L - 1);
  const int64_t nvec = a.V / VEC;
  const float c = kLog2e / a.temperature;
  const float inv_t = 1.0f / a.temperature;
  const T* lg = static_cast<const T*>(a.logits);
  T* dl = static_cast<T*>(a.dlogits);
  for (int64_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    int64_t lrow, tok;
    row_of(a, q, lrow, tok);
    const T* row = lg + lrow * a.ld;
    T* drow = dl + lrow * a.ld;
    const int64_t tid_raw = a.input_ids[tok];
    const int64_t tgt = (uint64_t)tid_raw >= (uint64_t)a.V ? -1 : tid_raw;
    const float g_lp = glp_in[q] * scale, g_h = gh_in[q] * scale;
    const float H = ent_in[q];
    const float M = max_in[q], l2s = l2s_in[q];
    const float alpha = -(g_lp + g_h * H) * inv_t;
    const float beta = -g_h * kLn2 * inv_t;
    const float gadd = g_lp * inv_t;
    const bool zero_row = (g_lp == 0.f && g_h == 0.f);
    for (int64_t gv = tid; gv < nvec; gv += BLOCK) {
      float d[VEC];
      if (zero_row) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) d[j] = 0.f;
      } else {
        float x[VEC];
        RowIO<T, VEC>::load(row, gv, x);
        grad_vec<VEC>(x, d, c, M, l2s, alpha, beta, gv * VEC, tgt, gadd);
      }
      RowIO<T, VEC>::store(drow, gv, d);
    }
  }
}

// Statistics (rl/__init__.py:315-375) and value-head gradient from the per-row outputs.
// Block b owns rows [b*chunk, (b+1)*chunk); each thread folds its rows in a fixed order,
// then the block folds threads in index order: deterministic for a given row count.
constexpr int kStatThreads = 64;  // one wave per block: no LDS, several blocks per CU
__global__ __launch_bounds__(kStatThreads) void grpo_stats_partial(KArgs a, int64_t chunk) {
  const int tid = threadIdx.x;
  const int64_t nrows = a.B * (a.L - 1);
  double acc[PRL_NSTAT];
#pragma unroll
  for (int i = 0; i < PRL_NSTAT; ++i) acc[i] = stat_identity(i);
  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  const int64_t r1 = r0 + chunk < nrows ? r0 + chunk : nrows;
  const bool has_v = a.values != nullptr;
  for (int64_t q = r0 + tid; q < r1; q += kStatThreads) {
    int64_t lrow, tok;
    row_of(a, q, lrow, tok);
    const float lp = a.o_lp[q], H = a.o_ent[q];
    const TokVals v = token_values(a, tok, lp, H);
    const bool m = v.m;
    const float reward = a.rewards[tok], ref = a.ref_lp[tok], old = a.old_lp[tok];
    const float nl = a.num_labels[tok];
    const int64_t tidv = a.input_ids[tok];
    const float vp = has_v ? a.values[tok - 1] : 0.f;
    float vl = 0.f;
    if (has_v) {
      const float dvr = vp - reward;
      vl = 0.5f * (dvr * dvr) * v.w;  // :304
      a.o_dv[tok - 1] = (m && __builtin_isfinite(vl)) ? a.gscale * a.value_coef * v.w * dvr : 0.f;
    }
    const float C = a.clampC;
    float c[PRL_NSTAT];
    // masked sums: rl/utils.py mask_sum -> m ? nan_to_num(v) : 0  (v / nl order kept)
    c[PRL_S_LOSS_SUM] = m ? nz(v.tl) : 0.f;
    c[PRL_S_VALUE_LOSS] = m ? nz(vl) : 0.f;
    c[PRL_S_REWARD] = m ? nz(reward / nl) : 0.f;
    c[PRL_S_ENTROPY] = m ? nz(H / nl) : 0.f;
    c[PRL_S_OLD_LP] = m ? nz(old / nl) : 0.f;
    c[PRL_S_NEW_LP] = m ? nz(lp / nl) : 0.f;
    c[PRL_S_REF_LP] = m ? nz(ref / nl) : 0.f;
    c[PRL_S_ADVANTAGE] = m ? nz(v.adv / nl) : 0.f;
    c[PRL_S_KL] = m ? nz(v.kl / nl) : 0.f;
    c[PRL_S_POLICY_LOSS] = m ? nz(v.pol / nl) : 0.f;
    c[PRL_S_SURR1] = m ? nz(v.s1 / nl) : 0.f;
    c[PRL_S_SURR2] = m ? nz(v.s2 / nl) : 0.f;
    c[PRL_S_RATIO] = m ? nz(v.ratio_used / nl) : 0.f;
    c[PRL_S_RATIO_SUM] = m ? nz(v.ratio_used) : 0.f;
    c[PRL_S_RATIO_SQ_SUM] = m ? nz(v.ratio_used * v.ratio_used) : 0.f;
    c[PRL_S_RATIO_REF_NEW] = m ? nz(expf(v.lrrn) / nl) : 0.f;
    c[PRL_S_RATIO_REF_OLD] = m ? nz(expf(ref - old) / nl) : 0.f;
    c[PRL_S_CLAMP_REF_NEW] = m ? nz((fabsf(v.lrrn) > C ? 1.f : 0.f) / nl) : 0.f;  // :254
    c[PRL_S_CLAMP_NEW_OLD] = m ? nz((v.ind_no ? 1.f : 0.f) / nl) : 0.f;
    c[PRL_S_TOKEN_WEIGHT] = m ? nz(v.w / nl) : 0.f;
    c[PRL_S_VALUE_MEAN] = (m && has_v) ? nz(vp / nl) : 0.f;
    c[PRL_S_VALUE_MSE] = (m && has_v) ? nz(((vp - reward) * (vp - reward)) / nl) : 0.f;
    c[PRL_S_NUM_NANS] = (v.tl != v.tl) ? 1.f : 0.f;
    c[PRL_S_NUM_OUT] = m ? 1.f : 0.f;
    c[PRL_S_BAD_LP] = __builtin_isfinite(lp) ? 0.f : 1.f;
    c[PRL_S_BAD_LRRN] = __builtin_isfinite(v.lrrn) ? 0.f : 1.f;
    c[PRL_S_BAD_KL] = __builtin_isfinite(v.kl) ? 0.f : 1.f;
    c[PRL_S_BAD_GT] = (a.group_norm && !(a.group_tokens[tok] > 0.f)) ? 1.f : 0.f;
    c[PRL_S_BAD_ID] = ((uint64_t)tidv >= (uint64_t)a.V) ? 1.f : 0.f;
    const float ninf = -__builtin_inff(), pinf = __builtin_inff();
    c[PRL_S_MAX_REWARD] = m ? reward : ninf;
    c[PRL_S_MIN_REWARD] = m ? reward : pinf;
    c[PRL_S_MAX_ADV] = m ? v.adv : ninf;
    c[PRL_S_MIN_ADV] = m ? v.adv : pinf;
    c[PRL_S_MAX_KL] = m ? v.kl : ninf;
    c[PRL_S_MIN_KL] = m ? v.kl : pinf;
    c[PRL_S_MAX_W] = m ? v.w : ninf;
    c[PRL_S_MIN_W] = m ? v.w : pinf;
    c[PRL_S_MAX_VALUE] = (m && has_v) ? vp : ninf;
    c[PRL_S_MIN_VALUE] = (m && has_v) ? vp : pinf;
#pragma unroll
    for (int i = 0; i < PRL_NSTAT; ++i) acc[i] = stat_fold(i, acc[i], (double)c[i]);
  }
  // block (= wave) fold per statistic: a fixed xor tree across the lanes — deterministic (both
  // partners of a tree step compute the same commutative fold).  Was 256-thread blocks folded by
  // one thread per statistic walking all 256 threads serially: 93 us per launch at C2, now ~10x less.
  // fully unrolled so acc[] stays in registers (a dynamic index would put it in scratch)
  static_assert(PRL_NSTAT == 39, "unroll count below");
#pragma unroll 39
  for (int i = 0; i < PRL_NSTAT; ++i) {
    double r = acc[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r = stat_fold(i, r, __shfl_xor(r, o, 64));
    if (tid == 0) a.partials[(int64_t)i * gridDim.x + blockIdx.x] = r;  // stat-major: finalize reads coalesced
  }
}

// Fold the per-block partials (stat-major, partials[i * nblocks + b]): one workgroup per
// statistic; thread t folds blocks t, t + 256, ... in order (4 loads in flight), each wave folds
// its lanes with a fixed xor tree, then thread 0 folds the 4 waves in index order: deterministic
// for a given block count.  One launch latency for all 39 statistics (was one 1024-thread
// workgroup looping over them: 11-28 us).
constexpr int kFinThreads = 256;
__global__ __launch_bounds__(kFinThreads) void grpo_finalize(const double* __restrict__ partials, int nblocks,
                                                             double* __restrict__ stats) {
  __shared__ double wsum[kFinThreads / 64];
  const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const double* p = partials + (int64_t)i * nblocks;
  double acc = stat_identity(i);
  for (int b0 = 0; b0 < nblocks; b0 += kFinThreads * 4) {
    double v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = b0 + t + kFinThreads * k;
      v[k] = b < nblocks ? p[b] : stat_identity(i);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = stat_fold(i, acc, v[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc = stat_fold(i, acc, __shfl_xor(acc, o, 64));
  if (lane == 0) wsum[wid] = acc;
  __syncthreads();
  if (t == 0) {
    double r = wsum[0];
#pragma unroll
    for (int w = 1; w < kFinThreads / 64; ++w) r = stat_fold(i, r, wsum[w]);
    stats[i] = r;
  }
}

// ---------------------------------------------------------------------------------------
// host side
struct DevInfo {
  int cus = 0;
};
static DevInfo g_dev[64];

static int device_cus(int dev) {
  if (dev < 0 || dev >= 64) return 256;
  if (g_dev[dev].cus == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    g_dev[dev].cus = n;
  }
  return g_dev[dev].cus;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static int fill_args(KArgs& a, const PrlGrpoBatch* b, const PrlGrpoParams* p, bool need_logits = true) {
  if (!b || !p) return PRL_E_INVALID;
  if (b->B < 1 || b->L < 1 || b->V < 1 || b->ld < b->V) return PRL_E_INVALID;
  if ((need_logits && !b->logits) || !b->input_ids || !b->labels || !b->rewards || !b->advantages || !b->ref_logprobs ||
      !b->old_logprobs || !b->group_tokens || !b->num_labels || !b->overflow)
    return PRL_E_INVALID;
  if (b->logits_dtype != PRL_BF16 && b->logits_dtype != PRL_F32) return PRL_E_UNSUPPORTED;
  if (p->policy_loss != PRL_PPO && p->policy_loss != PRL_REINFORCE) return PRL_E_INVALID;
  if (!(p->grad_scale > 0.f && p->grad_scale < 3.0e38f)) return PRL_E_INVALID;  // finite, positive
  a = KArgs{};
  a.logits = b->logits;
  a.B = b->B;
  a.L = b->L;
  a.V = b->V;
  a.ld = b->ld;
  a.input_ids = b->input_ids;
  a.labels = b->labels;
  a.rewards = b->rewards;
  a.advantages = b->advantages;
  a.ref_lp = b->ref_logprobs;
  a.old_lp = b->old_logprobs;
  a.group_tokens = b->group_tokens;
  a.num_labels = b->num_labels;
  a.overflow = b->overflow;
  a.values = b->values;
  a.policy = p->policy_loss;
  a.use_adv = p->use_advantages;
  a.relu = p->relu_log_p_weights;
  a.group_norm = p->group_normalization;
  a.overlong = p->overlong_filtering;
  a.write_grad = p->write_grad;
  a.eps = p->epsilon;
  a.kl_c = p->kl_coef;
  a.ent_c = p->entropy_coef;
  a.clampC = p->clamp_log_ratio;
  a.temperature = p->temperature;
  a.batch_size = p->batch_size;
  a.value_coef = p->value_loss_coef;
  a.gscale = p->grad_scale;
  return PRL_OK;
}

constexpr int kMaxNV = 24;
static int resident_nv(int64_t nvec) {
  const int64_t nv = (nvec + 1023) / 1024;
  return nv <= kMaxNV ? (int)nv : 0;
}

template <int NV>
static hipError_t launch_resident(const KArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(grpo_fwd_resident<NV>, dim3(grid), dim3(1024), 0, s, a);
  return hipGetLastError();
}

template <int... NVs>
static hipError_t launch_resident_table(int nv, const KArgs& a, int grid, hipStream_t s,
                                        std::integer_sequence<int, NVs...>) {
  hipError_t e = hipErrorInvalidValue;
  ((nv == NVs + 1 ? (e = launch_resident<NVs + 1>(a, grid, s), true) : false) || ...);
  return e;
}

static hipError_t launch_resident_nv(int nv, const KArgs& a, int grid, hipStream_t s) {
  return launch_resident_table(nv, a, grid, s, std::make_integer_sequence<int, kMaxNV>{});
}

// The caller's workspace (prl_grpo_workspace_bytes): the statistics' per-block partials, then the
// row kernels' scratch — the fp32 pair kernel's row counter (16 B) and hand-off slots
// (kPairSlotStride bytes per pair for up to 1024 CUs; both zeroed before each pair launch), its
// fallback counter (accumulated over launches;
// prl_grpo_pair_fallbacks reads and resets it) and the resident kernel's row counter (zeroed before
// each launch).  No library-held device memory: a workspace serves one stream at a time.
constexpr int kPairMaxCUs = 1024;
constexpr size_t kPartialsBytes = sizeof(double) * (size_t)kMaxGrid * PRL_NSTAT;
constexpr size_t kPairSlotBytes = 16 + (size_t)(kPairMaxCUs / 2) * kPairSlotStride;
constexpr size_t kPairCounterBytes = 16;
constexpr size_t kRowCounterBytes = 16;
constexpr size_t kWorkspaceBytes = kPartialsBytes + kPairSlotBytes + kPairCounterBytes + kRowCounterBytes;

struct Scratch {
  uint32_t* slots;      // pair hand-off slots
  uint32_t* fallbacks;  // pair fallback counter
  uint32_t* row_ctr;    // resident kernel's row counter
};
static Scratch scratch_of(void* ws) {
  char* p = static_cast<char*>(ws) + kPartialsBytes;
  return Scratch{reinterpret_cast<uint32_t*>(p), reinterpret_cast<uint32_t*>(p + kPairSlotBytes),
                 reinterpret_cast<uint32_t*>(p + kPairSlotBytes + kPairCounterBytes)};
}

// the device a stream belongs to (the null stream: the current device)
static int stream_device(hipStream_t s) {
  int dev = 0;
  if (s == nullptr || hipStreamGetDevice(s, &dev) != hipSuccess) (void)hipGetDevice(&dev);
  return dev;
}

// the fp32 pair kernel's partner wait (PrlGrpoParams.pair_spin_ticks: 0 = the default, < 0 = none)
static int64_t pair_spin_ticks(const PrlGrpoParams* p) {
  return p->pair_spin_ticks == 0 ? (int64_t)PRL_PAIR_SPIN_TICKS : (p->pair_spin_ticks < 0 ? 0 : p->pair_spin_ticks);
}

template <int NV>
static hipError_t launch_pair(const KArgs& a, const PairArgs& pa, int grid, hipStream_t s) {
  hipLaunchKernelGGL(grpo_fwd_pair_f32<NV>, dim3(grid), dim3(1024), 0, s, a, pa);
  return hipGetLastError();
}
template <int... NVs>
static hipError_t launch_pair_table(int nv, const KArgs& a, const PairArgs& pa, int grid, hipStream_t s,
                                    std::integer_sequence<int, NVs...>) {
  hipError_t e = hipErrorInvalidValue;
  ((nv == NVs + kPairMinNV ? (e = launch_pair<NVs + kPairMinNV>(a, pa, grid, s), true) : false) || ...);
  return e;
}

// fp32 rows of 16-B vectors whose halves fit NV in [kPairMinNV, kPairMaxNV] vectors per lane: the
// pair kernel over min(#CUs, pairs needed) blocks, rounded down to a multiple of 16 (pairs b, b ^ 8)
static int pair_nv(int64_t V) {
  const int64_t half = ((V >> 2) + 1) >> 1;
  const int64_t nv = (half + 1023) / 1024;
  return (nv >= kPairMinNV && nv <= kPairMaxNV) ? (int)nv : 0;
}
static hipError_t launch_pair_rows(const KArgs& a, int nv, int64_t nrows, int cus, const Scratch& sc,
                                   int64_t spin_ticks, hipStream_t s) {
  int grid = cus < kPairMaxCUs ? cus : kPairMaxCUs;
  const int64_t need = 2 * nrows;
  if (need < grid) grid = (int)need;
  grid = (grid + 15) / 16 * 16;
  if (grid > cus) grid = cus / 16 * 16;
  if (grid < 16) grid = 16;
  PairArgs pa{};
  pa.row_ctr = sc.slots;
  pa.slots = sc.slots + 4;
  pa.slot_bytes = (int64_t)(kPairSlotBytes - 16);
  pa.spin_ticks = spin_ticks;
  pa.fallbacks = sc.fallbacks;
  // the counter and the launch's pairs' slots (tags restart at 1)
  const hipError_t e = hipMemsetAsync(sc.slots, 0, 16 + (size_t)(grid / 2) * kPairSlotStride, s);
  if (e != hipSuccess) return e;
  return launch_pair_table(nv, a, pa, grid, s, std::make_integer_sequence<int, kPairMaxNV - kPairMinNV + 1>{});
}

// the resident kernel's rows claimed from the workspace's counter (zeroed here, stream-ordered)
static hipError_t launch_resident_rows(KArgs a, int nv, int grid, const Scratch& sc, hipStream_t s) {
  a.row_ctr = sc.row_ctr;
  const hipError_t e = hipMemsetAsync(a.row_ctr, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
  return launch_resident_nv(nv, a, grid, s);
}

// per-row outputs (+ dlogits); the row arrays are indexed by batch row q
static int fill_outputs(KArgs& a, const PrlGrpoBatch* b, const PrlGrpoParams* p, const PrlGrpoOutputs* out,
                        bool need_stats) {
  if (!out || !out->new_logprobs || !out->entropy || !out->lse || !out->token_loss || !out->g_lp ||
      !out->g_h || !out->row_max || !out->row_log2sum || (need_stats && !out->stats))
    return PRL_E_INVALID;
  if (b->values && !out->dvalues) return PRL_E_INVALID;
  if (p->write_grad && !out->dlogits) return PRL_E_INVALID;
  a.o_lp = out->new_logprobs;
  a.o_ent = out->entropy;
  a.o_lse = out->lse;
  a.o_max = out->row_max;
  a.o_l2s = out->row_log2sum;
  a.o_tok = out->token_loss;
  a.o_glp = out->g_lp;
  a.o_gh = out->g_h;
  a.o_dv = out->dvalues;
  a.dlogits = out->dlogits;
  return PRL_OK;
}

// the vocab pass over `nrows` logits rows: register-resident kernel when a bf16 row fits,
// streaming kernels otherwise
static hipError_t launch_rows(const KArgs& a, const PrlGrpoBatch* b, const PrlGrpoParams* p,
                              const PrlGrpoOutputs* out, int64_t nrows, const Scratch& sc, hipStream_t s) {
  if (nrows <= 0) return hipSuccess;
  const int cus = device_cus(stream_device(s));
  const bool bf16 = b->logits_dtype == PRL_BF16;
  const bool vec_ok_bf = bf16 && b->V % 8 == 0 && b->ld % 8 == 0 && aligned16(b->logits) &&
                         (!p->write_grad || aligned16(out->dlogits));
  const int nv = vec_ok_bf ? resident_nv(b->V / 8) : 0;  // row <= 24*16 KiB
  if (nv > 0) return launch_resident_rows(a, nv, (int)(nrows < cus ? nrows : cus), sc, s);
  const int64_t want = (int64_t)cus * 4;
  int grid = (int)(nrows < want ? nrows : want);
  if (grid > kMaxGrid) grid = kMaxGrid;
  if (vec_ok_bf) {
    hipLaunchKernelGGL((grpo_fwd_stream<uint16_t, 8>), dim3(grid), dim3(256), 0, s, a);
  } else if (bf16) {
    hipLaunchKernelGGL((grpo_fwd_stream<uint16_t, 1>), dim3(grid), dim3(256), 0, s, a);
  } else if (b->V % 4 == 0 && b->ld % 4 == 0 && aligned16(b->logits) &&
             (!p->write_grad || aligned16(out->dlogits))) {
    const int pnv = p->f32_rows == 0 ? pair_nv(b->V) : 0;  // PrlGrpoParams.f32_rows 1: the part-resident kernel
    if (pnv > 0 && nrows < ((int64_t)1 << 31)) return launch_pair_rows(a, pnv, nrows, cus, sc, pair_spin_ticks(p), s);  // resident over two CUs
    if (PRL_HYB_NL >= 0 && b->V / 4 >= (int64_t)(kHybNR + kHybNL) * 1024) {  // a tail to stream: the row part-resident
      const int g1 = (int)(nrows < cus ? nrows : cus);  // one workgroup per CU (the LDS slab)
      hipLaunchKernelGGL((grpo_fwd_hybrid_f32<kHybNR, kHybNL>), dim3(g1), dim3(1024), 0, s, a);
      return hipGetLastError();
    }
    const int64_t want1 = (int64_t)cus * PRL_STREAM_F32_WG_PER_CU;  // 1024-thread workgroups
    const int g1 = (int)(nrows < want1 ? nrows : want1);
    hipLaunchKernelGGL((grpo_fwd_stream<float, 4, 1024, PRL_STREAM_F32_U>), dim3(g1), dim3(1024), 0, s, a);
  } else {
    hipLaunchKernelGGL((grpo_fwd_stream<float, 1>), dim3(grid), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

// statistics + value gradient over all batch rows: fixed row chunks per block (deterministic)
static hipError_t launch_stats(const KArgs& a, int64_t nrows, double* stats, hipStream_t s) {
  int sblocks = 0;
  if (nrows > 0) {
    // >= 64 rows per one-wave block (one row per thread at C2), at most kMaxGrid blocks
    int64_t chunk = (nrows + kMaxGrid - 1) / kMaxGrid;
    if (chunk < kStatThreads) chunk = kStatThreads;
    sblocks = (int)((nrows + chunk - 1) / chunk);
    hipLaunchKernelGGL(grpo_stats_partial, dim3(sblocks), dim3(kStatThreads), 0, s, a, chunk);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(grpo_finalize, dim3(PRL_NSTAT), dim3(kFinThreads), 0, s, a.partials, sblocks, stats);
  return hipGetLastError();
}

}  // namespace prl

using namespace prl;

extern "C" {

int prl_abi_version(void) { return PRL_ABI_VERSION; }

const char* prl_error_string(int code) {
  switch (code) {
    case PRL_OK: return "ok";
    case PRL_E_INVALID: return "invalid argument";
    case PRL_E_UNSUPPORTED: return "unsupported dtype or layout";
    case PRL_E_WORKSPACE: return "workspace too small";
    default: return hipGetErrorString(static_cast<hipError_t>(code));
  }
}

int prl_grpo_workspace_bytes(int device, size_t* bytes) {
  (void)device;
  if (!bytes) return PRL_E_INVALID;
  *bytes = kWorkspaceBytes;
  return PRL_OK;
}

int prl_grpo_forward(const PrlGrpoBatch* batch, const PrlGrpoParams* params,
                     const PrlGrpoOutputs* out, void* workspace, size_t workspace_bytes,
                     void* stream) {
  KArgs a;
  int rc = fill_args(a, batch, params);
  if (rc) return rc;
  rc = fill_outputs(a, batch, params, out, true);
  if (rc) return rc;
  if (!workspace || workspace_bytes < kWorkspaceBytes) return PRL_E_WORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  a.partials = static_cast<double*>(workspace);
  const size_t es = batch->logits_dtype == PRL_BF16 ? 2 : 4;
  hipError_t e;
  if (batch->values) {
    e = hipMemsetAsync(out->dvalues, 0, sizeof(float) * (size_t)(batch->B * batch->L), s);
    if (e != hipSuccess) return (int)e;
  }
  if (params->write_grad) {  // rows t = L-1 carry no loss: zero them (pitch = one sequence)
    char* last = static_cast<char*>(out->dlogits) + (size_t)(batch->L - 1) * batch->ld * es;
    e = hipMemset2DAsync(last, (size_t)batch->L * batch->ld * es, 0, (size_t)batch->V * es,
                         (size_t)batch->B, s);
    if (e != hipSuccess) return (int)e;
  }
  const int64_t nrows = batch->B * (batch->L - 1);
  e = launch_rows(a, batch, params, out, nrows, scratch_of(workspace), s);
  if (e != hipSuccess) return (int)e;
  return (int)launch_stats(a, nrows, out->stats, s);
}

int prl_grpo_forward_rows(const PrlGrpoBatch* batch, const PrlGrpoParams* params, const int64_t* row_ids,
                          int64_t n, const PrlGrpoOutputs* out, void* workspace, size_t workspace_bytes,
                          void* stream) {
  KArgs a;
  int rc = fill_args(a, batch, params);
  if (rc) return rc;
  // a value head's values enter the rows only through the advantage (reward - value,
  // rl/__init__.py:239-248); its loss, statistics and dvalues are prl_grpo_stats' (out->dvalues is
  // required as there but not written here)
  rc = fill_outputs(a, batch, params, out, false);
  if (rc) return rc;
  if (n < 0 || (n > 0 && !row_ids)) return PRL_E_INVALID;
  if (!workspace || workspace_bytes < kWorkspaceBytes) return PRL_E_WORKSPACE;
  if (n == 0) return PRL_OK;
  a.row_ids = row_ids;
  a.nsel = n;
  return (int)launch_rows(a, batch, params, out, n, scratch_of(workspace), static_cast<hipStream_t>(stream));
}

int prl_grpo_stats(const PrlGrpoBatch* batch, const PrlGrpoParams* params, const PrlGrpoOutputs* out,
                   void* workspace, size_t workspace_bytes, void* stream) {
  KArgs a;
  int rc = fill_args(a, batch, params, false);
  if (rc) return rc;
  if (!out || !out->new_logprobs || !out->entropy || !out->stats) return PRL_E_INVALID;
  if (batch->values && !out->dvalues) return PRL_E_INVALID;
  if (!workspace || workspace_bytes < kWorkspaceBytes) return PRL_E_WORKSPACE;
  a.o_lp = out->new_logprobs;
  a.o_ent = out->entropy;
  a.o_dv = out->dvalues;
  a.partials = static_cast<double*>(workspace);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (batch->values) {
    hipError_t e = hipMemsetAsync(out->dvalues, 0, sizeof(float) * (size_t)(batch->B * batch->L), s);
    if (e != hipSuccess) return (int)e;
  }
  return (int)launch_stats(a, batch->B * (batch->L - 1), out->stats, s);
}

int prl_grpo_backward(const PrlGrpoBatch* batch, const PrlGrpoParams* params, const float* row_max,
                      const float* row_log2sum, const float* entropy, const float* g_lp, const float* g_h,
                      const float* upstream, void* dlogits, void* stream) {
  KArgs a;
  int rc = fill_args(a, batch, params);
  if (rc) return rc;
  if (!row_max || !row_log2sum || !entropy || !g_lp || !g_h || !dlogits) return PRL_E_INVALID;
  a.dlogits = dlogits;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int skip = params->write_grad ? 1 : 0;
  if (!skip) {  // rows t = L-1 carry no loss
    const size_t es = batch->logits_dtype == PRL_BF16 ? 2 : 4;
    char* last = static_cast<char*>(dlogits) + (size_t)(batch->L - 1) * batch->ld * es;
    hipError_t e = hipMemset2DAsync(last, (size_t)batch->L * batch->ld * es, 0, (size_t)batch->V * es,
                                    (size_t)batch->B, s);
    if (e != hipSuccess) return (int)e;
  }
  const int64_t nrows = batch->B * (batch->L - 1);
  if (nrows == 0) return PRL_OK;
  const int64_t want = (int64_t)device_cus(stream_device(s)) * 8;
  const int grid = (int)(nrows < want ? nrows : want);
  const bool bf16 = batch->logits_dtype == PRL_BF16;
  if (bf16 && batch->V % 8 == 0 && batch->ld % 8 == 0 && aligned16(batch->logits) && aligned16(dlogits)) {
    hipLaunchKernelGGL((grpo_bwd_stream<uint16_t, 8>), dim3(grid), dim3(256), 0, s, a, row_max, row_log2sum, entropy, g_lp, g_h, upstream, skip);
  } else if (bf16) {
    hipLaunchKernelGGL((grpo_bwd_stream<uint16_t, 1>), dim3(grid), dim3(256), 0, s, a, row_max, row_log2sum, entropy, g_lp, g_h, upstream, skip);
  } else if (batch->V % 4 == 0 && batch->ld % 4 == 0 && aligned16(batch->logits) && aligned16(dlogits)) {
    hipLaunchKernelGGL((grpo_bwd_stream<float, 4>), dim3(grid), dim3(256), 0, s, a, row_max, row_log2sum, entropy, g_lp, g_h, upstream, skip);
  } else {
    hipLaunchKernelGGL((grpo_bwd_stream<float, 1>), dim3(grid), dim3(256), 0, s, a, row_max, row_log2sum, entropy, g_lp, g_h, upstream, skip);
  }
  return (int)hipGetLastError();
}

int prl_grpo_nstat(void) { return PRL_NSTAT; }

int prl_grpo_pair_fallbacks(void* workspace, size_t workspace_bytes, void* stream, uint64_t* count) {
  if (!count) return PRL_E_INVALID;
  *count = 0;
  if (!workspace || workspace_bytes < kWorkspaceBytes) return PRL_E_WORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t* ctr = scratch_of(workspace).fallbacks;
  uint32_t host = 0;
  hipError_t e = hipMemcpyAsync(&host, ctr, sizeof(host), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemsetAsync(ctr, 0, sizeof(uint32_t), s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return (int)e;
  *count = host;
  return PRL_OK;
}

}  // extern "C"
