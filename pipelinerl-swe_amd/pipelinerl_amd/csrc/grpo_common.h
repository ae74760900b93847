// Shared device code for the GRPO loss-head kernels (gfx950 / CDNA4, wave64).
//
// Math follows pipelinerl/finetune/rl/__init__.py:199-366 (see oracle/grpo_oracle.py for
// the CPU restatement it is tested against).  All per-vocab math is fp32 in the base-2
// domain: with c = log2(e)/temperature and raw logit x,
//   y_j = (x_j - m) c,   s = sum 2^y_j,   w = sum 2^y_j * y_j          (per row)
//   LSE = m/temperature + ln2 * log2(s)
//   H   = ln2 * (log2(s) - w/s)                     (entropy, no cancellation vs LSE)
//   lp_j = ln2 * t_j,  t_j = (x_j - m) c - log2(s),  p_j = 2^t_j
//   dlogit_j = p_j * (alpha + beta * t_j)
// (x_j - m) is formed first (exact for bf16 inputs), so large logit ranges / small
// temperatures keep full relative precision near the max (no rounding of m c).
//              alpha = -(g_lp + g_h H)/temperature,  beta = -g_h ln2 / temperature
//              plus g_lp/temperature at the target column.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "prl_hip.h"

namespace prl {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kFltMax = 3.402823466e+38f;
constexpr float kEmptyMax = -1.0e30f;  // running-max seed: finite so empty states combine to 0
constexpr float kRescaleSlack = 8.0f;  // lazy rescale: keep 2^y <= 2^8 (log2 units)
constexpr int kMaxGrid = 2048;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ float bf_to_f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even pack (v_cvt_pk_bf16_f32 on gfx950; NaN stays NaN)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  f32x2 v = {lo, hi};
  bf16x2_t r = __builtin_convertvector(v, bf16x2_t);
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint16_t f_to_bf(float x) {
  __bf16 r = (__bf16)x;
  return __builtin_bit_cast(uint16_t, r);
}

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---------------------------------------------------------------------------------------
// Online (max, sum 2^y, sum 2^y y) state
struct Lse {
  float m, s, w;
};

__device__ __forceinline__ Lse lse_empty() { return Lse{kEmptyMax, 0.f, 0.f}; }

// move reference point from st.m to mn (mn >= st.m)
__device__ __forceinline__ void lse_rebase(Lse& st, float mn, float c) {
  const float d = (st.m - mn) * c;  // <= 0
  const float f = fexp2(d);
  st.w = f * __builtin_fmaf(st.s, d, st.w);
  st.s = st.s * f;
  st.m = mn;
}

__device__ __forceinline__ Lse lse_combine(Lse a, Lse b, float c) {
  const float M = fmaxf(a.m, b.m);
  const float da = (a.m - M) * c, db = (b.m - M) * c;
  const float fa = fexp2(da), fb = fexp2(db);
  Lse r;
  r.m = M;
  r.s = a.s * fa + b.s * fb;
  r.w = fa * __builtin_fmaf(a.s, da, a.w) + fb * __builtin_fmaf(b.s, db, b.w);
  // NaN in either max poisons the row (torch semantics: non-finite logits -> NaN lp)
  if (a.m != a.m || b.m != b.m) r.s = __builtin_nanf("");
  return r;
}

// Add N raw values.  Lazy rescale: the reference point only moves when a value exceeds it
// by more than kRescaleSlack/c, so 2^y stays <= 2^8 and the rebase is rare.
template <int N>
__device__ __forceinline__ void lse_add(Lse& st, const float (&x)[N], float c) {
  float vm = x[0];
#pragma unroll
  for (int j = 1; j < N; ++j) vm = fmaxf(vm, x[j]);
  if ((vm - st.m) * c > kRescaleSlack) lse_rebase(st, vm, c);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float y = (x[j] - st.m) * c;
    const float e = fexp2(y);
    st.s += e;
    st.w = __builtin_fmaf(e, y, st.w);
  }
  if (vm != vm) st.m = __builtin_nanf("");  // a NaN logit poisons the state
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ Lse lse_dpp_step(Lse st, float c) {
  return lse_combine(st, Lse{dpp<CTRL>(st.m), dpp<CTRL>(st.s), dpp<CTRL>(st.w)}, c);
}
__device__ __forceinline__ Lse lse_readlane(Lse st, int lane) {
  return Lse{__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, st.m), lane)),
             __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, st.s), lane)),
             __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, st.w), lane))};
}
// Wave64 reduction without LDS address registers: DPP quad_perm xor1 / xor2, row half-mirror,
// row mirror (16-lane totals in every lane), then the four row totals via readlane.  The
// result is wave-uniform.
__device__ __forceinline__ Lse wave_reduce_lse(Lse st, float c) {
  st = lse_dpp_step<0xB1>(st, c);   // quad_perm [1,0,3,2]
  st = lse_dpp_step<0x4E>(st, c);   // quad_perm [2,3,0,1]
  st = lse_dpp_step<0x141>(st, c);  // row_half_mirror
  st = lse_dpp_step<0x140>(st, c);  // row_mirror
  const Lse r0 = lse_readlane(st, 0), r1 = lse_readlane(st, 16);
  const Lse r2 = lse_readlane(st, 32), r3 = lse_readlane(st, 48);
  return lse_combine(lse_combine(r0, r1, c), lse_combine(r2, r3, c), c);
}

// ---------------------------------------------------------------------------------------
// Kernel arguments (by value)
struct KArgs {
  const void* logits;
  int64_t B, L, V, ld;
  const int64_t* input_ids;
  const int64_t* labels;
  const float* rewards;
  const float* advantages;
  const float* ref_lp;
  const float* old_lp;
  const float* group_tokens;
  const float* num_labels;
  const float* overflow;
  const float* values;
  // params
  int policy, use_adv, relu, group_norm, overlong, write_grad;
  float eps, kl_c, ent_c, clampC, temperature, batch_size, value_coef, gscale;
  // outputs
  float *o_lp, *o_ent, *o_lse, *o_tok, *o_glp, *o_gh, *o_max, *o_l2s, *o_dv;
  void* dlogits;
  double* partials;  // [gridDim.x][PRL_NSTAT]
  // row selection (prl_grpo_forward_rows): logits row i scores batch row row_ids[i]
  const int64_t* row_ids;
  int64_t nsel;
  // grpo_fwd_resident: rows after each workgroup's first are claimed from this counter (zeroed
  // before the launch); null: the static stride q += gridDim.x
  uint32_t* row_ctr;
};

// Per-token quantities of rl/__init__.py:212-292 for one loss row.
struct TokVals {
  bool m;                    // label mask (labels != -100)
  float w, ratio, lrrn, adv, lpw, cc, ecc, kl, s1, s2, pol, ratio_used, tl;
  bool ind_no;
};

__device__ __forceinline__ float nz(float v) {  // torch.nan_to_num for float32
  if (v != v) return 0.f;
  if (v == __builtin_inff()) return kFltMax;
  if (v == -__builtin_inff()) return -kFltMax;
  return v;
}
// NaN-propagating clamp / min (torch.clamp, torch.minimum)
__device__ __forceinline__ float tclamp(float v, float lo, float hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}
__device__ __forceinline__ float tmin(float a, float b) {
  if (a != a || b != b) return __builtin_nanf("");
  return a < b ? a : b;
}

// reductions of statistic i: sum, or masked max / min (NaN-propagating like torch.max)
__device__ __forceinline__ bool stat_is_max(int i) {
  return i == PRL_S_MAX_REWARD || i == PRL_S_MAX_ADV || i == PRL_S_MAX_KL || i == PRL_S_MAX_W ||
         i == PRL_S_MAX_VALUE;
}
__device__ __forceinline__ bool stat_is_min(int i) {
  return i == PRL_S_MIN_REWARD || i == PRL_S_MIN_ADV || i == PRL_S_MIN_KL || i == PRL_S_MIN_W ||
         i == PRL_S_MIN_VALUE;
}
__device__ __forceinline__ double stat_identity(int i) {
  if (stat_is_max(i)) return -__builtin_inf();
  if (stat_is_min(i)) return __builtin_inf();
  return 0.0;
}
__device__ __forceinline__ double stat_fold(int i, double acc, double v) {
  if (stat_is_max(i)) return (acc != acc || v != v) ? __builtin_nan("") : (v > acc ? v : acc);
  if (stat_is_min(i)) return (acc != acc || v != v) ? __builtin_nan("") : (v < acc ? v : acc);
  return acc + v;
}

// Loads of the per-token inputs (never written by the loss kernels).  VecLd: plain vector loads,
// any index.  SclLd: a wave-uniform index read through the scalar cache (s_load into SGPRs): no
// VGPRs, and counted by lgkmcnt, so waiting for it never waits for the row's vector loads in
// flight (a vector load of a token input behind the row's 19 buffer loads had to wait for all of them).
struct VecLd {
  template <typename T>
  static __device__ __forceinline__ T ld(const T* p, int64_t i) { return p[i]; }
};
struct SclLd {
  template <typename T>
  static __device__ __forceinline__ T ld(const T* p, int64_t i) {
    return ((const __attribute__((address_space(4))) T*)p)[i];
  }
};

// the per-token inputs token_values reads (rl/__init__.py:212-248)
struct TokIn {
  int64_t label;
  float reward, ref, old, gt, ovf, advsrc;
};
template <typename LD>
__device__ __forceinline__ TokIn tok_in(const KArgs& a, int64_t tok) {
  TokIn t;
  t.label = LD::ld(a.labels, tok);
  t.reward = LD::ld(a.rewards, tok);
  t.ref = LD::ld(a.ref_lp, tok);
  t.old = LD::ld(a.old_lp, tok);
  t.gt = a.group_norm ? LD::ld(a.group_tokens, tok) : 1.0f;
  t.ovf = a.overlong ? LD::ld(a.overflow, tok) : 0.0f;
  t.advsrc = a.values != nullptr ? LD::ld(a.values, tok - 1) : LD::ld(a.advantages, tok);  // values unshifted
  return t;
}

__device__ __forceinline__ TokVals token_values(const KArgs& a, const TokIn& in, float lp, float H) {
  TokVals v;
  v.m = in.label != -100;
  const float reward = in.reward;
  const float ref = in.ref;
  const float old = in.old;
  const bool has_v = a.values != nullptr;
  float w = a.group_norm ? 1.0f / in.gt : 1.0f / a.batch_size;  // :220-225
  if (a.overlong) w = w * (1.0f - in.ovf);                      // :227-230
  v.w = w;
  v.ratio = expf(lp - old);  // :234-236
  v.lrrn = ref - lp;
  v.adv = has_v ? reward - in.advsrc : in.advsrc;  // :239-248
  float lpw = a.use_adv ? v.adv : reward;                          // :250-252
  if (a.relu) lpw = lpw < 0.f ? 0.f : lpw;
  v.lpw = lpw;
  const float C = a.clampC;
  v.cc = tclamp(v.lrrn, -C, C);  // :256-260
  v.ecc = expf(v.cc);
  v.kl = v.ecc - v.cc - 1.0f;  // :262
  if (a.policy == PRL_PPO) {   // :270-275
    v.s1 = v.ratio * lpw;
    const float cr = tclamp(v.ratio, 1.0f - a.eps, 1.0f + a.eps);
    v.ind_no = cr != v.ratio;
    v.s2 = cr * lpw;
    v.pol = tmin(v.s1, v.s2);
    v.ratio_used = v.ratio;
  } else {  // reinforce :276-281
    v.s1 = 0.f;
    v.s2 = 0.f;
    v.ind_no = v.ratio > 1.0f + a.eps;
    v.ratio_used = tclamp(v.ratio, 0.0f, 1.0f + a.eps);
    v.pol = lp * lpw * v.ratio_used;
  }
  v.tl = ((v.pol - a.kl_c * v.kl) + a.ent_c * H) * w;  // :286-290
  return v;
}
__device__ __forceinline__ TokVals token_values(const KArgs& a, int64_t tok, float lp, float H) {
  return token_values(a, tok_in<VecLd>(a, tok), lp, H);
}

// d final / d new_lp and d final / d entropy for one row (analytic backward with torch's
// rules: minimum splits ties, clamp passes on the closed interval, nan_to_num passes where
// finite; masked rows get exactly zero).
struct TokGrad {
  float g_lp, g_h;
};
__device__ __forceinline__ TokGrad token_grad(const KArgs& a, const TokVals& v) {
  const bool fin = __builtin_isfinite(v.tl);
  const float g_tok = (v.m && fin) ? -a.gscale : 0.f;
  TokGrad g{0.f, 0.f};
  if (g_tok == 0.f) return g;
  const float g_pol = g_tok * v.w;
  const float g_kl = -g_tok * v.w * a.kl_c;
  float g_lp;
  if (a.policy == PRL_PPO) {
    const bool tie = v.s1 == v.s2;
    const float gs1 = g_pol * (tie ? 0.5f : (v.s1 < v.s2 ? 1.f : 0.f));
    const float gs2 = g_pol * (tie ? 0.5f : (v.s2 < v.s1 ? 1.f : 0.f));
    const float inr = (v.ratio >= 1.0f - a.eps && v.ratio <= 1.0f + a.eps) ? 1.f : 0.f;
    g_lp = (gs1 * v.lpw + gs2 * v.lpw * inr) * v.ratio;
  } else {
    g_lp = g_pol * v.lpw * v.ratio_used;
  }
  const float C = a.clampC;
  const float inr_c = (v.lrrn >= -C && v.lrrn <= C) ? 1.f : 0.f;
  g.g_lp = g_lp - g_kl * (v.ecc - 1.0f) * inr_c;
  g.g_h = g_tok * v.w * a.ent_c;
  return g;
}

// Row mapping: loss row q -> (logits row, shifted token index)
__device__ __forceinline__ void row_of(const KArgs& a, int64_t q, int64_t& lrow, int64_t& tok) {
  const int64_t Lm1 = a.L - 1;
  const int64_t b = q / Lm1;
  const int64_t t = q - b * Lm1;
  lrow = b * a.L + t;
  tok = lrow + 1;
}

// number of logits rows a forward kernel walks
__device__ __forceinline__ int64_t fwd_rows(const KArgs& a) { return a.row_ids ? a.nsel : a.B * (a.L - 1); }

// logits row i -> (logits row offset, token index, output row q)
template <typename LD = VecLd>
__device__ __forceinline__ void map_row(const KArgs& a, int64_t i, int64_t& lrow, int64_t& tok, int64_t& q) {
  if (a.row_ids) {
    q = LD::ld(a.row_ids, i);
    int64_t full;
    row_of(a, q, full, tok);
    lrow = i;
  } else {
    q = i;
    row_of(a, i, lrow, tok);
  }
}

}  // namespace prl
