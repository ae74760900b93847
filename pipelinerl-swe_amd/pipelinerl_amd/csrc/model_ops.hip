// Fused element-wise ops of the trainer's model step (Qwen2 / Llama-style decoder), bf16.
//
// In the reference's trainer these run as HF eager op chains (transformers Qwen2RMSNorm,
// Qwen2MLP act_fn(gate) * up, apply_rotary_pos_emb): ~25 % of a 1.5B trainer step on MI355X
// is those chains (profiles/r01_trainer_step_kernel_stats.csv).  Each op here is one HBM pass
// forward and one backward, and the forward reproduces the eager chain's bf16 roundings
// exactly (same intermediate casts), so patched and unpatched models agree bit for bit in
// the forward pass.
//   rmsnorm   y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps)))         (fp32 statistics)
//   add_rmsnorm  h = bf16(residual + x), y = rmsnorm(h)            (decoder residual add fused)
//   swiglu    h = bf16(bf16(silu(g)) * u)
//   rope      q' = bf16(bf16(q * cos) + bf16(rotate_half(q) * sin))  (q and k in one launch)
// HBM-bound: 16-B vector loads/stores, one wave per row for the norms.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "prl_hip.h"

namespace prl_ops {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lo(uint32_t v) { return __builtin_bit_cast(float, v << 16); }
__device__ __forceinline__ float hi(uint32_t v) { return __builtin_bit_cast(float, v & 0xFFFF0000u); }
// float -> bf16, round to nearest even.  gfx950 converts in hardware (v_cvt_pk_bf16_f32, two
// values per instruction, RNE, NaN stays NaN): 1-2 vector instructions where the integer
// sequence below takes 5-6 per value, and these kernels run ~40 such roundings per element pair
// (the eager chain's intermediate bf16 casts).  PRL_HW_BF16=0 keeps the integer sequence (A/B).
#ifndef PRL_HW_BF16
#define PRL_HW_BF16 1
#endif
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t rne(float f) {  // bf16 bits in the low half
#if PRL_HW_BF16
  return __builtin_bit_cast(uint16_t, (__bf16)f);
#else
  const uint32_t u = __builtin_bit_cast(uint32_t, f);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (u >> 16) | 0x40u;  // NaN stays NaN
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
#endif
}
__device__ __forceinline__ float r16(float f) { return __builtin_bit_cast(float, rne(f) << 16); }  // bf16 round
__device__ __forceinline__ uint32_t pack(float a, float b) {
#if PRL_HW_BF16
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
#else
  return rne(a) | (rne(b) << 16);
#endif
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------------
// RMSNorm.  One wave per row; the row (H <= 64 * 8 * NV bf16) stays in registers.
// ADD: x is the sublayer output and the row normalised is h = bf16(res + x) (the decoder's
// residual add, eager `residual + hidden_states`), also written to `hout`.
template <int NV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                   uint16_t* __restrict__ y, float* __restrict__ rstd,
                                                   int64_t rows, int H, float eps, const uint16_t* __restrict__ res,
                                                   uint16_t* __restrict__ hout) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int nv8 = H >> 3;
  u32x4 wv[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 64 + lane;
    wv[k] = c < nv8 ? reinterpret_cast<const u32x4*>(w)[c] : u32x4{0, 0, 0, 0};
  }
  for (int64_t r = wave; r < rows; r += nwaves) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + r * H);
    u32x4 xv[NV];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      xv[k] = c < nv8 ? __builtin_nontemporal_load(xr + c) : u32x4{0, 0, 0, 0};
      if constexpr (ADD) {
        if (c < nv8) {
          const u32x4 rv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(res + r * H) + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[k][j] = pack(lo(rv[j]) + lo(xv[k][j]), hi(rv[j]) + hi(xv[k][j]));
          __builtin_nontemporal_store(xv[k], reinterpret_cast<u32x4*>(hout + r * H) + c);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = lo(xv[k][j]), b = hi(xv[k][j]);
        ss = __builtin_fmaf(a, a, __builtin_fmaf(b, b, ss));
      }
    }
    ss = wave_sum(ss);
    const float rs = 1.0f / __builtin_sqrtf(ss / (float)H + eps);
    if (lane == 0) rstd[r] = rs;
    u32x4* yr = reinterpret_cast<u32x4*>(y + r * H);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      if (c < nv8) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t0 = r16(lo(xv[k][j]) * rs), t1 = r16(hi(xv[k][j]) * rs);
          o[j] = pack(lo(wv[k][j]) * t0, hi(wv[k][j]) * t1);
        }
        __builtin_nontemporal_store(o, yr + c);
      }
    }
  }
}

// dx_i = r g_i - (r^3 / H) x_i sum_j g_j x_j with g = bf16(dy * w);  dw partial per block:
// sum over the block's rows of bf16(dy * bf16(x r)) (the eager chain's weight-grad product).
// dx_i = r g_i - (r^3 / H) x_i sum_j g_j x_j with g = bf16(dy * w);  dw partial per block:
// sum over the block's rows of bf16(dy * bf16(x r)) (the eager chain's weight-grad product).
template <int NV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_bwd_narrow(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                   const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                                                   uint16_t* __restrict__ dx, float* __restrict__ partial,
                                                   int64_t rows, int H, const uint16_t* __restrict__ dres) {
  __shared__ float red[4][64 * 8 * NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wid;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int nv8 = H >> 3;
  const float invH = 1.0f / (float)H;
  u32x4 wv[NV];
  float acc[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 64 + lane;
    wv[k] = c < nv8 ? reinterpret_cast<const u32x4*>(w)[c] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  }
  for (int64_t r = wave; r < rows; r += nwaves) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + r * H);
    const u32x4* gr = reinterpret_cast<const u32x4*>(dy + r * H);
    const float rs = rstd[r];
    u32x4 xv[NV], gv[NV], dv[ADD ? NV : 1];
    float dot = 0.f;
    // keep w packed across the row loop (no hoisted unpacked copy): registers go to occupancy
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(wv[k]));
    if constexpr (ADD) {  // issued with the row's other loads: in flight across the reduction
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = k * 64 + lane;
        dv[k] = c < nv8 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dres + r * H) + c)
                        : u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      xv[k] = c < nv8 ? __builtin_nontemporal_load(xr + c) : u32x4{0, 0, 0, 0};
      gv[k] = c < nv8 ? __builtin_nontemporal_load(gr + c) : u32x4{0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g0 = r16(lo(gv[k][j]) * lo(wv[k][j])), g1 = r16(hi(gv[k][j]) * hi(wv[k][j]));
        dot = __builtin_fmaf(g0, lo(xv[k][j]), __builtin_fmaf(g1, hi(xv[k][j]), dot));
        const float t0 = r16(lo(xv[k][j]) * rs), t1 = r16(hi(xv[k][j]) * rs);
        acc[k][2 * j] += r16(lo(gv[k][j]) * t0);
        acc[k][2 * j + 1] += r16(hi(gv[k][j]) * t1);
      }
    }
    dot = wave_sum(dot);
    const float cfac = rs * rs * rs * invH * dot;
    u32x4* dr = reinterpret_cast<u32x4*>(dx + r * H);
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(xv[k]), "+v"(gv[k]), "+v"(wv[k]));  // re-unpack below
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      if (c < nv8) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g0 = r16(lo(gv[k][j]) * lo(wv[k][j])), g1 = r16(hi(gv[k][j]) * hi(wv[k][j]));
          o[j] = pack(rs * g0 - cfac * lo(xv[k][j]), rs * g1 - cfac * hi(xv[k][j]));
        }
        if constexpr (ADD) {  // + the residual branch's gradient, summed as autograd would (bf16 + bf16)
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = pack(lo(o[j]) + lo(dv[k][j]), hi(o[j]) + hi(dv[k][j]));
        }
        __builtin_nontemporal_store(o, dr + c);
      }
    }
  }
  // block partial of dw: fold the 4 waves in LDS, one row of H floats per block
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wid][(k * 64 + lane) * 8 + j] = acc[k][j];
  __syncthreads();
  for (int i = threadIdx.x; i < H; i += 256)
    partial[(int64_t)blockIdx.x * H + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// Wide rows (NV > 4, e.g. H = 3584): the dw partials of the 4 waves fold through ONE LDS row, in
// wave order, so the block needs H floats of LDS instead of 4 H, and w / x / dy stay packed
// between uses: 0.254 -> 0.217 ms at 16384 x 3584 (tools/ew_bench.py [round 1-3 tool, in git history]).  Narrow rows keep the
// 4-row fold (rmsnorm_bwd_narrow), which measured faster at H = 1536 (0.179 vs 0.193 ms).
#ifndef PRL_NORM_WIDE_DRES_EARLY
#define PRL_NORM_WIDE_DRES_EARLY 1  // A/B (add_rmsnorm 8192 x 3584 bwd incl. autograd): 0.144-0.148 -> 0.130 ms
#endif
template <int NV, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_bwd_wide(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                   const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                                                   uint16_t* __restrict__ dx, float* __restrict__ partial,
                                                   int64_t rows, int H, const uint16_t* __restrict__ dres) {
  __shared__ float red[64 * 8 * NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wid;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int nv8 = H >> 3;
  const float invH = 1.0f / (float)H;
  u32x4 wv[NV];
  float acc[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 64 + lane;
    wv[k] = c < nv8 ? reinterpret_cast<const u32x4*>(w)[c] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  }
  u32x4 xv[NV], gv[NV];
  constexpr bool kEarly = ADD && PRL_NORM_WIDE_DRES_EARLY;  // dres loaded with x / dy (in flight across the reduction)
  u32x4 dvv[kEarly ? NV : 1];
  auto load_row = [&](int64_t r, u32x4* xo, u32x4* go) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + r * H);
    const u32x4* gr = reinterpret_cast<const u32x4*>(dy + r * H);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      xo[k] = c < nv8 ? __builtin_nontemporal_load(xr + c) : u32x4{0, 0, 0, 0};
      go[k] = c < nv8 ? __builtin_nontemporal_load(gr + c) : u32x4{0, 0, 0, 0};
      if constexpr (kEarly)
        dvv[k] = c < nv8 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dres + r * H) + c)
                         : u32x4{0, 0, 0, 0};
    }
  };
  if (wave < rows) load_row(wave, xv, gv);
  float rs = wave < rows ? rstd[wave] : 0.f;
  for (int64_t r = wave; r < rows; r += nwaves) {
    constexpr bool kPrefetch = false;  // measured: no gain at H = 1536, registers better spent on occupancy
    u32x4 xn[kPrefetch ? NV : 1], gn[kPrefetch ? NV : 1];
    const int64_t rn = r + nwaves;
    float rsn = 0.f;
    if (kPrefetch && rn < rows) {  // in flight during this row's math
      load_row(rn, xn, gn);
      rsn = rstd[rn];
    }
    // register pressure: keep w packed (no hoisted unpacked copy across the loop) so the kernel
    // runs more than one wave per SIMD
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(wv[k]));
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g0 = r16(lo(gv[k][j]) * lo(wv[k][j])), g1 = r16(hi(gv[k][j]) * hi(wv[k][j]));
        dot = __builtin_fmaf(g0, lo(xv[k][j]), __builtin_fmaf(g1, hi(xv[k][j]), dot));
        const float t0 = r16(lo(xv[k][j]) * rs), t1 = r16(hi(xv[k][j]) * rs);
        acc[k][2 * j] += r16(lo(gv[k][j]) * t0);
        acc[k][2 * j + 1] += r16(hi(gv[k][j]) * t1);
      }
    }
    dot = wave_sum(dot);
    const float cfac = rs * rs * rs * invH * dot;
    u32x4* dr = reinterpret_cast<u32x4*>(dx + r * H);
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(xv[k]), "+v"(gv[k]), "+v"(wv[k]));  // re-unpack below
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      if (c < nv8) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g0 = r16(lo(gv[k][j]) * lo(wv[k][j])), g1 = r16(hi(gv[k][j]) * hi(wv[k][j]));
          o[j] = pack(rs * g0 - cfac * lo(xv[k][j]), rs * g1 - cfac * hi(xv[k][j]));
        }
        if constexpr (ADD) {  // + the residual branch's gradient, summed as autograd would (bf16 + bf16)
          u32x4 dv;
          if constexpr (kEarly) dv = dvv[k];
          else dv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dres + r * H) + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = pack(lo(o[j]) + lo(dv[j]), hi(o[j]) + hi(dv[j]));
        }
        __builtin_nontemporal_store(o, dr + c);
      }
    }
    if (rn < rows) {
      if constexpr (kPrefetch) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          xv[k] = xn[k];
          gv[k] = gn[k];
        }
        rs = rsn;
      } else {
        load_row(rn, xv, gv);
        rs = rstd[rn];
      }
    }
  }
  // block partial of dw: the 4 waves fold into one LDS row in wave order (deterministic)
  for (int wi = 0; wi < 4; ++wi) {
    if (wid == wi) {
#pragma unroll
      for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float& cell = red[(k * 64 + lane) * 8 + j];
          cell = wi ? cell + acc[k][j] : acc[k][j];
        }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < H; i += 256) partial[(int64_t)blockIdx.x * H + i] = red[i];
}

// Wide rows with the dw accumulators in LDS instead of registers (PRL_NORM_BWD_LDS, 5 <= NV <= 8):
// rmsnorm_bwd_wide keeps 8 fp32 accumulators per 16-B vector (56 per lane at H = 3 584) beside the
// packed x / dy / dres of the row and of the next one the compiler prefetches: 339 registers, one
// wave per SIMD (3.8 TB/s).  Here each wave owns one H-float row of LDS (its rows' sums in the same
// order, so the partials are bit-identical), the four rows fold in wave order at the end, and the
// kernel fits 256 registers: two workgroups (two waves per SIMD) per CU, 2 x 4 x H x 4 B of LDS.
// LDS layout per wave: [vector k][half h][lane][4 floats] (16-B, lane-contiguous: conflict-free).
#ifndef PRL_NORM_BWD_LDS
#define PRL_NORM_BWD_LDS 1
#endif
template <int NV, bool ADD>
__global__ __launch_bounds__(256, 2) void rmsnorm_bwd_lds(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                          const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                                                          uint16_t* __restrict__ dx, float* __restrict__ partial,
                                                          int64_t rows, int H, const uint16_t* __restrict__ dres) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  __shared__ f32x4_t acc[4][NV * 2 * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wid;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int nv8 = H >> 3;
  const float invH = 1.0f / (float)H;
  f32x4_t* my = acc[wid];
#pragma unroll
  for (int i = 0; i < NV * 2; ++i) my[i * 64 + lane] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  u32x4 wv[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 64 + lane;
    wv[k] = c < nv8 ? reinterpret_cast<const u32x4*>(w)[c] : u32x4{0, 0, 0, 0};
  }
  for (int64_t r = wave; r < rows; r += nwaves) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + r * H);
    const u32x4* gr = reinterpret_cast<const u32x4*>(dy + r * H);
    const float rs = rstd[r];
    u32x4 xv[NV], gv[NV], dv[ADD ? NV : 1];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      xv[k] = c < nv8 ? __builtin_nontemporal_load(xr + c) : u32x4{0, 0, 0, 0};
      gv[k] = c < nv8 ? __builtin_nontemporal_load(gr + c) : u32x4{0, 0, 0, 0};
      if constexpr (ADD)
        dv[k] = c < nv8 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dres + r * H) + c)
                        : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(wv[k]));
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      f32x4_t a0 = my[(2 * k) * 64 + lane], a1 = my[(2 * k + 1) * 64 + lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g0 = r16(lo(gv[k][j]) * lo(wv[k][j])), g1 = r16(hi(gv[k][j]) * hi(wv[k][j]));
        dot = __builtin_fmaf(g0, lo(xv[k][j]), __builtin_fmaf(g1, hi(xv[k][j]), dot));
        const float t0 = r16(lo(xv[k][j]) * rs), t1 = r16(hi(xv[k][j]) * rs);
        const float c0 = r16(lo(gv[k][j]) * t0), c1 = r16(hi(gv[k][j]) * t1);
        if (j < 2) {
          a0[2 * j] += c0;
          a0[2 * j + 1] += c1;
        } else {
          a1[2 * j - 4] += c0;
          a1[2 * j - 3] += c1;
        }
      }
      my[(2 * k) * 64 + lane] = a0;
      my[(2 * k + 1) * 64 + lane] = a1;
    }
    dot = wave_sum(dot);
    const float cfac = rs * rs * rs * invH * dot;
    u32x4* dr = reinterpret_cast<u32x4*>(dx + r * H);
#pragma unroll
    for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(xv[k]), "+v"(gv[k]), "+v"(wv[k]));  // re-unpack below
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = k * 64 + lane;
      if (c < nv8) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g0 = r16(lo(gv[k][j]) * lo(wv[k][j])), g1 = r16(hi(gv[k][j]) * hi(wv[k][j]));
          o[j] = pack(rs * g0 - cfac * lo(xv[k][j]), rs * g1 - cfac * hi(xv[k][j]));
        }
        if constexpr (ADD) {  // + the residual branch's gradient, summed as autograd would (bf16 + bf16)
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = pack(lo(o[j]) + lo(dv[k][j]), hi(o[j]) + hi(dv[k][j]));
        }
        __builtin_nontemporal_store(o, dr + c);
      }
    }
  }
  __syncthreads();
  // block partial of dw: the 4 waves' rows folded in wave order (as rmsnorm_bwd_wide does)
  const float* a = reinterpret_cast<const float*>(&acc[0][0]);
  constexpr int kRow = NV * 2 * 64 * 4;  // floats per wave row
  for (int i = threadIdx.x; i < H; i += 256) {
    const int v8 = i >> 3, j = i & 7, k = v8 >> 6, ln = v8 & 63;
    const int off = ((2 * k + (j >> 2)) * 64 + ln) * 4 + (j & 3);
    float sum = a[off];
#pragma unroll
    for (int wi = 1; wi < 4; ++wi) sum = sum + a[wi * kRow + off];
    partial[(int64_t)blockIdx.x * H + i] = sum;
  }
}

// dw = sum over the bwd kernel's block partials, deterministic, two levels:
// stage 1: block (column tile of 64, slice s) -> 4 waves x (rows of the slice) -> LDS fold;
// stage 2: one thread per column folds the slices in order.
constexpr int kDwSlices = 32;
__global__ __launch_bounds__(256) void rmsnorm_dw_stage1(const float* __restrict__ partial, int nblocks, int H,
                                                         float* __restrict__ mid) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int per = (nblocks + kDwSlices - 1) / kDwSlices;
  const int b0 = blockIdx.y * per, b1 = b0 + per < nblocks ? b0 + per : nblocks;
  float s = 0.f;
  if (col < H) {
#pragma unroll 8
    for (int b = b0 + wid; b < b1; b += 4) s += partial[(int64_t)b * H + col];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && col < H) mid[(int64_t)blockIdx.y * H + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

__global__ __launch_bounds__(256) void rmsnorm_dw_stage2(const float* __restrict__ mid, int H, uint16_t* __restrict__ dw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= H) return;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kDwSlices; ++k) s += mid[(int64_t)k * H + i];
  dw[i] = (uint16_t)rne(s);
}

// ---------------------------------------------------------------------------------------
// SwiGLU: h = bf16(bf16(silu(g)) * u)
__device__ __forceinline__ float silu(float g) { return g / (1.0f + expf(-g)); }

// SWIGLU_UNROLL vectors per thread per iteration, all loads issued before any math: with one
// vector per thread a CU had ~64 KB of loads in flight, short of the ~60-100 KB per CU the HBM
// latency needs at 5 TB/s (the kernels ran at 4.4 / 4.7 TB/s).
#ifndef SWIGLU_UNROLL
#define SWIGLU_UNROLL 4
#endif
__device__ __forceinline__ u32x4 swiglu_vec(u32x4 gv, u32x4 uv) {
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    o[j] = pack(r16(silu(lo(gv[j]))) * lo(uv[j]), r16(silu(hi(gv[j]))) * hi(uv[j]));
  return o;
}
__global__ __launch_bounds__(256) void swiglu_fwd(const u32x4* __restrict__ g, const u32x4* __restrict__ u,
                                                  u32x4* __restrict__ h, int64_t n8) {
  constexpr int U = SWIGLU_UNROLL;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    u32x4 gv[U], uv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      gv[k] = __builtin_nontemporal_load(g + i + k * stride);
      uv[k] = __builtin_nontemporal_load(u + i + k * stride);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) __builtin_nontemporal_store(swiglu_vec(gv[k], uv[k]), h + i + k * stride);
  }
  for (; i < n8; i += stride)
    __builtin_nontemporal_store(swiglu_vec(__builtin_nontemporal_load(g + i), __builtin_nontemporal_load(u + i)), h + i);
}

// du = bf16(dh * s), s = bf16(silu(g));  dg = bf16(bf16(dh * u) * sig (1 + g (1 - sig)))
__device__ __forceinline__ void swiglu_bwd_vec(u32x4 dv, u32x4 gv, u32x4 uv, u32x4& og, u32x4& ou) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float dgr[2], dur[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float gg = e ? hi(gv[j]) : lo(gv[j]);
      const float uu = e ? hi(uv[j]) : lo(uv[j]);
      const float dd = e ? hi(dv[j]) : lo(dv[j]);
      const float sig = 1.0f / (1.0f + expf(-gg));
      dur[e] = dd * r16(silu(gg));  // the saved bf16 activation, as the eager chain keeps it
      const float ds = r16(dd * uu);
      dgr[e] = ds * (sig * (1.0f + gg * (1.0f - sig)));
    }
    og[j] = pack(dgr[0], dgr[1]);
    ou[j] = pack(dur[0], dur[1]);
  }
}
__global__ __launch_bounds__(256) void swiglu_bwd(const u32x4* __restrict__ dh, const u32x4* __restrict__ g,
                                                  const u32x4* __restrict__ u, u32x4* __restrict__ dg,
                                                  u32x4* __restrict__ du, int64_t n8) {
  constexpr int U = SWIGLU_UNROLL > 2 ? 2 : SWIGLU_UNROLL;  // 3 loads per vector: 2 is enough in flight
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    u32x4 dv[U], gv[U], uv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      dv[k] = __builtin_nontemporal_load(dh + i + k * stride);
      gv[k] = __builtin_nontemporal_load(g + i + k * stride);
      uv[k] = __builtin_nontemporal_load(u + i + k * stride);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      u32x4 og, ou;
      swiglu_bwd_vec(dv[k], gv[k], uv[k], og, ou);
      __builtin_nontemporal_store(og, dg + i + k * stride);
      __builtin_nontemporal_store(ou, du + i + k * stride);
    }
  }
  for (; i < n8; i += stride) {
    u32x4 og, ou;
    swiglu_bwd_vec(__builtin_nontemporal_load(dh + i), __builtin_nontemporal_load(g + i), __builtin_nontemporal_load(u + i),
                   og, ou);
    __builtin_nontemporal_store(og, dg + i);
    __builtin_nontemporal_store(ou, du + i);
  }
}

// Read / write phased SwiGLU (PRL_SWIGLU_PHASED, the loss head's schedule: csrc/grpo_loss.hip):
// one 1024-thread workgroup per CU walks chunks of 1024 x UP vectors; per chunk every thread loads
// all of its inputs, computes, stores, and waits for its stores to retire before the next chunk's
// loads, so a CU never mixes HBM reads and writes.  Same per-element arithmetic (bit-identical).
#ifndef PRL_SWIGLU_PHASED
// contiguous kernels (micro-batches above the fused gate/up limit, e.g. C2's 65 536 tokens):
// fwd 0.81 -> 0.74-0.77 ms, bwd 1.29-1.33 -> 1.07-1.08 ms at 65 536 x 8 960 (profiles/r02_swiglu_phased_ab.jsonl)
#define PRL_SWIGLU_PHASED 1
#endif
#ifndef PRL_SWIGLU_ROWS_PHASED
// row-strided kernels (fused gate/up, C3): the C3 step measured no gain (1477-1481 vs 1480-1483 ms)
#define PRL_SWIGLU_ROWS_PHASED 0
#endif
constexpr int kPhFwdU = 8, kPhBwdU = 6;
// Chunks after each workgroup's first are claimed from `ctr` (zeroed before the launch; null: the
// static stride), as the loss head claims rows (csrc/grpo_loss.hip): a workgroup whose CU is held by
// another queue's kernel (an RCCL channel during the overlapped gradient all-reduce) takes fewer
// chunks instead of a full static share after the others.  One vector atomic per chunk by thread 0,
// issued behind the chunk's loads; the index is published in LDS at the chunk's end (the store wait
// covers the atomic) — results are unchanged.
__device__ __forceinline__ int64_t next_chunk(uint32_t* ctr, uint32_t claim, int64_t cur, int64_t* slot) {
  if (threadIdx.x == 0) *slot = ctr ? (int64_t)gridDim.x + (int64_t)claim : cur + gridDim.x;
  __syncthreads();
  const int64_t v = *slot;
  __syncthreads();  // every wave has read the slot before thread 0 writes the next chunk's
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v));
}
__global__ __launch_bounds__(1024) void swiglu_fwd_phased(const u32x4* __restrict__ g, const u32x4* __restrict__ u,
                                                         u32x4* __restrict__ h, int64_t n8, uint32_t* ctr) {
  constexpr int U = kPhFwdU;
  const int64_t chunk = 1024 * U;
  const int64_t nchunks = (n8 + chunk - 1) / chunk;
  __shared__ int64_t slot;
  for (int64_t c = blockIdx.x; c < nchunks;) {
    const int64_t base = c * chunk;
    u32x4 gv[U], uv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = base + k * 1024 + threadIdx.x;
      gv[k] = i < n8 ? __builtin_nontemporal_load(g + i) : u32x4{0, 0, 0, 0};
      uv[k] = i < n8 ? __builtin_nontemporal_load(u + i) : u32x4{0, 0, 0, 0};
    }
    uint32_t claim = 0;
    if (ctr && threadIdx.x == 0) claim = atomicAdd(ctr, 1u);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = base + k * 1024 + threadIdx.x;
      if (i < n8) __builtin_nontemporal_store(swiglu_vec(gv[k], uv[k]), h + i);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    c = next_chunk(ctr, claim, c, &slot);
  }
}
__global__ __launch_bounds__(1024) void swiglu_bwd_phased(const u32x4* __restrict__ dh, const u32x4* __restrict__ g,
                                                         const u32x4* __restrict__ u, u32x4* __restrict__ dg,
                                                         u32x4* __restrict__ du, int64_t n8, uint32_t* ctr) {
  constexpr int U = kPhBwdU;
  const int64_t chunk = 1024 * U;
  const int64_t nchunks = (n8 + chunk - 1) / chunk;
  __shared__ int64_t slot;
  for (int64_t c = blockIdx.x; c < nchunks;) {
    const int64_t base = c * chunk;
    u32x4 dv[U], gv[U], uv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = base + k * 1024 + threadIdx.x;
      dv[k] = i < n8 ? __builtin_nontemporal_load(dh + i) : u32x4{0, 0, 0, 0};
      gv[k] = i < n8 ? __builtin_nontemporal_load(g + i) : u32x4{0, 0, 0, 0};
      uv[k] = i < n8 ? __builtin_nontemporal_load(u + i) : u32x4{0, 0, 0, 0};
    }
    uint32_t claim = 0;
    if (ctr && threadIdx.x == 0) claim = atomicAdd(ctr, 1u);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = base + k * 1024 + threadIdx.x;
      u32x4 og, ou;
      swiglu_bwd_vec(dv[k], gv[k], uv[k], og, ou);
      if (i < n8) {
        __builtin_nontemporal_store(og, dg + i);
        __builtin_nontemporal_store(ou, du + i);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    c = next_chunk(ctr, claim, c, &slot);
  }
}

// the same for the row-strided forms below: vector i of the [rows, cols8] problem is (i / cols8,
// i % cols8), a thread's vectors 1024 apart (row / column advanced incrementally)
__device__ __forceinline__ void rc_of(int64_t i, int cols8, int64_t& r, int& c) {
  r = i / cols8;
  c = (int)(i - r * cols8);
}
__device__ __forceinline__ void rc_step(int cols8, int64_t& r, int& c) {
  c += 1024;
  while (c >= cols8) {
    c -= cols8;
    ++r;
  }
}
__global__ __launch_bounds__(1024) void swiglu_fwd_rows_phased(const u32x4* __restrict__ g, const u32x4* __restrict__ u,
                                                              u32x4* __restrict__ h, int64_t rows, int cols8,
                                                              int64_t ldg, int64_t ldu, int64_t ldh) {
  constexpr int U = kPhFwdU;
  const int64_t n8 = rows * cols8, chunk = 1024 * U;
  for (int64_t base = (int64_t)blockIdx.x * chunk; base < n8; base += (int64_t)gridDim.x * chunk) {
    u32x4 gv[U], uv[U];
    int64_t r;
    int c;
    rc_of(base + threadIdx.x, cols8, r, c);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool ok = r < rows;
      gv[k] = ok ? __builtin_nontemporal_load(g + r * ldg + c) : u32x4{0, 0, 0, 0};
      uv[k] = ok ? __builtin_nontemporal_load(u + r * ldu + c) : u32x4{0, 0, 0, 0};
      rc_step(cols8, r, c);
    }
    rc_of(base + threadIdx.x, cols8, r, c);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (r < rows) __builtin_nontemporal_store(swiglu_vec(gv[k], uv[k]), h + r * ldh + c);
      rc_step(cols8, r, c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}
__global__ __launch_bounds__(1024) void swiglu_bwd_rows_phased(const u32x4* __restrict__ dh, const u32x4* __restrict__ g,
                                                              const u32x4* __restrict__ u, u32x4* __restrict__ dg,
                                                              u32x4* __restrict__ du, int64_t rows, int cols8,
                                                              int64_t lddh, int64_t ldg, int64_t ldu, int64_t lddg,
                                                              int64_t lddu) {
  constexpr int U = kPhBwdU;
  const int64_t n8 = rows * cols8, chunk = 1024 * U;
  for (int64_t base = (int64_t)blockIdx.x * chunk; base < n8; base += (int64_t)gridDim.x * chunk) {
    u32x4 dv[U], gv[U], uv[U];
    int64_t r;
    int c;
    rc_of(base + threadIdx.x, cols8, r, c);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool ok = r < rows;
      dv[k] = ok ? __builtin_nontemporal_load(dh + r * lddh + c) : u32x4{0, 0, 0, 0};
      gv[k] = ok ? __builtin_nontemporal_load(g + r * ldg + c) : u32x4{0, 0, 0, 0};
      uv[k] = ok ? __builtin_nontemporal_load(u + r * ldu + c) : u32x4{0, 0, 0, 0};
      rc_step(cols8, r, c);
    }
    rc_of(base + threadIdx.x, cols8, r, c);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      u32x4 og, ou;
      swiglu_bwd_vec(dv[k], gv[k], uv[k], og, ou);
      if (r < rows) {
        __builtin_nontemporal_store(og, dg + r * lddg + c);
        __builtin_nontemporal_store(ou, du + r * lddu + c);
      }
      rc_step(cols8, r, c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Row-strided SwiGLU for the fused gate/up GEMM (finetune/model_ops.py GateUpSwiGLUFn): gate and up
// are the two column halves of one [rows, 2 I] GEMM output (row stride ld, 8-element vectors), the
// backward writes dgate / dup into the two halves of one [rows, 2 I] buffer, which the fused dgrad
// and wgrad GEMMs read as they stand.  Same per-element arithmetic as swiglu_fwd / swiglu_bwd
// (bit-identical outputs).  Grid-stride over rows; a row's vectors over the block, SWIGLU_UNROLL
// (bwd: 2) vectors in flight per thread.
__global__ __launch_bounds__(256) void swiglu_fwd_rows(const u32x4* __restrict__ g, const u32x4* __restrict__ u,
                                                       u32x4* __restrict__ h, int64_t rows, int cols8, int64_t ldg,
                                                       int64_t ldu, int64_t ldh) {
  constexpr int U = SWIGLU_UNROLL;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const u32x4 *gr = g + r * ldg, *ur = u + r * ldu;
    u32x4* hr = h + r * ldh;
    int c = threadIdx.x;
    for (; c + (U - 1) * 256 < cols8; c += U * 256) {
      u32x4 gv[U], uv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        gv[k] = __builtin_nontemporal_load(gr + c + k * 256);
        uv[k] = __builtin_nontemporal_load(ur + c + k * 256);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) __builtin_nontemporal_store(swiglu_vec(gv[k], uv[k]), hr + c + k * 256);
    }
    for (; c < cols8; c += 256)
      __builtin_nontemporal_store(swiglu_vec(__builtin_nontemporal_load(gr + c), __builtin_nontemporal_load(ur + c)),
                                  hr + c);
  }
}
__global__ __launch_bounds__(256) void swiglu_bwd_rows(const u32x4* __restrict__ dh, const u32x4* __restrict__ g,
                                                       const u32x4* __restrict__ u, u32x4* __restrict__ dg,
                                                       u32x4* __restrict__ du, int64_t rows, int cols8, int64_t lddh,
                                                       int64_t ldg, int64_t ldu, int64_t lddg, int64_t lddu) {
  constexpr int U = SWIGLU_UNROLL > 2 ? 2 : SWIGLU_UNROLL;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const u32x4 *dr = dh + r * lddh, *gr = g + r * ldg, *ur = u + r * ldu;
    u32x4 *dgr = dg + r * lddg, *dur = du + r * lddu;
    int c = threadIdx.x;
    for (; c + (U - 1) * 256 < cols8; c += U * 256) {
      u32x4 dv[U], gv[U], uv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        dv[k] = __builtin_nontemporal_load(dr + c + k * 256);
        gv[k] = __builtin_nontemporal_load(gr + c + k * 256);
        uv[k] = __builtin_nontemporal_load(ur + c + k * 256);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        u32x4 og, ou;
        swiglu_bwd_vec(dv[k], gv[k], uv[k], og, ou);
        __builtin_nontemporal_store(og, dgr + c + k * 256);
        __builtin_nontemporal_store(ou, dur + c + k * 256);
      }
    }
    for (; c < cols8; c += 256) {
      u32x4 og, ou;
      swiglu_bwd_vec(__builtin_nontemporal_load(dr + c), __builtin_nontemporal_load(gr + c),
                     __builtin_nontemporal_load(ur + c), og, ou);
      __builtin_nontemporal_store(og, dgr + c);
      __builtin_nontemporal_store(ou, dur + c);
    }
  }
}


// ---------------------------------------------------------------------------------------
// RoPE on q [T, Hq, D] and k [T, Hkv, D] (token-major, contiguous), cos / sin [T, D].
// One thread per (token, head, 4 rotation pairs).  dir = +1 forward, -1 backward
// (backward: dx = dy cos + rotate_half^T(dy sin), with rotate_half^T(z) = [z2, -z1]).
template <int DIR>
__global__ __launch_bounds__(256) void rope_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                   const uint16_t* __restrict__ cs, const uint16_t* __restrict__ sn,
                                                   uint16_t* __restrict__ qo, uint16_t* __restrict__ ko,
                                                   int64_t tokens, int hq, int hkv, int D, int64_t ldq, int64_t ldk) {
  const int half = D >> 1, chunks = half >> 2;  // 4 pairs per thread
  const int per_tok = (hq + hkv) * chunks;
  const int64_t total = tokens * per_tok;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += stride) {
    const int64_t t = idx / per_tok;
    const int rem = (int)(idx - t * per_tok);
    const int h = rem / chunks, c = rem - h * chunks;
    const bool isq = h < hq;
    const uint16_t* src = isq ? q + t * ldq + h * D : k + t * ldk + (h - hq) * D;  // token strides (fused qkv)
    uint16_t* dst = isq ? qo + (t * hq + h) * D : ko + (t * hkv + (h - hq)) * D;
    const int i = c * 4;
    const u32x2 x1 = *reinterpret_cast<const u32x2*>(src + i), x2 = *reinterpret_cast<const u32x2*>(src + half + i);
    const u32x2 c1 = *reinterpret_cast<const u32x2*>(cs + t * D + i),
                c2 = *reinterpret_cast<const u32x2*>(cs + t * D + half + i);
    const u32x2 s1 = *reinterpret_cast<const u32x2*>(sn + t * D + i),
                s2 = *reinterpret_cast<const u32x2*>(sn + t * D + half + i);
    u32x2 o1, o2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float a[2], b[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float xa = e ? hi(x1[j]) : lo(x1[j]), xb = e ? hi(x2[j]) : lo(x2[j]);
        const float ca = e ? hi(c1[j]) : lo(c1[j]), cb = e ? hi(c2[j]) : lo(c2[j]);
        const float sa = e ? hi(s1[j]) : lo(s1[j]), sb = e ? hi(s2[j]) : lo(s2[j]);
        if (DIR > 0) {  // [x1 c1 - x2 s1, x2 c2 + x1 s2]
          a[e] = r16(xa * ca) + r16(-xb * sa);
          b[e] = r16(xb * cb) + r16(xa * sb);
        } else {        // [y1 c1 + y2 s2, y2 c2 - y1 s1]
          a[e] = r16(xa * ca) + r16(xb * sb);
          b[e] = r16(xb * cb) + (-r16(xa * sa));
        }
      }
      o1[j] = pack(a[0], a[1]);
      o2[j] = pack(b[0], b[1]);
    }
    *reinterpret_cast<u32x2*>(dst + i) = o1;
    *reinterpret_cast<u32x2*>(dst + half + i) = o2;
  }
}

constexpr int kMaxNV = 16;     // forward: H <= 8192
constexpr int kMaxNVBwd = 10;  // backward keeps 8 x NV fp32 dw accumulators per lane: H <= 5120

template <int NV>
hipError_t launch_norm_fwd(const void* x, const void* w, void* y, float* rstd, int64_t rows, int H, float eps,
                           int grid, hipStream_t s, const void* res, void* hout) {
  if (res)
    hipLaunchKernelGGL((rmsnorm_fwd<NV, true>), dim3(grid), dim3(256), 0, s, (const uint16_t*)x, (const uint16_t*)w,
                       (uint16_t*)y, rstd, rows, H, eps, (const uint16_t*)res, (uint16_t*)hout);
  else
    hipLaunchKernelGGL((rmsnorm_fwd<NV, false>), dim3(grid), dim3(256), 0, s, (const uint16_t*)x, (const uint16_t*)w,
                       (uint16_t*)y, rstd, rows, H, eps, (const uint16_t*)nullptr, (uint16_t*)nullptr);
  return hipGetLastError();
}
template <int NV, bool ADD>
hipError_t launch_norm_bwd_t(const void* dy, const void* x, const void* w, const float* rstd, void* dx, float* partial,
                             int64_t rows, int H, int grid, hipStream_t s, const void* dres) {
  auto kern = NV <= 4 ? rmsnorm_bwd_narrow<NV, ADD>
                      : (PRL_NORM_BWD_LDS && NV <= 8 ? rmsnorm_bwd_lds<NV, ADD> : rmsnorm_bwd_wide<NV, ADD>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const uint16_t*)dy, (const uint16_t*)x, (const uint16_t*)w,
                     rstd, (uint16_t*)dx, partial, rows, H, (const uint16_t*)dres);
  return hipGetLastError();
}
template <int NV>
hipError_t launch_norm_bwd(const void* dy, const void* x, const void* w, const float* rstd, void* dx, float* partial,
                           int64_t rows, int H, int grid, hipStream_t s, const void* dres) {
  return dres ? launch_norm_bwd_t<NV, true>(dy, x, w, rstd, dx, partial, rows, H, grid, s, dres)
              : launch_norm_bwd_t<NV, false>(dy, x, w, rstd, dx, partial, rows, H, grid, s, nullptr);
}
template <int... N>
hipError_t norm_fwd_table(int nv, const void* x, const void* w, void* y, float* rstd, int64_t rows, int H, float eps,
                          int grid, hipStream_t s, const void* res, void* hout, std::integer_sequence<int, N...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((nv == N + 1 ? (e = launch_norm_fwd<N + 1>(x, w, y, rstd, rows, H, eps, grid, s, res, hout), true) : false) ||
         ...);
  return e;
}
template <int... N>
hipError_t norm_bwd_table(int nv, const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                          float* partial, int64_t rows, int H, int grid, hipStream_t s, const void* dres,
                          std::integer_sequence<int, N...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((nv == N + 1 ? (e = launch_norm_bwd<N + 1>(dy, x, w, rstd, dx, partial, rows, H, grid, s, dres), true) : false) ||
         ...);
  return e;
}

bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
bool a8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }
// one 1024-thread workgroup per CU (x PRL_SWIGLU_PHASED_WG)
#ifndef PRL_SWIGLU_PHASED_WG
#define PRL_SWIGLU_PHASED_WG 1
#endif
// the phased SwiGLU kernels claim chunks from the caller's counter (zeroed here, stream-ordered);
// without one they take the static stride
static hipError_t reset_counter(uint32_t* ctr, hipStream_t s) {
  return ctr ? hipMemsetAsync(ctr, 0, sizeof(uint32_t), s) : hipSuccess;
}

// one workgroup per CU of the stream's device (cached per device)
static int phased_grid(hipStream_t s) {
  static int cus[64] = {};
  int dev = 0;
  if (s == nullptr || hipStreamGetDevice(s, &dev) != hipSuccess) (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 256 * PRL_SWIGLU_PHASED_WG;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev] * PRL_SWIGLU_PHASED_WG;
}
int ew_grid(int64_t n8) {
  const int64_t g = (n8 + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}
constexpr int kNormBlocks = 2048;  // rmsnorm backward blocks (4 waves each): enough waves in flight
// Backward grid cap (<= kNormBlocks, the workspace's partial rows): one resident round, 3 blocks of 4
// waves per CU on 256 CUs at the kernels' 3 waves per SIMD, so no partial last round of blocks
// (A/B vs 2048: 0.187 -> 0.178 ms at 65536 x 1536, 0.213 -> 0.196 at 16384 x 3584;
// profiles/r01_norm_grid_ab.jsonl)
// Forward grid cap: one resident round (6 blocks of 4 waves per CU on 256 CUs; the add form runs
// 6 waves per SIMD): 0.078 -> 0.073 ms at 65536 x 1536, add form 0.152 -> 0.145 ms, vs 2048
// (profiles/r01_norm_grid_ab.jsonl)
#ifndef PRL_NORM_FWD_GRID
#define PRL_NORM_FWD_GRID 1536
#endif
#ifndef PRL_NORM_LDS_GRID
#define PRL_NORM_LDS_GRID 512
#endif
#ifndef PRL_NORM_GRID
#define PRL_NORM_GRID 768
#endif

}  // namespace prl_ops

using namespace prl_ops;

extern "C" {

int prl_rmsnorm_workspace_bytes(int64_t H, size_t* bytes) {
  if (!bytes || H <= 0) return PRL_E_INVALID;
  *bytes = sizeof(float) * (size_t)(kNormBlocks + kDwSlices) * (size_t)H;
  return PRL_OK;
}

static int norm_forward(const void* x, const void* w, void* y, float* rstd, int64_t rows, int64_t H, float eps,
                        void* stream, const void* res, void* hout) {
  if (!x || !w || !y || !rstd || rows < 0 || H <= 0) return PRL_E_INVALID;
  if (H % 8 || H > 64 * 8 * kMaxNV || !a16(x) || !a16(w) || !a16(y)) return PRL_E_UNSUPPORTED;
  if (res && (!a16(res) || !a16(hout))) return PRL_E_UNSUPPORTED;
  if (rows == 0) return PRL_OK;
  const int nv = (int)((H / 8 + 63) / 64);
  const int64_t g = (rows + 3) / 4;
  const int grid = (int)(g < PRL_NORM_FWD_GRID ? g : PRL_NORM_FWD_GRID);
  return (int)norm_fwd_table(nv, x, w, y, rstd, rows, (int)H, eps, grid, static_cast<hipStream_t>(stream), res, hout,
                             std::make_integer_sequence<int, kMaxNV>{});
}

static int norm_backward(const void* dy, const void* x, const void* w, const float* rstd, void* dx, void* dw,
                         void* workspace, size_t workspace_bytes, int64_t rows, int64_t H, void* stream,
                         const void* dres) {
  if (!dy || !x || !w || !rstd || !dx || !dw || !workspace || rows < 0 || H <= 0) return PRL_E_INVALID;
  if (H % 8 || H > 64 * 8 * kMaxNVBwd || !a16(x) || !a16(w) || !a16(dy) || !a16(dx)) return PRL_E_UNSUPPORTED;
  if (dres && !a16(dres)) return PRL_E_UNSUPPORTED;
  if (workspace_bytes < sizeof(float) * (size_t)(kNormBlocks + kDwSlices) * (size_t)H) return PRL_E_WORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nv = (int)((H / 8 + 63) / 64);
  const int64_t g = (rows + 3) / 4;
  // the LDS-accumulator kernel holds two workgroups per CU: one resident round is 2 x 256
  const int cap = (PRL_NORM_BWD_LDS && nv > 4 && nv <= 8) ? PRL_NORM_LDS_GRID : PRL_NORM_GRID;
  const int grid = (int)(g < cap ? (g > 0 ? g : 1) : cap);
  float* partial = static_cast<float*>(workspace);
  hipError_t e = norm_bwd_table(nv, dy, x, w, rstd, dx, partial, rows, (int)H, grid, s, dres,
                                std::make_integer_sequence<int, kMaxNVBwd>{});
  if (e != hipSuccess) return (int)e;
  float* mid = partial + (size_t)kNormBlocks * (size_t)H;
  hipLaunchKernelGGL(rmsnorm_dw_stage1, dim3((unsigned)((H + 63) / 64), kDwSlices), dim3(256), 0, s, partial, grid,
                     (int)H, mid);
  hipLaunchKernelGGL(rmsnorm_dw_stage2, dim3((unsigned)((H + 255) / 256)), dim3(256), 0, s, mid, (int)H,
                     (uint16_t*)dw);
  return (int)hipGetLastError();
}

int prl_rmsnorm_forward(const void* x, const void* w, void* y, float* rstd, int64_t rows, int64_t H, float eps,
                        void* stream) {
  return norm_forward(x, w, y, rstd, rows, H, eps, stream, nullptr, nullptr);
}

int prl_add_rmsnorm_forward(const void* residual, const void* x, const void* w, void* h, void* y, float* rstd,
                            int64_t rows, int64_t H, float eps, void* stream) {
  if (!residual || !h) return PRL_E_INVALID;
  return norm_forward(x, w, y, rstd, rows, H, eps, stream, residual, h);
}

int prl_rmsnorm_backward(const void* dy, const void* x, const void* w, const float* rstd, void* dx, void* dw,
                         void* workspace, size_t workspace_bytes, int64_t rows, int64_t H, void* stream) {
  return norm_backward(dy, x, w, rstd, dx, dw, workspace, workspace_bytes, rows, H, stream, nullptr);
}

int prl_add_rmsnorm_backward(const void* dy, const void* dh, const void* h, const void* w, const float* rstd, void* dx,
                             void* dw, void* workspace, size_t workspace_bytes, int64_t rows, int64_t H, void* stream) {
  if (!dh) return PRL_E_INVALID;
  return norm_backward(dy, h, w, rstd, dx, dw, workspace, workspace_bytes, rows, H, stream, dh);
}

int prl_swiglu_forward(const void* gate, const void* up, void* out, int64_t n, uint32_t* counter, void* stream) {
  if (!gate || !up || !out || n < 0) return PRL_E_INVALID;
  if (n % 8 || !a16(gate) || !a16(up) || !a16(out)) return PRL_E_UNSUPPORTED;
  if (n == 0) return PRL_OK;
  const int64_t n8 = n / 8;
  if (PRL_SWIGLU_PHASED) {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t chunks = (n8 + 1024 * kPhFwdU - 1) / (1024 * kPhFwdU);
    const int grid = (int)(chunks < phased_grid(s) ? chunks : phased_grid(s));
    const hipError_t e = reset_counter(counter, s);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(swiglu_fwd_phased, dim3(grid), dim3(1024), 0, s,
                       (const u32x4*)gate, (const u32x4*)up, (u32x4*)out, n8, counter);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(swiglu_fwd, dim3(ew_grid(n8)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (const u32x4*)gate, (const u32x4*)up, (u32x4*)out, n8);
  return (int)hipGetLastError();
}

int prl_swiglu_backward(const void* dout, const void* gate, const void* up, void* dgate, void* dup, int64_t n,
                        uint32_t* counter, void* stream) {
  if (!dout || !gate || !up || !dgate || !dup || n < 0) return PRL_E_INVALID;
  if (n % 8 || !a16(dout) || !a16(gate) || !a16(up) || !a16(dgate) || !a16(dup)) return PRL_E_UNSUPPORTED;
  if (n == 0) return PRL_OK;
  const int64_t n8 = n / 8;
  if (PRL_SWIGLU_PHASED) {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t chunks = (n8 + 1024 * kPhBwdU - 1) / (1024 * kPhBwdU);
    const int grid = (int)(chunks < phased_grid(s) ? chunks : phased_grid(s));
    const hipError_t e = reset_counter(counter, s);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(swiglu_bwd_phased, dim3(grid), dim3(1024), 0, s,
                       (const u32x4*)dout, (const u32x4*)gate, (const u32x4*)up, (u32x4*)dgate, (u32x4*)dup, n8, counter);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(swiglu_bwd, dim3(ew_grid(n8)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (const u32x4*)dout, (const u32x4*)gate, (const u32x4*)up, (u32x4*)dgate, (u32x4*)dup, n8);
  return (int)hipGetLastError();
}

static int rows_grid(int64_t rows) { return (int)(rows < 2048 ? (rows > 0 ? rows : 1) : 2048); }

int prl_swiglu_forward_rows(const void* gate, const void* up, void* out, int64_t rows, int64_t cols, int64_t ld_gate,
                            int64_t ld_up, int64_t ld_out, void* stream) {
  if (!gate || !up || !out || rows < 0 || cols < 0 || ld_gate < cols || ld_up < cols || ld_out < cols)
    return PRL_E_INVALID;
  if (cols % 8 || ld_gate % 8 || ld_up % 8 || ld_out % 8 || !a16(gate) || !a16(up) || !a16(out) ||
      cols / 8 > 0x7FFFFFFF)
    return PRL_E_UNSUPPORTED;
  if (rows == 0 || cols == 0) return PRL_OK;
  if (PRL_SWIGLU_ROWS_PHASED) {
    const int64_t chunks = (rows * (cols / 8) + 1024 * kPhFwdU - 1) / (1024 * kPhFwdU);
    const int grid = (int)(chunks < phased_grid(static_cast<hipStream_t>(stream)) ? chunks
                                                                               : phased_grid(static_cast<hipStream_t>(stream)));
    hipLaunchKernelGGL(swiglu_fwd_rows_phased, dim3(grid), dim3(1024), 0, static_cast<hipStream_t>(stream),
                       (const u32x4*)gate, (const u32x4*)up, (u32x4*)out, rows, (int)(cols / 8), ld_gate / 8,
                       ld_up / 8, ld_out / 8);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(swiglu_fwd_rows, dim3(rows_grid(rows)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (const u32x4*)gate, (const u32x4*)up, (u32x4*)out, rows, (int)(cols / 8), ld_gate / 8, ld_up / 8,
                     ld_out / 8);
  return (int)hipGetLastError();
}

int prl_swiglu_backward_rows(const void* dout, const void* gate, const void* up, void* dgate, void* dup, int64_t rows,
                             int64_t cols, int64_t ld_dout, int64_t ld_gate, int64_t ld_up, int64_t ld_dgate,
                             int64_t ld_dup, void* stream) {
  if (!dout || !gate || !up || !dgate || !dup || rows < 0 || cols < 0 || ld_dout < cols || ld_gate < cols ||
      ld_up < cols || ld_dgate < cols || ld_dup < cols)
    return PRL_E_INVALID;
  if (cols % 8 || ld_dout % 8 || ld_gate % 8 || ld_up % 8 || ld_dgate % 8 || ld_dup % 8 || !a16(dout) ||
      !a16(gate) || !a16(up) || !a16(dgate) || !a16(dup) || cols / 8 > 0x7FFFFFFF)
    return PRL_E_UNSUPPORTED;
  if (rows == 0 || cols == 0) return PRL_OK;
  if (PRL_SWIGLU_ROWS_PHASED) {
    const int64_t chunks = (rows * (cols / 8) + 1024 * kPhBwdU - 1) / (1024 * kPhBwdU);
    const int grid = (int)(chunks < phased_grid(static_cast<hipStream_t>(stream)) ? chunks
                                                                               : phased_grid(static_cast<hipStream_t>(stream)));
    hipLaunchKernelGGL(swiglu_bwd_rows_phased, dim3(grid), dim3(1024), 0, static_cast<hipStream_t>(stream),
                       (const u32x4*)dout, (const u32x4*)gate, (const u32x4*)up, (u32x4*)dgate, (u32x4*)dup, rows,
                       (int)(cols / 8), ld_dout / 8, ld_gate / 8, ld_up / 8, ld_dgate / 8, ld_dup / 8);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(swiglu_bwd_rows, dim3(rows_grid(rows)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (const u32x4*)dout, (const u32x4*)gate, (const u32x4*)up, (u32x4*)dgate, (u32x4*)dup, rows,
                     (int)(cols / 8), ld_dout / 8, ld_gate / 8, ld_up / 8, ld_dgate / 8, ld_dup / 8);
  return (int)hipGetLastError();
}

static int rope_launch(int dir, const void* q, const void* k, const void* cs, const void* sn, void* qo, void* ko,
                       int64_t tokens, int32_t hq, int32_t hkv, int32_t d, void* stream, int64_t ldq = -1,
                       int64_t ldk = -1) {
  if (ldq < 0) ldq = (int64_t)hq * d;
  if (ldk < 0) ldk = (int64_t)hkv * d;
  if (!q || !k || !cs || !sn || !qo || !ko || tokens < 0 || hq <= 0 || hkv < 0 || d <= 0 || ldq < (int64_t)hq * d ||
      ldk < (int64_t)hkv * d)
    return PRL_E_INVALID;
  if (d % 8 || ldq % 4 || ldk % 4 || !a8(q) || !a8(k) || !a8(cs) || !a8(sn) || !a8(qo) || !a8(ko))
    return PRL_E_UNSUPPORTED;
  if (tokens == 0) return PRL_OK;
  const int64_t total = tokens * (int64_t)(hq + hkv) * (d / 8);
  const int64_t g = (total + 255) / 256;
  const int grid = (int)(g < 8192 ? g : 8192);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dir > 0)
    hipLaunchKernelGGL(rope_kernel<1>, dim3(grid), dim3(256), 0, s, (const uint16_t*)q, (const uint16_t*)k,
                       (const uint16_t*)cs, (const uint16_t*)sn, (uint16_t*)qo, (uint16_t*)ko, tokens, hq, hkv, d, ldq,
                       ldk);
  else
    hipLaunchKernelGGL(rope_kernel<-1>, dim3(grid), dim3(256), 0, s, (const uint16_t*)q, (const uint16_t*)k,
                       (const uint16_t*)cs, (const uint16_t*)sn, (uint16_t*)qo, (uint16_t*)ko, tokens, hq, hkv, d, ldq,
                       ldk);
  return (int)hipGetLastError();
}

int prl_rope_forward_strided(const void* q, const void* k, const void* cos, const void* sin, void* q_out,
                             void* k_out, int64_t tokens, int32_t hq, int32_t hkv, int32_t d, int64_t ld_q,
                             int64_t ld_k, void* stream) {
  return rope_launch(1, q, k, cos, sin, q_out, k_out, tokens, hq, hkv, d, stream, ld_q, ld_k);
}

int prl_rope_forward(const void* q, const void* k, const void* cos, const void* sin, void* q_out, void* k_out,
                     int64_t tokens, int32_t hq, int32_t hkv, int32_t d, void* stream) {
  return rope_launch(1, q, k, cos, sin, q_out, k_out, tokens, hq, hkv, d, stream);
}

int prl_rope_backward(const void* dq_out, const void* dk_out, const void* cos, const void* sin, void* dq, void* dk,
                      int64_t tokens, int32_t hq, int32_t hkv, int32_t d, void* stream) {
  return rope_launch(-1, dq_out, dk_out, cos, sin, dq, dk, tokens, hq, hkv, d, stream);
}

}  // extern "C"
