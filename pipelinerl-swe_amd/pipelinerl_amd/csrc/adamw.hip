// The trainer's optimizer step on MI355X: AdamW over every parameter with the gradient-clipping
// scale applied on the fly.
//
// Replaces, at the optimizer-step boundary of the DP step (pipelinerl/finetune_loop.py:700-719:
// clip_grad_norm_ then optimizer.step()), torch's
//   torch._foreach_mul_(grads, clip_coef)          one read + one write of every gradient
//   torch._fused_adamw_(params, grads, m, v, ...)  launched 320 blocks at a time (65 536-element
//                                                  chunks: ~360 launches for a 7B model)
// with one pass that reads p, g, m, v and writes p, m, v once (14 B per bf16 parameter), in
// launches of 32 tensors whose blocks grid-stride over each tensor with 16-B accesses.
//
// The arithmetic is torch's fused AdamW (ATen/native/cuda/fused_adam_utils.cuh, adam_math,
// ADAMW mode) operation for operation, including which steps run in double: the same
// roundings, so the update is bit-identical (tests/test_adamw_gpu.py).  The clip multiply is
// foreach_mul_'s: g = T(float(g) * float(coef)), coef read on the device (no host sync).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grpo_common.h"
#include "prl_hip.h"

namespace prl {

constexpr int kAdamGroup = 32;

struct AdamWGroup {
  void* p[kAdamGroup];
  const void* g[kAdamGroup];
  void* m[kAdamGroup];
  void* v[kAdamGroup];
  const float* step[kAdamGroup];
  int64_t numel[kAdamGroup];
  int32_t n;
};

struct AdamWHyper {
  double lr, beta1, beta2, weight_decay, eps;
};

// one element: torch's adam_math (kParamIdx..kExpAvgSqIdx), float opmath, doubles where it has them.
// The multiply-adds are spelled out as the fused form torch's build contracts them to (measured
// element by element, tools/adamw_debug.py [round 1-3 tool, in git history]: beta1 m + (1 - beta1) g is fma(beta1, m, (1 - beta1) g),
// not fma(1 - beta1, g, beta1 m) as this compiler would choose); nothing else is contracted.
__device__ __forceinline__ void adamw_elem(float& param, float grad, float& exp_avg, float& exp_avg_sq,
                                           const AdamWHyper& h, float bias_correction1, float bias_correction2_sqrt) {
#pragma clang fp contract(off)
  if (h.weight_decay != 0) param = (float)__builtin_fma(-(h.lr * h.weight_decay), (double)param, (double)param);
  exp_avg = (float)__builtin_fma(h.beta1, (double)exp_avg, (1 - h.beta1) * grad);
  exp_avg_sq = (float)__builtin_fma(h.beta2, (double)exp_avg_sq, (1 - h.beta2) * grad * grad);
  const float step_size = h.lr / bias_correction1;
  const float denom = (sqrtf(exp_avg_sq) / bias_correction2_sqrt) + h.eps;
  param -= step_size * exp_avg / denom;
}

// T: uint16_t (bf16 parameters, gradients and moments) or float.  CLIP: multiply the gradient by
// *clip (a bf16 / float scalar of T's type) first, rounded to T as foreach_mul_ stores it.
template <typename T, bool CLIP>
__global__ __launch_bounds__(256) void adamw_kernel(AdamWGroup grp, AdamWHyper h, const T* __restrict__ clip) {
  const int t = blockIdx.y;
  if (t >= grp.n) return;
  const int64_t n = grp.numel[t];
  // torch: bias corrections in double from the float step count, then narrowed to float
  const float step = *grp.step[t];
  const float bc1 = (float)(1 - pow(h.beta1, (double)step));
  const float bc2s = (float)sqrt(1 - pow(h.beta2, (double)step));
  constexpr bool kBf = sizeof(T) == 2;
  auto ld = [](T x) -> float {
    if constexpr (kBf) return bf_to_f(x);
    else return x;
  };
  auto st = [](float x) -> T {
    if constexpr (kBf) return f_to_bf(x);
    else return x;
  };
  const float c = CLIP ? ld(*clip) : 1.f;
  auto grad_of = [&](float g) -> float { return CLIP ? ld(st(g * c)) : g; };
  T* P = static_cast<T*>(grp.p[t]);
  const T* G = static_cast<const T*>(grp.g[t]);
  T* M = static_cast<T*>(grp.m[t]);
  T* V = static_cast<T*>(grp.v[t]);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  constexpr int kE = 16 / sizeof(T);  // elements per 16-B vector
  const bool vec = !((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) |
                      reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V)) & 15);
  int64_t done = 0;
  if (vec) {
    const int64_t nv = n / kE;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
      u32x4 pv = reinterpret_cast<const u32x4*>(P)[i], gv = reinterpret_cast<const u32x4*>(G)[i];
      u32x4 mv = reinterpret_cast<const u32x4*>(M)[i], vv = reinterpret_cast<const u32x4*>(V)[i];
      T* pe = reinterpret_cast<T*>(&pv);
      const T* ge = reinterpret_cast<const T*>(&gv);
      T* me = reinterpret_cast<T*>(&mv);
      T* ve = reinterpret_cast<T*>(&vv);
#pragma unroll
      for (int j = 0; j < kE; ++j) {
        float p = ld(pe[j]), m = ld(me[j]), v = ld(ve[j]);
        adamw_elem(p, grad_of(ld(ge[j])), m, v, h, bc1, bc2s);
        pe[j] = st(p);
        me[j] = st(m);
        ve[j] = st(v);
      }
      reinterpret_cast<u32x4*>(P)[i] = pv;
      reinterpret_cast<u32x4*>(M)[i] = mv;
      reinterpret_cast<u32x4*>(V)[i] = vv;
    }
    done = nv * kE;
  }
  for (int64_t i = done + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float p = ld(P[i]), m = ld(M[i]), v = ld(V[i]);
    adamw_elem(p, grad_of(ld(G[i])), m, v, h, bc1, bc2s);
    P[i] = st(p);
    M[i] = st(m);
    V[i] = st(v);
  }
}

static int adamw_grid_x(const AdamWGroup& g, int elems_per_vec) {
  int64_t mx = 1;
  for (int i = 0; i < g.n; ++i) mx = g.numel[i] > mx ? g.numel[i] : mx;
  int64_t blocks = (mx / elems_per_vec + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  return (int)blocks;
}

template <typename T>
static hipError_t adamw_launch(const AdamWGroup& g, const AdamWHyper& h, const void* clip, hipStream_t s) {
  const dim3 grid(adamw_grid_x(g, 16 / (int)sizeof(T)), g.n);
  if (clip)
    hipLaunchKernelGGL((adamw_kernel<T, true>), grid, dim3(256), 0, s, g, h, static_cast<const T*>(clip));
  else
    hipLaunchKernelGGL((adamw_kernel<T, false>), grid, dim3(256), 0, s, g, h, static_cast<const T*>(nullptr));
  return hipGetLastError();
}

// ---- fp32 master weights -----------------------------------------------------------------------
// The optimizer state of the reference's default backends: DeepSpeed's bf16 ZeRO optimizer
// (conf/deepspeed/deepspeed_stage3_bf16.json) and accelerate's FSDP mixed precision both update an
// fp32 copy of every weight with fp32 AdamW moments and hand the model a bf16 rounding of it.  At the
// reference's lr (5e-7, conf/finetune/base.yaml) a bf16 weight cannot hold such an update: it is far
// below half a bf16 ulp and rounds away.
//
// One pass per element: read the bf16 (or fp32) gradient, the fp32 master, exp_avg, exp_avg_sq;
// write the fp32 master, exp_avg, exp_avg_sq and the bf16 parameter (round-to-nearest-even of the
// new master) — 14 B read + 14 B written per parameter with bf16 gradients.  The bf16 parameter is
// written in place, so the flat parameter buffer the weight broadcast reads stays the model's.
//
// Work split: every launch covers up to kMasterGroup tensors, cut into kMasterChunk-element chunks,
// one workgroup per chunk (first_block[t] = the first workgroup of tensor t): every workgroup moves
// the same bytes, whatever the tensor sizes, and a 7B model's 339 tensors take 11 launches.
// Per lane, units of 4 elements: one 16-B load of each fp32 stream and one 8-B load of each bf16
// stream, consecutive lanes on consecutive units (each instruction covers one contiguous span).
#ifndef PRL_ADAMW_UNROLL  // 4 units per lane (90 VGPRs: 5 waves per SIMD instead of 3 at 8):
#define PRL_ADAMW_UNROLL 4   // 36.2 vs 37.4 ms per 7B step with nontemporal streams, three alternated
#endif                       // rounds (profiles/r06_adamw_unroll_ab.jsonl)
#ifndef PRL_ADAMW_NT  // nontemporal fp32 loads (1) / stores (2) in whole chunks: 3 measured best
#define PRL_ADAMW_NT 3   // (7B: 37.3 ms vs 38.6 ms plain, profiles/r06_adamw_master_ab.jsonl)
#endif
constexpr int kMasterGroup = 32;
constexpr int kMasterUnroll = PRL_ADAMW_UNROLL;            // units per lane in flight
constexpr int kMasterChunk = 256 * 4 * kMasterUnroll;      // elements per workgroup

struct AdamWMasterGroup {
  void* p[kMasterGroup];          // bf16 parameters (written)
  const void* g[kMasterGroup];    // gradients, bf16 or fp32
  float* w[kMasterGroup];         // fp32 master weights
  float* m[kMasterGroup];
  float* v[kMasterGroup];
  const float* step[kMasterGroup];
  int64_t numel[kMasterGroup];
  int32_t first_block[kMasterGroup + 1];
  int32_t aligned[kMasterGroup];  // 1: every stream of tensor t aligned for the vector path
  int32_t n;
};

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <bool GBF16>
__device__ __forceinline__ f32x4 load_grad4(const void* G, int64_t i) {
  if constexpr (GBF16) {
    const u32x2 r = *reinterpret_cast<const u32x2*>(static_cast<const uint16_t*>(G) + i);
    return f32x4{bf_lo(r.x), bf_hi(r.x), bf_lo(r.y), bf_hi(r.y)};
  } else {
    return *reinterpret_cast<const f32x4*>(static_cast<const float*>(G) + i);
  }
}

template <bool GBF16>
__device__ __forceinline__ float load_grad1(const void* G, int64_t i) {
  if constexpr (GBF16) return bf_to_f(static_cast<const uint16_t*>(G)[i]);
  else return static_cast<const float*>(G)[i];
}

template <bool GBF16, bool CLIP>
__global__ __launch_bounds__(256) void adamw_master_kernel(AdamWMasterGroup grp, AdamWHyper h,
                                                           const float* __restrict__ clip) {
  const int b = blockIdx.x;
  int t = 0;  // uniform: the tensor whose chunks include workgroup b
  for (int i = 1; i < grp.n; ++i) t += b >= grp.first_block[i];
  const int64_t n = grp.numel[t];
  const int64_t lo = (int64_t)(b - grp.first_block[t]) * kMasterChunk;
  const int64_t hi = lo + kMasterChunk < n ? lo + kMasterChunk : n;
  const float step = *grp.step[t];
  const float bc1 = (float)(1 - pow(h.beta1, (double)step));
  const float bc2s = (float)sqrt(1 - pow(h.beta2, (double)step));
  // the clip multiply on the fp32 gradient (DeepSpeed / torch clip_grad_norm_ on fp32 gradients)
  const float c = CLIP ? *clip : 1.f;
  uint16_t* P = static_cast<uint16_t*>(grp.p[t]);
  const void* G = grp.g[t];
  float* W = grp.w[t];
  float* M = grp.m[t];
  float* V = grp.v[t];
  int64_t done = lo;
  if (grp.aligned[t]) {
    const int64_t units = (hi - lo) >> 2;  // whole 4-element units in this chunk
    const int64_t full = units >= 256 * kMasterUnroll ? kMasterUnroll : 0;
    if (full) {  // the common case: a whole chunk, every load issued before the first use
      f32x4 g[kMasterUnroll], w[kMasterUnroll], m[kMasterUnroll], v[kMasterUnroll];
#pragma unroll
      for (int k = 0; k < kMasterUnroll; ++k) {
        const int64_t i = lo + 4 * ((int64_t)k * 256 + threadIdx.x);
        g[k] = load_grad4<GBF16>(G, i);
#if PRL_ADAMW_NT & 1
        w[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(W + i));
        m[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(M + i));
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(V + i));
#else
        w[k] = *reinterpret_cast<const f32x4*>(W + i);
        m[k] = *reinterpret_cast<const f32x4*>(M + i);
        v[k] = *reinterpret_cast<const f32x4*>(V + i);
#endif
      }
#pragma unroll
      for (int k = 0; k < kMasterUnroll; ++k) {
        const int64_t i = lo + 4 * ((int64_t)k * 256 + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float wj = w[k][j], mj = m[k][j], vj = v[k][j];
          adamw_elem(wj, CLIP ? g[k][j] * c : g[k][j], mj, vj, h, bc1, bc2s);
          w[k][j] = wj;
          m[k][j] = mj;
          v[k][j] = vj;
        }
#if PRL_ADAMW_NT & 2
        __builtin_nontemporal_store(w[k], reinterpret_cast<f32x4*>(W + i));
        __builtin_nontemporal_store(m[k], reinterpret_cast<f32x4*>(M + i));
        __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(V + i));
        __builtin_nontemporal_store(u32x2{pack_bf16x2(w[k][0], w[k][1]), pack_bf16x2(w[k][2], w[k][3])},
                                    reinterpret_cast<u32x2*>(P + i));
#else
        *reinterpret_cast<f32x4*>(W + i) = w[k];
        *reinterpret_cast<f32x4*>(M + i) = m[k];
        *reinterpret_cast<f32x4*>(V + i) = v[k];
        *reinterpret_cast<u32x2*>(P + i) = u32x2{pack_bf16x2(w[k][0], w[k][1]), pack_bf16x2(w[k][2], w[k][3])};
#endif
      }
      done = hi;
    } else {  // a tensor's last, partial chunk: whole units, then the scalar tail below
      for (int64_t u = threadIdx.x; u < units; u += 256) {
        const int64_t i = lo + 4 * u;
        const f32x4 gg = load_grad4<GBF16>(G, i);
        f32x4 ww = *reinterpret_cast<const f32x4*>(W + i);
        f32x4 mm = *reinterpret_cast<const f32x4*>(M + i);
        f32x4 vv = *reinterpret_cast<const f32x4*>(V + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float wj = ww[j], mj = mm[j], vj = vv[j];
          adamw_elem(wj, CLIP ? gg[j] * c : gg[j], mj, vj, h, bc1, bc2s);
          ww[j] = wj;
          mm[j] = mj;
          vv[j] = vj;
        }
        *reinterpret_cast<f32x4*>(W + i) = ww;
        *reinterpret_cast<f32x4*>(M + i) = mm;
        *reinterpret_cast<f32x4*>(V + i) = vv;
        *reinterpret_cast<u32x2*>(P + i) = u32x2{pack_bf16x2(ww[0], ww[1]), pack_bf16x2(ww[2], ww[3])};
      }
      done = lo + 4 * units;
    }
  }
  for (int64_t i = done + threadIdx.x; i < hi; i += 256) {  // misaligned tensors and tails
    float w = W[i], m = M[i], v = V[i];
    const float g = load_grad1<GBF16>(G, i);
    adamw_elem(w, CLIP ? g * c : g, m, v, h, bc1, bc2s);
    W[i] = w;
    M[i] = m;
    V[i] = v;
    P[i] = f_to_bf(w);
  }
}

template <bool GBF16>
static hipError_t adamw_master_launch(const AdamWMasterGroup& g, const AdamWHyper& h, const float* clip,
                                      hipStream_t s) {
  const int blocks = g.first_block[g.n];
  if (blocks == 0) return hipSuccess;
  if (clip)
    hipLaunchKernelGGL((adamw_master_kernel<GBF16, true>), dim3(blocks), dim3(256), 0, s, g, h, clip);
  else
    hipLaunchKernelGGL((adamw_master_kernel<GBF16, false>), dim3(blocks), dim3(256), 0, s, g, h, clip);
  return hipGetLastError();
}

}  // namespace prl

using namespace prl;

extern "C" {

int prl_adamw_master_step(int32_t n, void* const* params, const void* const* grads, float* const* masters,
                          float* const* exp_avgs, float* const* exp_avg_sqs, const float* const* steps,
                          const int64_t* numels, int32_t grad_dtype, double lr, double beta1, double beta2,
                          double weight_decay, double eps, const float* grad_scale, void* stream) {
  if (n < 0 || (n > 0 && (!params || !grads || !masters || !exp_avgs || !exp_avg_sqs || !steps || !numels)))
    return PRL_E_INVALID;
  if (grad_dtype != PRL_BF16 && grad_dtype != PRL_F32) return PRL_E_UNSUPPORTED;
  for (int j = 0; j < n; ++j)  // every entry checked before the first launch: all tensors step, or none
    if (numels[j] < 0 || (numels[j] > 0 && (!params[j] || !grads[j] || !masters[j] || !exp_avgs[j] ||
                                            !exp_avg_sqs[j])) || !steps[j] ||
        (numels[j] + kMasterChunk - 1) / kMasterChunk > (int64_t)1 << 30)
      return PRL_E_INVALID;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const AdamWHyper h{lr, beta1, beta2, weight_decay, eps};
  const uintptr_t galign = grad_dtype == PRL_BF16 ? 7 : 15;
  int j = 0;
  while (j < n) {
    AdamWMasterGroup g{};
    int64_t blocks = 0;
    // up to kMasterGroup tensors, and at most 2^30 workgroups, per launch
    while (j < n && g.n < kMasterGroup) {
      const int64_t nb = (numels[j] + kMasterChunk - 1) / kMasterChunk;
      if (g.n > 0 && blocks + nb > ((int64_t)1 << 30)) break;
      const int i = g.n++;
      g.p[i] = params[j];
      g.g[i] = grads[j];
      g.w[i] = masters[j];
      g.m[i] = exp_avgs[j];
      g.v[i] = exp_avg_sqs[j];
      g.step[i] = steps[j];
      g.numel[i] = numels[j];
      g.first_block[i] = (int32_t)blocks;
      g.aligned[i] = !((reinterpret_cast<uintptr_t>(params[j]) & 7) | (reinterpret_cast<uintptr_t>(grads[j]) & galign) |
                       ((reinterpret_cast<uintptr_t>(masters[j]) | reinterpret_cast<uintptr_t>(exp_avgs[j]) |
                         reinterpret_cast<uintptr_t>(exp_avg_sqs[j])) & 15));
      blocks += nb;
      ++j;
    }
    g.first_block[g.n] = (int32_t)blocks;
    for (int i = g.n + 1; i <= kMasterGroup; ++i) g.first_block[i] = (int32_t)blocks;
    const hipError_t e = grad_dtype == PRL_BF16 ? adamw_master_launch<true>(g, h, grad_scale, s)
                                                : adamw_master_launch<false>(g, h, grad_scale, s);
    if (e != hipSuccess) return (int)e;
  }
  return PRL_OK;
}

int prl_adamw_step(int32_t n, void* const* params, const void* const* grads, void* const* exp_avgs,
                   void* const* exp_avg_sqs, const float* const* steps, const int64_t* numels, int32_t dtype,
                   double lr, double beta1, double beta2, double weight_decay, double eps, const void* grad_scale,
                   void* stream) {
  if (n < 0 || (n > 0 && (!params || !grads || !exp_avgs || !exp_avg_sqs || !steps || !numels))) return PRL_E_INVALID;
  if (dtype != PRL_BF16 && dtype != PRL_F32) return PRL_E_UNSUPPORTED;
  for (int j = 0; j < n; ++j)  // every entry checked before the first launch: all tensors step, or none
    if (numels[j] < 0 || (numels[j] > 0 && (!params[j] || !grads[j] || !exp_avgs[j] || !exp_avg_sqs[j])) ||
        !steps[j])
      return PRL_E_INVALID;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const AdamWHyper h{lr, beta1, beta2, weight_decay, eps};
  for (int base = 0; base < n; base += kAdamGroup) {
    AdamWGroup g{};
    g.n = (n - base) < kAdamGroup ? (n - base) : kAdamGroup;
    for (int i = 0; i < g.n; ++i) {
      const int j = base + i;
      g.p[i] = params[j];
      g.g[i] = grads[j];
      g.m[i] = exp_avgs[j];
      g.v[i] = exp_avg_sqs[j];
      g.step[i] = steps[j];
      g.numel[i] = numels[j];
    }
    const hipError_t e = dtype == PRL_BF16 ? adamw_launch<uint16_t>(g, h, grad_scale, s)
                                           : adamw_launch<float>(g, h, grad_scale, s);
    if (e != hipSuccess) return (int)e;
  }
  return PRL_OK;
}

}  // extern "C"
