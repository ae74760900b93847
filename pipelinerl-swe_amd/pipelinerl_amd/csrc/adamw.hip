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

}  // namespace prl

using namespace prl;

extern "C" {

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
