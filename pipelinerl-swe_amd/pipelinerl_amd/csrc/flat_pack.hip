// Weight-broadcast staging for MI355X: many parameter tensors <-> one flat bf16 buffer.
//
// Replaces the reference's per-parameter `parameter.data.bfloat16()` + one dist.broadcast
// per tensor (pipelinerl/finetune_loop.py:202-205, :246-247) and the actor's per-tensor
// receive buffers (pipelinerl/vllm1.py:84-93).  The trainer packs every parameter into
// one bf16 bucket buffer (HBM-bound, 16-B vector accesses, round-to-nearest-even), RCCL
// broadcasts large buckets, and the actor unpacks into its parameters.
//
// Launch shape: tensors are processed in groups of kGroup; blockIdx.y = tensor in group,
// blockIdx.x grid-strides over that tensor's elements (descriptor table passed by value,
// so no host->device copy and the launch is graph-capturable).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grpo_common.h"
#include "prl_hip.h"

namespace prl {

constexpr int kGroup = 32;

struct PackGroup {
  const void* src[kGroup];
  void* dst[kGroup];
  int64_t numel[kGroup];
  int64_t off[kGroup];
  int32_t dtype[kGroup];
  int32_t n;
};

__device__ __forceinline__ float load_as_f(const void* p, int dt, int64_t i) {
  return dt == PRL_F32 ? static_cast<const float*>(p)[i] : bf_to_f(static_cast<const uint16_t*>(p)[i]);
}

// flatten: group.src[i] (f32|bf16) -> flat bf16 at group.off[i]
__global__ __launch_bounds__(256) void flatten_bf16_kernel(PackGroup g, uint16_t* __restrict__ flat) {
  const int t = blockIdx.y;
  if (t >= g.n) return;
  const int64_t n = g.numel[t];
  const int dt = g.dtype[t];
  uint16_t* out = flat + g.off[t];
  const void* src = g.src[t];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool vec = ((g.off[t] & 7) == 0) && ((reinterpret_cast<uintptr_t>(src) & 15) == 0);
  int64_t done = 0;
  if (vec) {
    const int64_t nv = n >> 3;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
      u32x4 o;
      if (dt == PRL_BF16) {
        o = reinterpret_cast<const u32x4*>(src)[v];
      } else {
        const f32x4 a = reinterpret_cast<const f32x4*>(src)[2 * v];
        const f32x4 b = reinterpret_cast<const f32x4*>(src)[2 * v + 1];
        o[0] = pack_bf16x2(a[0], a[1]);
        o[1] = pack_bf16x2(a[2], a[3]);
        o[2] = pack_bf16x2(b[0], b[1]);
        o[3] = pack_bf16x2(b[2], b[3]);
      }
      reinterpret_cast<u32x4*>(out)[v] = o;
    }
    done = nv << 3;
  }
  for (int64_t i = done + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = dt == PRL_BF16 ? static_cast<const uint16_t*>(src)[i] : f_to_bf(static_cast<const float*>(src)[i]);
}

// unflatten: flat bf16 at group.off[i] -> group.dst[i] (f32|bf16)
__global__ __launch_bounds__(256) void unflatten_bf16_kernel(PackGroup g, const uint16_t* __restrict__ flat) {
  const int t = blockIdx.y;
  if (t >= g.n) return;
  const int64_t n = g.numel[t];
  const int dt = g.dtype[t];
  const uint16_t* in = flat + g.off[t];
  void* dst = g.dst[t];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool vec = ((g.off[t] & 7) == 0) && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
  int64_t done = 0;
  if (vec) {
    const int64_t nv = n >> 3;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
      const u32x4 x = reinterpret_cast<const u32x4*>(in)[v];
      if (dt == PRL_BF16) {
        reinterpret_cast<u32x4*>(dst)[v] = x;
      } else {
        f32x4 a = {bf_lo(x[0]), bf_hi(x[0]), bf_lo(x[1]), bf_hi(x[1])};
        f32x4 b = {bf_lo(x[2]), bf_hi(x[2]), bf_lo(x[3]), bf_hi(x[3])};
        reinterpret_cast<f32x4*>(dst)[2 * v] = a;
        reinterpret_cast<f32x4*>(dst)[2 * v + 1] = b;
      }
    }
    done = nv << 3;
  }
  for (int64_t i = done + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint16_t x = in[i];
    if (dt == PRL_BF16)
      static_cast<uint16_t*>(dst)[i] = x;
    else
      static_cast<float*>(dst)[i] = bf_to_f(x);
  }
}

// sum of squares, deterministic: block (x, t) of a group accumulates (double) a fixed grid-stride
// share of tensor t and writes its partial to part[(group * kGroup + t) * gridDim.x + x]; sqnorm_fold
// adds every partial in a fixed order.  No atomics: the bits do not depend on scheduling.
__global__ __launch_bounds__(256) void sqnorm_kernel(PackGroup g, double* __restrict__ part) {
  const int t = blockIdx.y;
  double acc = 0.0;
  if (t < g.n) {
    const int64_t n = g.numel[t];
    const int dt = g.dtype[t];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const float v = load_as_f(g.src[t], dt, i);
      acc += (double)v * (double)v;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double w[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) w[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)t * gridDim.x + blockIdx.x] = (w[0] + w[1]) + (w[2] + w[3]);
}

// one workgroup: thread i adds partials i, i + 256, ... in order, then a fixed tree
__global__ __launch_bounds__(256) void sqnorm_fold(const double* __restrict__ part, int64_t n, double* __restrict__ out) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) acc += part[i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double w[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) w[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out = (w[0] + w[1]) + (w[2] + w[3]);
}

// Gradient scale / accumulate for the fused lm_head's weight gradient (finetune/rl/fused_linear.py):
// t = bf16(float(src) * s) with s = *scale read on the device (no host sync); then dst = t, or
// dst = bf16(float(dst) + float(t)) (autograd's AccumulateGrad add of the two bf16 tensors, in one
// pass instead of a float() copy, a multiply, a cast and an add).  In place (dst == src, bf16, no
// accumulate) the kernel returns at once when s == 1: t = src exactly.
template <bool SRC_F32, bool ACC>
__global__ __launch_bounds__(256) void grad_scale_kernel(const void* __restrict__ src, const float* __restrict__ scale,
                                                         uint16_t* dst, int64_t n, int skip_if_one) {
  const float s = *scale;
  if (skip_if_one && s == 1.0f) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nv = n >> 3;
  auto one = [&](float x, uint16_t d) -> uint16_t {
    const float t = bf_to_f(f_to_bf(x * s));
    return ACC ? f_to_bf(bf_to_f(d) + t) : f_to_bf(t);
  };
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    float x[8];
    if (SRC_F32) {
      const f32x4 a = reinterpret_cast<const f32x4*>(src)[2 * v], b = reinterpret_cast<const f32x4*>(src)[2 * v + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = a[j];
        x[4 + j] = b[j];
      }
    } else {
      const u32x4 a = reinterpret_cast<const u32x4*>(src)[v];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = bf_lo(a[j]);
        x[2 * j + 1] = bf_hi(a[j]);
      }
    }
    u32x4 d = ACC ? reinterpret_cast<const u32x4*>(dst)[v] : u32x4{0, 0, 0, 0};
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint16_t lo = one(x[2 * j], (uint16_t)(d[j] & 0xffffu)), hi = one(x[2 * j + 1], (uint16_t)(d[j] >> 16));
      o[j] = (uint32_t)lo | ((uint32_t)hi << 16);
    }
    reinterpret_cast<u32x4*>(dst)[v] = o;
  }
  for (int64_t i = (nv << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = SRC_F32 ? static_cast<const float*>(src)[i] : bf_to_f(static_cast<const uint16_t*>(src)[i]);
    dst[i] = one(x, ACC ? dst[i] : (uint16_t)0);
  }
}

static int grid_x_for(const PackGroup& g) {
  int64_t mx = 1;
  for (int i = 0; i < g.n; ++i) mx = g.numel[i] > mx ? g.numel[i] : mx;
  int64_t blocks = (mx / 8 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  return (int)blocks;
}

// Measurement helper (bench snapshot_overlap): the reads an RCCL broadcast root makes of the
// parameters it sends, emulated on one GPU with no receiver.  `blocks` workgroups of 256 threads (the
// communicator's channels: one workgroup per channel, each on its own CU for the whole transfer)
// stream the buffer with nontemporal 16-B loads, each paced against the realtime clock (100 MHz)
// to its share of `gbps`, the link rate the root sends at (one xGMI link ~153 GB/s).  What it
// costs the trainer step running beside it is the contention the zero-copy broadcast adds: CUs
// held and HBM read while the step's kernels run.  The loaded data is folded per thread and
// compared with a run-time key (a store only on a match), so the loads cannot be removed.
__global__ __launch_bounds__(256) void paced_read_kernel(const u32x4* __restrict__ src, int64_t nvec,
                                                         double vec_per_tick, uint32_t* sink, uint32_t key) {
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t a = (int64_t)blockIdx.x * per;
  const int64_t b = a + per < nvec ? a + per : nvec;
  constexpr int U = 16;  // 16 vectors per thread in flight: 64 KiB per workgroup per turn
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  int64_t done = 0;
  for (int64_t v = a + threadIdx.x; v < b; v += (int64_t)U * 256) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = v + (int64_t)u * 256;
      x[u] = i < b ? __builtin_nontemporal_load(src + i) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u][0] ^ x[u][1] ^ x[u][2] ^ x[u][3];
    done += (int64_t)U * 256;
    // wait until this workgroup's share of the link rate has caught up with what it has read: the
    // clock is read once per turn (a realtime read is a message to a chip-wide counter: polling it
    // in a tight loop delayed every other kernel's start), the wait itself is counted sleeps
    const uint64_t due = t0 + (uint64_t)((double)done / vec_per_tick);
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (now < due) {
      // s_sleep 127 ~ 127 x 64 cycles ~ 3.4-3.9 us at 2.1-2.4 GHz; a realtime tick is 10 ns
      for (int64_t k = (int64_t)(due - now) / 400; k > 0; --k) __builtin_amdgcn_s_sleep(127);
    }
  }
  if (acc == key) sink[blockIdx.x] = acc;  // depends on every load: they stay (almost never stores)
}

}  // namespace prl

using namespace prl;

extern "C" {

int prl_flatten_bf16(const void* const* srcs, const int32_t* dtypes, const int64_t* numels,
                     const int64_t* dst_offsets, int32_t n, void* dst, void* stream) {
  if (n < 0 || (n > 0 && (!srcs || !dtypes || !numels || !dst_offsets || !dst))) return PRL_E_INVALID;
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int base = 0; base < n; base += kGroup) {
    PackGroup g{};
    g.n = (n - base) < kGroup ? (n - base) : kGroup;
    for (int i = 0; i < g.n; ++i) {
      if (dtypes[base + i] != PRL_F32 && dtypes[base + i] != PRL_BF16) return PRL_E_UNSUPPORTED;
      if (numels[base + i] < 0 || dst_offsets[base + i] < 0) return PRL_E_INVALID;
      g.src[i] = srcs[base + i];
      g.dtype[i] = dtypes[base + i];
      g.numel[i] = numels[base + i];
      g.off[i] = dst_offsets[base + i];
    }
    hipLaunchKernelGGL(flatten_bf16_kernel, dim3(grid_x_for(g), g.n), dim3(256), 0, s, g,
                       static_cast<uint16_t*>(dst));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return PRL_OK;
}

int prl_unflatten_bf16(const void* src, void* const* dsts, const int32_t* dtypes, const int64_t* numels,
                       const int64_t* src_offsets, int32_t n, void* stream) {
  if (n < 0 || (n > 0 && (!src || !dsts || !dtypes || !numels || !src_offsets))) return PRL_E_INVALID;
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int base = 0; base < n; base += kGroup) {
    PackGroup g{};
    g.n = (n - base) < kGroup ? (n - base) : kGroup;
    for (int i = 0; i < g.n; ++i) {
      if (dtypes[base + i] != PRL_F32 && dtypes[base + i] != PRL_BF16) return PRL_E_UNSUPPORTED;
      if (numels[base + i] < 0 || src_offsets[base + i] < 0) return PRL_E_INVALID;
      g.dst[i] = dsts[base + i];
      g.dtype[i] = dtypes[base + i];
      g.numel[i] = numels[base + i];
      g.off[i] = src_offsets[base + i];
    }
    hipLaunchKernelGGL(unflatten_bf16_kernel, dim3(grid_x_for(g), g.n), dim3(256), 0, s, g,
                       static_cast<const uint16_t*>(src));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return PRL_OK;
}

int prl_grad_scale_bf16(const void* src, int32_t src_dtype, const float* scale, void* dst, int64_t n,
                        int32_t accumulate, void* stream) {
  if (!src || !scale || !dst || n < 0) return PRL_E_INVALID;
  if (src_dtype != PRL_F32 && src_dtype != PRL_BF16) return PRL_E_UNSUPPORTED;
  if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15)) return PRL_E_INVALID;
  if (n == 0) return PRL_OK;
  const bool f32 = src_dtype == PRL_F32;
  const int skip = !accumulate && !f32 && src == dst;
  int64_t blocks = (n / 8 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint16_t* d = static_cast<uint16_t*>(dst);
  if (f32 && accumulate)
    hipLaunchKernelGGL((grad_scale_kernel<true, true>), dim3((unsigned)blocks), dim3(256), 0, s, src, scale, d, n, skip);
  else if (f32)
    hipLaunchKernelGGL((grad_scale_kernel<true, false>), dim3((unsigned)blocks), dim3(256), 0, s, src, scale, d, n, skip);
  else if (accumulate)
    hipLaunchKernelGGL((grad_scale_kernel<false, true>), dim3((unsigned)blocks), dim3(256), 0, s, src, scale, d, n, skip);
  else
    hipLaunchKernelGGL((grad_scale_kernel<false, false>), dim3((unsigned)blocks), dim3(256), 0, s, src, scale, d, n, skip);
  return (int)hipGetLastError();
}

int prl_grad_sqnorm(const void* const* srcs, const int32_t* dtypes, const int64_t* numels, int32_t n,
                    double* out, void* workspace, size_t workspace_bytes, void* stream) {
  if (!out || n < 0 || (n > 0 && (!srcs || !dtypes || !numels))) return PRL_E_INVALID;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n == 0) return (int)hipMemsetAsync(out, 0, sizeof(double), s);
  // one partial per (tensor, block): a fixed kSqBlocks blocks per tensor, so the layout (and the
  // summation order) depends only on n
  constexpr int kSqBlocks = 256;
  const size_t need = sizeof(double) * (size_t)n * kSqBlocks;
  double* part = static_cast<double*>(workspace);
  if (!part || workspace_bytes < need) return PRL_E_WORKSPACE;
  for (int base = 0; base < n; base += kGroup) {
    PackGroup g{};
    g.n = (n - base) < kGroup ? (n - base) : kGroup;
    for (int i = 0; i < g.n; ++i) {
      if (dtypes[base + i] != PRL_F32 && dtypes[base + i] != PRL_BF16) return PRL_E_UNSUPPORTED;
      g.src[i] = srcs[base + i];
      g.dtype[i] = dtypes[base + i];
      g.numel[i] = numels[base + i];
    }
    hipLaunchKernelGGL(sqnorm_kernel, dim3(kSqBlocks, g.n), dim3(256), 0, s, g, part + (size_t)base * kSqBlocks);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(sqnorm_fold, dim3(1), dim3(256), 0, s, part, (int64_t)n * kSqBlocks, out);
  return (int)hipGetLastError();
}

int prl_paced_read(const void* src, int64_t bytes, double gbps, int32_t blocks, uint32_t* sink, void* stream) {
  // sink: a word per workgroup, written only when a thread's folded data equals the key
  if (!src || !sink || bytes < 0 || !(gbps > 0.0) || blocks < 1 || blocks > 1024) return PRL_E_INVALID;
  if (reinterpret_cast<uintptr_t>(src) & 15) return PRL_E_INVALID;
  const int64_t nvec = bytes / 16;
  if (nvec == 0) return PRL_OK;
  // 16-B vectors per realtime tick (10 ns) and workgroup
  const double vec_per_tick = gbps * 1e9 / 16.0 / 1e8 / (double)blocks;
  hipLaunchKernelGGL(paced_read_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x4*>(src), nvec, vec_per_tick, sink, 0x9E3779B9u);
  return (int)hipGetLastError();
}

}  // extern "C"
