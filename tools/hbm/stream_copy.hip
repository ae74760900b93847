// HBM streaming ceiling probe (not part of the product): read N bytes, write N bytes, 16 B per
// lane, the same 50/50 read/write mix as the loss head (logits in, dlogits out).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, int AUX>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = AUX ? __builtin_nontemporal_load(in + i + u * stride) : in[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (AUX) __builtin_nontemporal_store(v[u], out + i + u * stride);
      else out[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) out[i] = in[i];
}

// read-only: fold 16-B loads into one word per thread (written once, ~0 bytes)
template <int UNROLL>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ in, uint32_t* __restrict__ sink, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(in + i + u * stride);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads alive; practically never stores
}

// write-only: 16-B nontemporal stores of a constant
__global__ __launch_bounds__(256) void write_kernel(u32x4* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const u32x4 z = {0u, 1u, 2u, 3u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) __builtin_nontemporal_store(z, out + i);
}

extern "C" int probe_copy(const void* in, void* out, int64_t bytes, int grid, int variant, void* stream) {
  const int64_t n = bytes / 16;
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL((copy_kernel<4, 0>), dim3(grid), dim3(256), 0, s, (const u32x4*)in, (u32x4*)out, n); break;
    case 1: hipLaunchKernelGGL((copy_kernel<4, 1>), dim3(grid), dim3(256), 0, s, (const u32x4*)in, (u32x4*)out, n); break;
    case 2: hipLaunchKernelGGL((copy_kernel<8, 1>), dim3(grid), dim3(256), 0, s, (const u32x4*)in, (u32x4*)out, n); break;
    case 3: hipLaunchKernelGGL((read_kernel<8>), dim3(grid), dim3(256), 0, s, (const u32x4*)in, (uint32_t*)out, n); break;
    case 4: hipLaunchKernelGGL((write_kernel), dim3(grid), dim3(256), 0, s, (u32x4*)out, n); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}
