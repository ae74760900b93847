// Read/write phasing probe (measurement tool, not product).  The loss head reads a 297 KB logits
// row into a 1024-thread workgroup's registers and writes the 297 KB dlogits row while the next
// row streams in, one workgroup per CU: HBM sees reads and writes mixed all the time, and the
// 20 GB in / 20 GB out copy it is bound by runs at ~5.3 TB/s while reads alone reach ~6.8 and
// writes alone ~6.0 TB/s.  Does separating the two directions in time help?
//   overlap   the loss head's schedule: store vector k of row r, then load vector k of row r+1
//   phased    load the whole row, wait, store the whole row, wait (vmcnt(0): stores retired), next
//   sync<K>   phased, plus a grid-wide soft barrier every K rows so every CU reads (and then
//             writes) at the same time; bounded spin (falls through after ~2^20 polls), so the
//             grid always drains even if a workgroup is not resident
//   *_inplace the same schedules writing each row back over itself (out == in)
// One JSON line per variant (ms per 20 GB copy, GB/s counting read + write).
//   hipcc -O3 --offload-arch=gfx950 tools/hbm/phased_copy.hip -o tools/hbm/phased_copy.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int NV = 19;        // 16-B vectors per thread per row (the loss head's NV at V = 151 936)
constexpr int THREADS = 1024;
constexpr int64_t ROW_WORDS = 18992;  // 151 936 bf16 = 303 872 B = 18 992 16-B words

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ u32x4 ld(const u32x4* p, int64_t i, int64_t lim) {
  return i < lim ? __builtin_nontemporal_load(p + i) : u32x4{0, 0, 0, 0};
}
__device__ __forceinline__ void st(u32x4* p, int64_t i, int64_t lim, u32x4 v) {
  if (i < lim) __builtin_nontemporal_store(v, p + i);
}

__device__ __forceinline__ void grid_sync(unsigned* ctr, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int spin = 0; spin < (1 << 20); ++spin) {
      if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// MODE 0 overlap, 1 phased, 2 phased + grid sync every `K` rows
template <int MODE>
__global__ __launch_bounds__(THREADS) void rowcopy(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                    int64_t nrows, unsigned* ctr, int K) {
  const int t = threadIdx.x;
  const int64_t G = gridDim.x;
  u32x4 buf[NV];
  int64_t r = blockIdx.x;
  if (r >= nrows) return;
  const u32x4* src = in + r * ROW_WORDS;
#pragma unroll
  for (int k = 0; k < NV; ++k) buf[k] = ld(src, t + k * THREADS, ROW_WORDS);
  unsigned epoch = 0;
  for (int64_t it = 0;; ++it, r += G) {
    const int64_t rn = r + G;
    u32x4* dst = out + r * ROW_WORDS;
    if (MODE == 0) {
      const u32x4* nsrc = in + rn * ROW_WORDS;
      const bool more = rn < nrows;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        st(dst, t + k * THREADS, ROW_WORDS, buf[k] ^ u32x4{1u, 0u, 0u, 0u});
        if (more) buf[k] = ld(nsrc, t + k * THREADS, ROW_WORDS);
      }
      if (!more) break;
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) st(dst, t + k * THREADS, ROW_WORDS, buf[k] ^ u32x4{1u, 0u, 0u, 0u});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (rn >= nrows) break;
      if (MODE == 2 && (it + 1) % K == 0) grid_sync(ctr, (unsigned)G * ++epoch);
      const u32x4* nsrc = in + rn * ROW_WORDS;
#pragma unroll
      for (int k = 0; k < NV; ++k) buf[k] = ld(nsrc, t + k * THREADS, ROW_WORDS);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

int main(int argc, char** argv) {
  const int64_t nrows = argc > 1 ? atoll(argv[1]) : 65536;
  const int64_t words = nrows * ROW_WORDS;
  const size_t bytes = (size_t)words * 16;
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  void *in, *out;
  unsigned* ctr;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&ctr, sizeof(unsigned)));
  CK(hipMemset(in, 1, bytes));
  CK(hipMemset(out, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const u32x4* I = (const u32x4*)in;
  u32x4* O = (u32x4*)out;
  auto run = [&](const char* name, auto launch) {
    float best = 1e30f, sum = 0.f;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipMemset(ctr, 0, sizeof(unsigned)));
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0) {  // first launch: warm-up
        best = ms < best ? ms : best;
        sum += ms;
      }
    }
    printf("{\"variant\": \"%s\", \"rows\": %lld, \"bytes_each_way\": %zu, \"ms_best\": %.3f, \"ms_mean\": %.3f, "
           "\"GBps_best\": %.1f, \"cus\": %d}\n",
           name, (long long)nrows, bytes, best, sum / 5, 2.0 * bytes / best / 1e6, cus);
    fflush(stdout);
  };
  const int G = cus;
  run("overlap", [&] { rowcopy<0><<<G, THREADS>>>(I, O, nrows, ctr, 1); });
  run("phased", [&] { rowcopy<1><<<G, THREADS>>>(I, O, nrows, ctr, 1); });
  for (int K : {1, 4, 16}) {
    char nm[32];
    snprintf(nm, 32, "sync%d", K);
    run(nm, [&] { rowcopy<2><<<G, THREADS>>>(I, O, nrows, ctr, K); });
  }
  run("overlap", [&] { rowcopy<0><<<G, THREADS>>>(I, O, nrows, ctr, 1); });
  // in place (the row written back over the row read: the label-row lm_head's dlogits-over-logits)
  u32x4* IO = (u32x4*)in;
  run("phased_inplace", [&] { rowcopy<1><<<G, THREADS>>>(IO, IO, nrows, ctr, 1); });
  run("overlap_inplace", [&] { rowcopy<0><<<G, THREADS>>>(IO, IO, nrows, ctr, 1); });
  run("phased", [&] { rowcopy<1><<<G, THREADS>>>(I, O, nrows, ctr, 1); });
  run("phased_inplace", [&] { rowcopy<1><<<G, THREADS>>>(IO, IO, nrows, ctr, 1); });
  return 0;
}
