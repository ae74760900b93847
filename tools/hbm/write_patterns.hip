// HBM write-pattern probe (measurement tool, not product): how fast can 20 GB be WRITTEN (and
// copied 50/50) with different store placements?  The loss head writes its dlogits row by row
// (one ~297 KB row per workgroup, 256 rows in flight); a grid-stride nontemporal store stream
// measured 4.3-5.3 TB/s, the copy 4.7-5.1 TB/s.  Variants:
//   gs_nt / gs_plain   grid-stride 16-B stores, nontemporal / default policy
//   chunk<C>           block b writes contiguous C-byte chunks b, b+G, b+2G, ... (row-per-block
//                      like the loss head at C = 297 KB)
//   rows2304           2,304-B rows in a pseudo-random order (the microarch guide's store probe)
// and the same placements for a 50/50 copy.  Prints one JSON line per variant.
//   hipcc -O3 --offload-arch=gfx950 tools/hbm/write_patterns.hip -o tools/hbm/write_patterns.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

template <bool NT, bool COPY>
__global__ __launch_bounds__(256) void gs(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const u32x4 z = {(uint32_t)threadIdx.x, 1u, 2u, 3u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    st<NT>(out + i, COPY ? __builtin_nontemporal_load(in + i) : z);
}

// contiguous chunks of `cw` 16-B words per block, unrolled by 4 per thread
template <bool NT, bool COPY>
__global__ __launch_bounds__(256) void chunk(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t n,
                                             int64_t cw) {
  const u32x4 z = {(uint32_t)threadIdx.x, 1u, 2u, 3u};
  const int64_t nchunks = (n + cw - 1) / cw;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t a = c * cw, b = a + cw < n ? a + cw : n;
    int64_t i = a + threadIdx.x;
    for (; i + 768 < b; i += 1024) {
      u32x4 v0 = COPY ? __builtin_nontemporal_load(in + i) : z;
      u32x4 v1 = COPY ? __builtin_nontemporal_load(in + i + 256) : z;
      u32x4 v2 = COPY ? __builtin_nontemporal_load(in + i + 512) : z;
      u32x4 v3 = COPY ? __builtin_nontemporal_load(in + i + 768) : z;
      st<NT>(out + i, v0);
      st<NT>(out + i + 256, v1);
      st<NT>(out + i + 512, v2);
      st<NT>(out + i + 768, v3);
    }
    for (; i < b; i += 256) st<NT>(out + i, COPY ? __builtin_nontemporal_load(in + i) : z);
  }
}

// 2,304-B rows (144 words) in a scrambled order: one wave per row, 8 waves per block
template <bool NT, bool COPY>
__global__ __launch_bounds__(512) void rows(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t nrows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const u32x4 z = {(uint32_t)lane, 1u, 2u, 3u};
  const int64_t nw = (int64_t)gridDim.x * 8;
  for (int64_t r = (int64_t)blockIdx.x * 8 + w; r < nrows; r += nw) {
    const int64_t rr = (r * 2654435761ll) % nrows;  // a permutation when gcd(2654435761, nrows) = 1
    u32x4* o = out + rr * 144;
    const u32x4* s = in + rr * 144;
    for (int j = lane; j < 144; j += 64) st<NT>(o + j, COPY ? __builtin_nontemporal_load(s + j) : z);
  }
}

int main(int argc, char** argv) {
  const int64_t bytes = (argc > 1 ? atoll(argv[1]) : 19914555392ll) / (144 * 16) * (144 * 16);
  const int64_t n = bytes / 16;
  void *in, *out;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMemset(in, 1, bytes));
  CK(hipMemset(out, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, bool copy, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 3;
    const double moved = copy ? 2.0 * bytes : (double)bytes;
    printf("{\"variant\": \"%s\", \"bytes\": %lld, \"ms\": %.3f, \"GBps\": %.1f}\n", name, (long long)bytes, ms,
           moved / ms / 1e6);
    fflush(stdout);
  };
  const u32x4* I = (const u32x4*)in;
  u32x4* O = (u32x4*)out;
  for (int copy = 0; copy < 2; ++copy) {
    const bool C = copy;
    char nm[64];
    for (int g : {1024, 2048, 8192}) {
      snprintf(nm, 64, "%s_gs_nt_g%d", C ? "copy" : "write", g);
      run(nm, C, [&] { if (C) gs<true, true><<<g, 256>>>(I, O, n); else gs<true, false><<<g, 256>>>(I, O, n); });
      snprintf(nm, 64, "%s_gs_plain_g%d", C ? "copy" : "write", g);
      run(nm, C, [&] { if (C) gs<false, true><<<g, 256>>>(I, O, n); else gs<false, false><<<g, 256>>>(I, O, n); });
    }
    for (int64_t cb : {65536ll, 303872ll, 2097152ll}) {
      for (int g : {256, 512, 1024}) {
        snprintf(nm, 64, "%s_chunk%lldB_nt_g%d", C ? "copy" : "write", (long long)cb, g);
        run(nm, C, [&] {
          if (C) chunk<true, true><<<g, 256>>>(I, O, n, cb / 16); else chunk<true, false><<<g, 256>>>(I, O, n, cb / 16);
        });
        snprintf(nm, 64, "%s_chunk%lldB_plain_g%d", C ? "copy" : "write", (long long)cb, g);
        run(nm, C, [&] {
          if (C) chunk<false, true><<<g, 256>>>(I, O, n, cb / 16); else chunk<false, false><<<g, 256>>>(I, O, n, cb / 16);
        });
      }
    }
    const int64_t nrows = n / 144;
    for (int g : {512, 2048}) {
      snprintf(nm, 64, "%s_rows2304_nt_g%d", C ? "copy" : "write", g);
      run(nm, C, [&] { if (C) rows<true, true><<<g, 512>>>(I, O, nrows); else rows<true, false><<<g, 512>>>(I, O, nrows); });
      snprintf(nm, 64, "%s_rows2304_plain_g%d", C ? "copy" : "write", g);
      run(nm, C, [&] { if (C) rows<false, true><<<g, 512>>>(I, O, nrows); else rows<false, false><<<g, 512>>>(I, O, nrows); });
    }
  }
  return 0;
}
