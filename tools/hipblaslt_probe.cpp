// Sweep every hipBLASLt solution for the trainer step's GEMM shapes (measurement tool).
//
// For each problem the heuristic's first choice and every supported solution are timed
// (hipEvents, 3 warm-up + 10 timed launches, rotating over 2 operand sets so no launch is served
// from a warm L2 / MALL); prints one JSON line per problem with the heuristic's time and the
// five fastest solutions (index and kernel name).
//
// Problems are given in torch's row-major terms: pass fwd  Y[T,N]  = X[T,K] W[N,K]^T
//                                               pass dgrad dX[T,K] = dY[T,N] W[N,K]
//                                               pass wgrad dW[N,K] = dY[T,N]^T X[T,K]
//   hipblaslt_probe [--heuristic-only | --top K] [--no-streamk] <pass> <T> <N> <K> [<pass> <T> <N> <K> ...]
// --no-streamk: time only candidates whose kernel is data-parallel (no "_SK<n>_" with n > 0 in
// its name: no cross-workgroup fix-up waits), and report the stream-K mode census of the
// candidates and of the heuristic's pick (stream-K beside RCCL).
// Build: hipcc -O2 --offload-arch=gfx950 tools/hipblaslt_probe.cpp -lhipblaslt -o tools/hipblaslt_probe.bin
//
// CAUTION: a full sweep runs every solution the library reports as supporting the problem, and
// one of them faulted the GPU (illegal address) at fwd T=16384 N=18944 K=3584 (7B gate/up) on
// MI355X / ROCm 7.2.  A faulting run counts against the GPU pool: sweep only shapes that have
// swept cleanly before, or use --heuristic-only.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    auto _e = (x);                                                                  \
    if ((int)_e != 0) {                                                             \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_e);         \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// deterministic pseudo-random bf16 in [-1, 1) (MFMA power and clocks depend on the data: a
// constant fill would flatter every solution)
__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    float f = (float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f;
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

struct Problem {
  // column-major hipBLASLt problem D[m,n] = op(A)[m,k] op(B)[k,n]
  hipblasOperation_t opA, opB;
  int64_t m, n, k, lda, ldb, ldc;
};

// row-major torch GEMMs -> column-major hipBLASLt (C^T = B^T A^T)
static Problem make(const char* pass, int64_t T, int64_t N, int64_t K) {
  Problem p{};
  if (!strcmp(pass, "fwd")) {  // Y^T[N,T] = W[N,K] (col-major KxN, op T) * X^T (col-major KxT, op N)
    p = {HIPBLAS_OP_T, HIPBLAS_OP_N, N, T, K, K, K, N};
  } else if (!strcmp(pass, "dgrad")) {  // dX^T[K,T] = W^T (col-major KxN, op N) * dY^T (col-major NxT, op N)
    p = {HIPBLAS_OP_N, HIPBLAS_OP_N, K, T, N, K, N, K};
  } else if (!strcmp(pass, "wgrad") || !strcmp(pass, "wgrad32") || !strcmp(pass, "wgradacc")) {  // dW^T[K,N] = X^T (col-major KxT, op N) * dY (col-major NxT, op T)
    p = {HIPBLAS_OP_N, HIPBLAS_OP_T, K, N, T, K, N, K};
  } else {
    fprintf(stderr, "unknown pass %s\n", pass);
    exit(2);
  }
  return p;
}

// stream-K mode from a Tensile kernel name ("..._SK3_..."): 0 = data-parallel
static int sk_mode(const std::string& name) {
  size_t p = name.find("_SK");
  while (p != std::string::npos) {
    if (p + 3 < name.size() && name[p + 3] >= '0' && name[p + 3] <= '9') return name[p + 3] - '0';
    p = name.find("_SK", p + 3);
  }
  return 0;
}

int main(int argc, char** argv) {
  bool heur_only = argc > 1 && !strcmp(argv[1], "--heuristic-only");  // skip the full sweep
  if (heur_only) {
    --argc;
    ++argv;
  }
  // --top K: time only the heuristic's K ranked candidates (the library's own picks for the
  // problem, not every solution of the catalog: the lower-risk sweep)
  int top = 0;
  bool no_sk = false;
  if (argc > 1 && !strcmp(argv[1], "--no-streamk")) {
    no_sk = true;
    --argc;
    ++argv;
  }
  if (argc > 2 && !strcmp(argv[1], "--top")) {
    top = atoi(argv[2]);
    argc -= 2;
    argv += 2;
  }
  // PRL_PROBE_SKIP=i,j,...: solution indices never launched (a blacklist of faulting solutions);
  // every index is logged to stderr (flushed) BEFORE its first launch, so a fault names it
  std::vector<int> skip;
  if (const char* env = getenv("PRL_PROBE_SKIP")) {
    for (const char* q = env; *q;) {
      skip.push_back(atoi(q));
      while (*q && *q != ',') ++q;
      if (*q == ',') ++q;
    }
  }
  if (argc < 5 || (argc - 1) % 4) {
    fprintf(stderr, "usage: %s <fwd|dgrad|wgrad> T N K [...]\n", argv[0]);
    return 2;
  }
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  const size_t ws_bytes = 256ull << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  for (int a = 1; a < argc; a += 4) {
    const char* pass = argv[a];
    int64_t T = atoll(argv[a + 1]), N = atoll(argv[a + 2]), K = atoll(argv[a + 3]);
    Problem p = make(pass, T, N, K);
    const bool f32 = !strcmp(pass, "wgrad32");  // fp32 dW accumulated over chunks (beta = 1)
    const bool acc = f32 || !strcmp(pass, "wgradacc");  // bf16 dW added into .grad (beta = 1)
    const hipDataType dt = f32 ? HIP_R_32F : HIP_R_16BF;
    int64_t a_rows = p.opA == HIPBLAS_OP_N ? p.m : p.k, a_cols = p.opA == HIPBLAS_OP_N ? p.k : p.m;
    int64_t b_rows = p.opB == HIPBLAS_OP_N ? p.k : p.n, b_cols = p.opB == HIPBLAS_OP_N ? p.n : p.k;
    size_t a_bytes = (size_t)p.lda * a_cols * 2, b_bytes = (size_t)p.ldb * b_cols * 2,
           c_bytes = (size_t)p.ldc * p.n * (f32 ? 4 : 2);
    void *A[2], *B[2], *C[2];
    for (int r = 0; r < 2; ++r) {
      CK(hipMalloc(&A[r], a_bytes));
      CK(hipMalloc(&B[r], b_bytes));
      CK(hipMalloc(&C[r], c_bytes));
      fill_bf16<<<2048, 256>>>((uint16_t*)A[r], a_bytes / 2, 17u + r);
      fill_bf16<<<2048, 256>>>((uint16_t*)B[r], b_bytes / 2, 91u + r);
    }
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &p.opA, sizeof(p.opA)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &p.opB, sizeof(p.opB)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, a_rows, a_cols, p.lda));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, b_rows, b_cols, p.ldb));
    CK(hipblasLtMatrixLayoutCreate(&lc, dt, p.m, p.n, p.ldc));
    float alpha = 1.f, beta = acc ? 1.f : 0.f;
    for (int r = 0; r < 2; ++r) CK(hipMemset(C[r], 0, c_bytes));

    // one timed probe launch first; only solutions within 1.3x of the best so far get the full
    // timing (3 warm-up + 10 timed launches) -- keeps a sweep over thousands of solutions short
    float best = 1e30f;
    auto launch = [&](hipblasLtMatmulAlgo_t* algo, int i) {
      return hipblasLtMatmul(h, desc, &alpha, A[i & 1], la, B[i & 1], lb, &beta, C[i & 1], lc, C[i & 1], lc, algo,
                             ws, ws_bytes, st);
    };
    auto time_algo = [&](hipblasLtMatmulAlgo_t* algo) -> float {
      if (launch(algo, 0) != HIPBLAS_STATUS_SUCCESS) return -1.f;
      float ms;
      CK(hipEventRecord(e0, st));
      launch(algo, 1);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms > 1.3f * best) return ms;
      for (int i = 0; i < 2; ++i) launch(algo, i);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < 10; ++i) launch(algo, i);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 10.f;
      best = std::min(best, ms);
      return ms;
    };

    // the heuristic's first choice (what an untuned caller gets)
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsb = ws_bytes;
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t heur[1];
    int nh = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 1, heur, &nh));
    float t_heur = nh ? time_algo(&heur[0].algo) : -1.f;
    int heur_idx = nh ? hipblaslt_ext::getIndexFromAlgo(heur[0].algo) : -1;

    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    if (top > 0) {
      all.resize(top);
      int nt = 0;
      CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, top, all.data(), &nt));
      all.resize(nt);
    } else if (!heur_only)
      CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, p.opA, p.opB, HIP_R_16BF, HIP_R_16BF,
                                  dt, dt, HIPBLAS_COMPUTE_32F, all));
    std::vector<std::pair<float, int>> res;
    int supported = 0;
    int sk_census[10] = {0};
    const int heur_sk = nh ? sk_mode(hipblaslt_ext::getKernelNameFromAlgo(h, heur[0].algo)) : -1;
    for (size_t i = 0; i < all.size(); ++i) {
      const int skm = sk_mode(hipblaslt_ext::getKernelNameFromAlgo(h, all[i].algo));
      sk_census[skm] += 1;
      if (no_sk && skm != 0) continue;
      size_t need = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(h, desc, &alpha, la, lb, &beta, lc, lc, all[i].algo, need) !=
              HIPBLAS_STATUS_SUCCESS ||
          need > ws_bytes)
        continue;
      const int idx = hipblaslt_ext::getIndexFromAlgo(all[i].algo);
      if (std::find(skip.begin(), skip.end(), idx) != skip.end()) continue;
      ++supported;
      fprintf(stderr, "launch %s %lld %lld %lld index %d (position %zu)\n", pass, (long long)T, (long long)N,
              (long long)K, idx, i);
      fflush(stderr);
      float t = time_algo(&all[i].algo);
      if (t > 0) res.emplace_back(t, (int)i);
      if (supported % 200 == 0) {
        fprintf(stderr, "%s %lld %lld %lld: %d supported of %zu tried, best %.4f ms\n", pass, (long long)T,
                (long long)N, (long long)K, supported, i + 1, best);
      }
    }
    std::sort(res.begin(), res.end());
    double flops = 2.0 * T * N * K;
    printf("{\"pass\": \"%s\", \"T\": %lld, \"N\": %lld, \"K\": %lld, \"solutions\": %zu, \"supported\": %d, "
           "\"heuristic_ms\": %.4f, \"heuristic_TFLOPs\": %.1f, \"heuristic_index\": %d, \"heuristic_sk\": %d, "
           "\"no_streamk\": %s, \"sk_census\": [%d, %d, %d, %d, %d], \"best\": [",
           pass, (long long)T, (long long)N, (long long)K, all.size(), supported, t_heur,
           t_heur > 0 ? flops / t_heur / 1e9 : 0.0, heur_idx, heur_sk, no_sk ? "true" : "false", sk_census[0],
           sk_census[1], sk_census[2], sk_census[3], sk_census[4]);
    for (size_t j = 0; j < std::min<size_t>(5, res.size()); ++j) {
      auto& alg = all[res[j].second].algo;
      const std::string kn = hipblaslt_ext::getKernelNameFromAlgo(h, alg);
      printf("%s{\"ms\": %.4f, \"TFLOPs\": %.1f, \"index\": %d, \"sk\": %d, \"kernel\": \"%s\"}", j ? ", " : "",
             res[j].first, flops / res[j].first / 1e9, hipblaslt_ext::getIndexFromAlgo(alg), sk_mode(kn),
             kn.substr(0, 120).c_str());
    }
    printf("]}\n");
    fflush(stdout);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(desc);
    for (int r = 0; r < 2; ++r) {
      hipFree(A[r]);
      hipFree(B[r]);
      hipFree(C[r]);
    }
  }
  return 0;
}
