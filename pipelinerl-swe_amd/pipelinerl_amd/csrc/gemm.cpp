// prl_gemm: the trainer step's library GEMMs through hipBLASLt with a per-problem solution
// choice (include/prl_gemm.h).  Host code only.
//
// The hipBLASLt used is the ROCm installation's (PRL_HIPBLASLT_PATH, baked in at build time;
// env PRL_HIPBLASLT overrides), opened with dlopen(RTLD_LOCAL | RTLD_DEEPBIND) and called through
// function pointers -- not torch's bundled copy: on MI355X the ROCm 7.2 library's solutions for
// the weight-gradient layout run 1.3-1.7x faster (tools/hipblaslt_probe.cpp, profiles/).  Loaded
// after torch, its libamdhip64.so.7 dependency resolves to the HIP runtime torch already loaded
// (same soname), so both libraries share one runtime, one device context and torch's streams.
//
// Per (op_a, op_b, m, n, k, lda, ldb, ldd, d_dtype, beta != 0) the matmul descriptor, the three
// matrix layouts and the chosen algorithm are built once and cached; a call is then one
// hipblasLtMatmul on the caller's stream.  Each (device, stream) pair gets its own hipBLASLt handle
// and its own workspace, so GEMMs issued on different streams share no library state: the gfx950
// solutions are stream-K kernels (Tensile "SK3": workgroups that finish a tile wait on flags other
// workgroups of the same launch set), and a stream-K launch must never see another launch's
// fix-up state ("stream-K beside RCCL").
#include "prl_gemm.h"

#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

namespace {

constexpr size_t kWorkspaceBytes = 128ull << 20;

#ifndef PRL_HIPBLASLT_PATH
#define PRL_HIPBLASLT_PATH "/opt/rocm/lib/libhipblaslt.so.1"
#endif

// hipBLASLt entry points, resolved at run time from the library opened below
struct Api {
  decltype(&::hipblasLtCreate) create = nullptr;
  decltype(&::hipblasLtGetVersion) version = nullptr;
  decltype(&::hipblasLtMatmulDescCreate) desc_create = nullptr;
  decltype(&::hipblasLtMatmulDescSetAttribute) desc_set = nullptr;
  decltype(&::hipblasLtMatmulDescDestroy) desc_destroy = nullptr;
  decltype(&::hipblasLtMatrixLayoutCreate) layout_create = nullptr;
  decltype(&::hipblasLtMatrixLayoutDestroy) layout_destroy = nullptr;
  decltype(&::hipblasLtMatmulPreferenceCreate) pref_create = nullptr;
  decltype(&::hipblasLtMatmulPreferenceSetAttribute) pref_set = nullptr;
  decltype(&::hipblasLtMatmulPreferenceDestroy) pref_destroy = nullptr;
  decltype(&::hipblasLtMatmulAlgoGetHeuristic) heuristic = nullptr;
  decltype(&::hipblasLtMatmul) matmul = nullptr;
  // C++ extension API (optional: solution indices)
  int (*index_from_algo)(hipblasLtMatmulAlgo_t&) = nullptr;
  hipblasStatus_t (*algos_from_index)(hipblasLtHandle_t, std::vector<int>&,
                                      std::vector<hipblasLtMatmulHeuristicResult_t>&) = nullptr;
  hipblasStatus_t (*is_supported)(hipblasLtHandle_t, hipblasLtMatmulDesc_t, const void*, hipblasLtMatrixLayout_t,
                                  hipblasLtMatrixLayout_t, const void*, hipblasLtMatrixLayout_t,
                                  hipblasLtMatrixLayout_t, hipblasLtMatmulAlgo_t&, size_t&) = nullptr;
  void* handle = nullptr;
  std::string path, error;
};

Api g_api;

struct Key {
  int op_a, op_b, d_dtype, accumulate, bias;
  int64_t m, n, k, lda, ldb, ldd;
  int solution;
  bool operator<(const Key& o) const {
    return std::tie(op_a, op_b, d_dtype, accumulate, bias, m, n, k, lda, ldb, ldd, solution) <
           std::tie(o.op_a, o.op_b, o.d_dtype, o.accumulate, o.bias, o.m, o.n, o.k, o.lda, o.ldb, o.ldd, o.solution);
  }
};

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  int index = -1;
};

std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, hipblasLtHandle_t> g_handles;
std::map<std::pair<int, hipStream_t>, void*> g_workspaces;
std::map<std::pair<hipblasLtHandle_t, Key>, Plan> g_plans;
// solution indices a caller may request (prl_gemm_allow_solutions): the set that ran clean in the
// MI355X sweeps shipped with the library; anything else is refused before it reaches the GPU
std::vector<int> g_allowed;
std::mutex g_allow_mu;

bool solution_allowed(int solution) {
  std::lock_guard<std::mutex> lock(g_allow_mu);
  return std::binary_search(g_allowed.begin(), g_allowed.end(), solution);
}

template <class F>
bool sym(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  return *out != nullptr;
}

int load_api() {
  if (g_api.matmul) return 0;
  if (!g_api.error.empty()) return PRL_GEMM_E_LOAD;
  const char* env = getenv("PRL_HIPBLASLT");
  g_api.path = env && *env ? env : PRL_HIPBLASLT_PATH;
  void* h = dlopen(g_api.path.c_str(), RTLD_LAZY | RTLD_LOCAL | RTLD_DEEPBIND);
  if (!h) {
    const char* e = dlerror();
    g_api.error = std::string("dlopen ") + g_api.path + ": " + (e ? e : "?");
    return PRL_GEMM_E_LOAD;
  }
  Api a;
  bool ok = sym(h, "hipblasLtCreate", &a.create) && sym(h, "hipblasLtGetVersion", &a.version) &&
            sym(h, "hipblasLtMatmulDescCreate", &a.desc_create) &&
            sym(h, "hipblasLtMatmulDescSetAttribute", &a.desc_set) &&
            sym(h, "hipblasLtMatmulDescDestroy", &a.desc_destroy) &&
            sym(h, "hipblasLtMatrixLayoutCreate", &a.layout_create) &&
            sym(h, "hipblasLtMatrixLayoutDestroy", &a.layout_destroy) &&
            sym(h, "hipblasLtMatmulPreferenceCreate", &a.pref_create) &&
            sym(h, "hipblasLtMatmulPreferenceSetAttribute", &a.pref_set) &&
            sym(h, "hipblasLtMatmulPreferenceDestroy", &a.pref_destroy) &&
            sym(h, "hipblasLtMatmulAlgoGetHeuristic", &a.heuristic) && sym(h, "hipblasLtMatmul", &a.matmul);
  if (!ok) {
    g_api.error = "missing hipBLASLt symbol in " + g_api.path;
    dlclose(h);
    return PRL_GEMM_E_LOAD;
  }
  sym(h, "_ZN13hipblaslt_ext16getIndexFromAlgoER22_hipblasLtMatmulAlgo_t", &a.index_from_algo);
  sym(h, "_ZN13hipblaslt_ext17getAlgosFromIndexEPvRSt6vectorIiSaIiEERS1_I33_hipblasLtMatmulHeuristicResult_tSaIS5_EE",
      &a.algos_from_index);
  sym(h,
      "_ZN13hipblaslt_ext21matmulIsAlgoSupportedEPvP27hipblasLtMatmulDescOpaque_tPKvP29hipblasLtMatrixLayoutOpaque_"
      "tS6_S4_S6_S6_R22_hipblasLtMatmulAlgo_tRm",
      &a.is_supported);
  a.handle = h;
  a.path = g_api.path;
  g_api = a;
  return 0;
}

inline int hb(hipblasStatus_t s) { return s == HIPBLAS_STATUS_SUCCESS ? 0 : PRL_GEMM_E_BASE + (int)s; }
inline int hp(hipError_t e) { return e == hipSuccess ? 0 : PRL_GEMM_E_HIP + (int)e; }

#define RET(x)               \
  do {                       \
    int _rc = (x);           \
    if (_rc) return _rc;     \
  } while (0)

hipblasOperation_t op(int o) { return o == PRL_GEMM_T ? HIPBLAS_OP_T : HIPBLAS_OP_N; }
hipDataType dtype(int d) { return d == PRL_GEMM_F32 ? HIP_R_32F : HIP_R_16BF; }

bool valid(int op_a, int op_b, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldd,
           int d_dtype) {
  if ((op_a != PRL_GEMM_N && op_a != PRL_GEMM_T) || (op_b != PRL_GEMM_N && op_b != PRL_GEMM_T)) return false;
  if (d_dtype != PRL_GEMM_F32 && d_dtype != PRL_GEMM_BF16) return false;
  if (m <= 0 || n <= 0 || k <= 0) return false;
  if (lda < (op_a == PRL_GEMM_N ? m : k) || ldb < (op_b == PRL_GEMM_N ? k : n) || ldd < m) return false;
  return true;
}

int handle_for(int dev, hipStream_t st, hipblasLtHandle_t* h) {
  auto key = std::make_pair(dev, st);
  auto it = g_handles.find(key);
  if (it != g_handles.end()) {
    *h = it->second;
    return 0;
  }
  RET(hb(g_api.create(h)));
  g_handles[key] = *h;
  return 0;
}

int workspace_for(int dev, hipStream_t st, void** ws) {
  auto key = std::make_pair(dev, st);
  auto it = g_workspaces.find(key);
  if (it != g_workspaces.end()) {
    *ws = it->second;
    return 0;
  }
  RET(hp(hipMalloc(ws, kWorkspaceBytes)));
  g_workspaces[key] = *ws;
  return 0;
}

int make_layouts(const Key& k, Plan* p) {
  RET(hb(g_api.desc_create(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F)));
  hipblasOperation_t oa = op(k.op_a), ob = op(k.op_b);
  RET(hb(g_api.desc_set(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa))));
  RET(hb(g_api.desc_set(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob))));
  if (k.bias) {  // bf16 bias along D's rows (the output features), added before rounding
    hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
    int32_t bt = HIP_R_16BF;
    RET(hb(g_api.desc_set(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi))));
    RET(hb(g_api.desc_set(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt))));
  }
  int64_t ar = k.op_a == PRL_GEMM_N ? k.m : k.k, ac = k.op_a == PRL_GEMM_N ? k.k : k.m;
  int64_t br = k.op_b == PRL_GEMM_N ? k.k : k.n, bc = k.op_b == PRL_GEMM_N ? k.n : k.k;
  RET(hb(g_api.layout_create(&p->la, HIP_R_16BF, ar, ac, k.lda)));
  RET(hb(g_api.layout_create(&p->lb, HIP_R_16BF, br, bc, k.ldb)));
  RET(hb(g_api.layout_create(&p->ld, dtype(k.d_dtype), k.m, k.n, k.ldd)));
  return 0;
}

int heuristic(hipblasLtHandle_t h, Plan* p) {
  hipblasLtMatmulPreference_t pref;
  RET(hb(g_api.pref_create(&pref)));
  uint64_t ws = kWorkspaceBytes;
  int rc = hb(g_api.pref_set(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t r[1];
  int got = 0;
  if (!rc) rc = hb(g_api.heuristic(h, p->desc, p->la, p->lb, p->ld, p->ld, pref, 1, r, &got));
  g_api.pref_destroy(pref);
  if (rc) return rc;
  if (got < 1) return PRL_GEMM_E_BASE + (int)HIPBLAS_STATUS_NOT_SUPPORTED;
  p->algo = r[0].algo;
  p->index = g_api.index_from_algo ? g_api.index_from_algo(p->algo) : -1;
  return 0;
}

// solution index -> algorithm, if that solution supports the problem within the workspace
bool from_index(hipblasLtHandle_t h, const Key& k, Plan* p) {
  if (!g_api.algos_from_index || !g_api.is_supported) return false;
  std::vector<int> idx{k.solution};
  std::vector<hipblasLtMatmulHeuristicResult_t> res;
  if (g_api.algos_from_index(h, idx, res) != HIPBLAS_STATUS_SUCCESS || res.empty()) return false;
  float alpha = 1.f, beta = k.accumulate ? 1.f : 0.f;
  size_t need = 0;
  if (g_api.is_supported(h, p->desc, &alpha, p->la, p->lb, &beta, p->ld, p->ld, res[0].algo,
                                           need) != HIPBLAS_STATUS_SUCCESS ||
      need > kWorkspaceBytes)
    return false;
  p->algo = res[0].algo;
  p->index = k.solution;
  return true;
}

void destroy(Plan& p) {
  if (p.desc) g_api.desc_destroy(p.desc);
  if (p.la) g_api.layout_destroy(p.la);
  if (p.lb) g_api.layout_destroy(p.lb);
  if (p.ld) g_api.layout_destroy(p.ld);
}

// Packed micro-batches have a different token count almost every time, so the cache is bounded:
// past kMaxPlans entries it is emptied (a plan costs one heuristic query, ~0.1 ms of host time).
constexpr size_t kMaxPlans = 4096;

int plan_for(hipblasLtHandle_t h, const Key& k, Plan** out) {
  auto key = std::make_pair(h, k);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) {
    *out = &it->second;
    return 0;
  }
  if (g_plans.size() >= kMaxPlans) {  // callers hold no Plan pointer across calls (one lock scope)
    for (auto& kv : g_plans) destroy(kv.second);
    g_plans.clear();
  }
  Plan p;
  int rc = make_layouts(k, &p);
  if (!rc && !(k.solution >= 0 && from_index(h, k, &p))) rc = heuristic(h, &p);
  if (rc) {
    destroy(p);
    return rc;
  }
  *out = &(g_plans[key] = p);
  return 0;
}

Key make_key(int op_a, int op_b, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldd,
             int d_dtype, float beta, int solution, bool bias = false) {
  return Key{op_a, op_b, d_dtype, beta != 0.f ? 1 : 0, bias ? 1 : 0, m, n, k, lda, ldb, ldd,
             solution < 0 ? -1 : solution};
}

}  // namespace

extern "C" {

int prl_gemm_abi_version(void) { return 4; }

const char* prl_gemm_error_string(int code) {
  if (code == 0) return "ok";
  if (code == PRL_GEMM_E_INVALID) return "invalid argument";
  if (code == PRL_GEMM_E_REFUSED) return "solution index not in the allowed (swept) set";
  if (code == PRL_GEMM_E_LOAD) return g_api.error.empty() ? "hipBLASLt not loaded" : g_api.error.c_str();
  if (code >= PRL_GEMM_E_BASE) {
    switch (code - PRL_GEMM_E_BASE) {
      case HIPBLAS_STATUS_NOT_INITIALIZED: return "hipBLASLt: not initialized";
      case HIPBLAS_STATUS_ALLOC_FAILED: return "hipBLASLt: allocation failed";
      case HIPBLAS_STATUS_INVALID_VALUE: return "hipBLASLt: invalid value";
      case HIPBLAS_STATUS_EXECUTION_FAILED: return "hipBLASLt: execution failed";
      case HIPBLAS_STATUS_NOT_SUPPORTED: return "hipBLASLt: no solution supports the problem";
      default: return "hipBLASLt error";
    }
  }
  if (code >= PRL_GEMM_E_HIP) return hipGetErrorString((hipError_t)(code - PRL_GEMM_E_HIP));
  return "unknown error";
}

int prl_gemm_bf16(int op_a, int op_b, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda,
                  const void* B, int64_t ldb, const void* bias, float beta, void* D, int64_t ldd, int d_dtype,
                  int solution, void* stream) {
  if (!valid(op_a, op_b, m, n, k, lda, ldb, ldd, d_dtype) || !A || !B || !D) return PRL_GEMM_E_INVALID;
  if (beta != 0.f && beta != 1.f) return PRL_GEMM_E_INVALID;
  if (bias && d_dtype != PRL_GEMM_BF16) return PRL_GEMM_E_INVALID;
  if (solution >= 0 && !solution_allowed(solution)) return PRL_GEMM_E_REFUSED;
  int dev;
  RET(hp(hipGetDevice(&dev)));
  hipStream_t st = (hipStream_t)stream;
  std::lock_guard<std::mutex> lock(g_mu);
  RET(load_api());
  hipblasLtHandle_t h;
  RET(handle_for(dev, st, &h));
  void* ws;
  RET(workspace_for(dev, st, &ws));
  Plan* p;
  RET(plan_for(h, make_key(op_a, op_b, m, n, k, lda, ldb, ldd, d_dtype, beta, solution, bias != nullptr), &p));
  if (bias) RET(hb(g_api.desc_set(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias))));
  float alpha = 1.f;
  return hb(g_api.matmul(h, p->desc, &alpha, A, p->la, B, p->lb, &beta, D, p->ld, D, p->ld, &p->algo, ws,
                            kWorkspaceBytes, st));
}

int prl_gemm_heuristic_index(int op_a, int op_b, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                             int64_t ldd, int d_dtype, float beta) {
  if (!valid(op_a, op_b, m, n, k, lda, ldb, ldd, d_dtype)) return -1;
  int dev;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  std::lock_guard<std::mutex> lock(g_mu);
  hipblasLtHandle_t h;
  Plan* p;
  if (load_api() || handle_for(dev, nullptr, &h) ||
      plan_for(h, make_key(op_a, op_b, m, n, k, lda, ldb, ldd, d_dtype, beta, -1), &p))
    return -1;
  return p->index;
}

int prl_gemm_handle_count(void) {
  std::lock_guard<std::mutex> lock(g_mu);
  return (int)g_handles.size();
}

int prl_gemm_allow_solutions(const int32_t* indices, int n) {
  if (n < 0 || (n > 0 && !indices)) return PRL_GEMM_E_INVALID;
  std::vector<int> v(indices, indices + n);
  for (int i : v)
    if (i < 0) return PRL_GEMM_E_INVALID;
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  std::lock_guard<std::mutex> lock(g_allow_mu);
  g_allowed.swap(v);
  return 0;
}

int prl_gemm_library(char* buf, int len) {
  if (!buf || len <= 0) return PRL_GEMM_E_INVALID;
  int rc;
  int ver = 0;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    rc = load_api();
    if (!rc) {
      int dev;
      hipblasLtHandle_t h;
      rc = hp(hipGetDevice(&dev));
      if (!rc) rc = handle_for(dev, nullptr, &h);
      if (!rc) rc = hb(g_api.version(h, &ver));
    }
  }
  std::string s = rc == PRL_GEMM_E_LOAD ? g_api.error : g_api.path + " version " + std::to_string(ver);
  strncpy(buf, s.c_str(), (size_t)len - 1);
  buf[len - 1] = 0;
  return rc;
}

}  // extern "C"
