/* prl_gemm — C ABI for the trainer step's library GEMMs (hipBLASLt, bf16 in, fp32 accumulate).
 *
 * The model's linear layers (transformers Qwen2 q/k/v/o, gate/up/down, lm_head; run by
 * pipelinerl/finetune_loop.py:620-629 through the autograd engine) are plain GEMMs: this library
 * issues them through hipBLASLt with a per-problem solution choice (the library heuristic, or a
 * solution index found by prl_gemm_sweep on MI355X and shipped in-tree), instead of the single
 * heuristic pick the framework's matmul makes.  The weight gradient (dW = dY^T X, reduction over
 * the tokens) is where the heuristic pick is weakest.
 *
 * Column-major BLAS convention: D[m,n] = op(A)[m,k] * op(B)[k,n] (+ beta * D), op = N or T.
 * A, B are bf16; D is bf16 or fp32 (fp32 with beta = 1 accumulates a weight gradient over
 * chunks).  Every call is asynchronous on the caller's stream; buffers are caller-owned device
 * memory.  Returns 0 on success, PRL_GEMM_E_BASE + hipblasStatus_t for a hipBLASLt error,
 * PRL_GEMM_E_INVALID for bad arguments, PRL_GEMM_E_HIP + hipError_t for a runtime error.
 * Built as libprl_gemm.so.  hipBLASLt is the ROCm installation's, opened at first use with
 * dlopen(RTLD_LOCAL | RTLD_DEEPBIND) (env PRL_HIPBLASLT overrides the path) so it does not clash
 * with the copy torch bundles; it shares torch's HIP runtime.  PRL_GEMM_E_LOAD if it cannot be
 * opened (prl_gemm_error_string then names the reason).
 */
#ifndef PRL_GEMM_H
#define PRL_GEMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRL_GEMM_E_INVALID 4001
#define PRL_GEMM_E_LOAD 4002
#define PRL_GEMM_E_REFUSED 4003
#define PRL_GEMM_E_HIP 4100
#define PRL_GEMM_E_BASE 4400

enum PrlGemmOp { PRL_GEMM_N = 0, PRL_GEMM_T = 1 };
enum PrlGemmDtype { PRL_GEMM_F32 = 0, PRL_GEMM_BF16 = 1 };

int prl_gemm_abi_version(void);
const char* prl_gemm_error_string(int code);

/* D = op(A) op(B) (+ bias broadcast over D's columns) + beta * D.  `bias`: nullable, bf16, m
 * elements, bf16 D only (a linear layer's bias: m = output features).  `solution` >= 0 selects a
 * hipBLASLt solution index (falls back to the heuristic if it does not support the problem),
 * -1 = heuristic.  A solution index outside the set registered with prl_gemm_allow_solutions is
 * refused (PRL_GEMM_E_REFUSED) before any device work: hipBLASLt's catalog holds solutions that
 * fault the GPU on some shapes, and only the swept ones are trusted. */
int prl_gemm_bf16(int op_a, int op_b, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda,
                  const void* B, int64_t ldb, const void* bias, float beta, void* D, int64_t ldd, int d_dtype,
                  int solution, void* stream);

/* Solution index prl_gemm_bf16 would use for this problem with solution = -1 (-1 if none). */
int prl_gemm_heuristic_index(int op_a, int op_b, int64_t m, int64_t n, int64_t k, int64_t lda,
                             int64_t ldb, int64_t ldd, int d_dtype, float beta);

/* Replace the set of solution indices prl_gemm_bf16 may run (n = 0: none, heuristic only).
 * The binding registers the indices of its shipped solution table (gemm_solutions.json). */
int prl_gemm_allow_solutions(const int32_t* indices, int n);

/* Number of hipBLASLt handles created so far: one per (device, stream) that issued a GEMM (and
 * one per device for prl_gemm_heuristic_index / prl_gemm_library).  Launches on different streams
 * share no handle, workspace or plan. */
int prl_gemm_handle_count(void);

/* Path and version of the hipBLASLt in use, NUL-terminated into buf (the load error if it could
 * not be opened).  Returns 0 or the load error code. */
int prl_gemm_library(char* buf, int len);

#ifdef __cplusplus
}
#endif

#endif /* PRL_GEMM_H */
