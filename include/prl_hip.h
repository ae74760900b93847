/* prl_hip.h — C ABI of the MI355X GRPO trainer-step library (libprl_hip.so).
 *
 * Plain C: device pointers, sizes and a hipStream_t (passed as void*).  No torch types.
 * Every entry point returns 0 on success or a PRL_E* / hipError_t-derived code; nothing
 * throws across the ABI.  All buffers are caller-owned device memory, scratch included (the
 * workspaces and counters below); nothing is allocated on a launch path.  The library keeps no
 * global state besides a per-device property cache.  A workspace or counter serves one stream at
 * a time (launches on two streams in flight at once need two).
 *
 * ABI history: 2 -> 3 (round 6): prl_grpo_forward_rows takes the loss-head workspace;
 * prl_grpo_pair_fallbacks reads the workspace's counter (not a per-stream library buffer);
 * PrlGrpoParams gains pair_spin_ticks and f32_rows (replacing the PRL_PAIR_SPIN_TICKS /
 * PRL_F32_PAIR environment reads); the phased SwiGLU entry points take their chunk counter;
 * prl_grad_sqnorm requires its workspace (since round 5; PRL_E_WORKSPACE without one).
 *
 * Reference interfaces replaced (paths under the reference repo, ServiceNow/PipelineRL-SWE):
 *   prl_grpo_forward   <- rl_step loss head + stats + autograd backward
 *                         pipelinerl/finetune/rl/__init__.py:130-377 (ATen ops :200-366)
 *                         and pipelinerl/finetune/rl/utils.py:25-30,66-87 (masked sums)
 *   prl_grpo_backward  <- the autograd backward of the same graph (loss.backward() at
 *                         pipelinerl/finetune_loop.py:620-629) when the upstream gradient
 *                         differs from the one assumed by the fused forward
 *   prl_flatten_bf16 / prl_unflatten_bf16
 *                      <- per-parameter `parameter.data.bfloat16()` + dist.broadcast loop
 *                         of WeightUpdateManager.send_weight_update
 *                         (pipelinerl/finetune_loop.py:202-205, :246-247) and the actor's
 *                         per-tensor receive buffers (pipelinerl/vllm1.py:84-93)
 *   prl_grad_sqnorm    <- clip_grad_norm_'s global norm (finetune_loop.py:642-643)
 */
#ifndef PRL_HIP_H
#define PRL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRL_ABI_VERSION 3

/* error codes (besides hipError_t values, which are < 1000) */
#define PRL_OK 0
#define PRL_E_INVALID 1001      /* bad argument: shape, null pointer, alignment */
#define PRL_E_UNSUPPORTED 1002  /* dtype / layout not supported */
#define PRL_E_WORKSPACE 1003    /* workspace too small */

/* dtypes */
#define PRL_F32 0
#define PRL_BF16 1

/* policy losses (rl/__init__.py:269-283) */
#define PRL_PPO 0
#define PRL_REINFORCE 1

/* statistics written by prl_grpo_forward into stats[PRL_NSTAT] (double) */
enum PrlStat {
  PRL_S_LOSS_SUM = 0,      /* sum nz(token_loss * mask)   -> policy_loss_total = -this */
  PRL_S_VALUE_LOSS,        /* sum nz(0.5 (v-r)^2 w mask) */
  PRL_S_REWARD,            /* sum nz(r / nl * mask) ... per-label-normalised sums */
  PRL_S_ENTROPY,
  PRL_S_OLD_LP,
  PRL_S_NEW_LP,
  PRL_S_REF_LP,
  PRL_S_ADVANTAGE,
  PRL_S_KL,
  PRL_S_POLICY_LOSS,
  PRL_S_SURR1,
  PRL_S_SURR2,
  PRL_S_RATIO,             /* sum nz(ratio/nl) */
  PRL_S_RATIO_SUM,         /* sum nz(ratio) */
  PRL_S_RATIO_SQ_SUM,      /* sum nz(ratio^2) */
  PRL_S_RATIO_REF_NEW,
  PRL_S_RATIO_REF_OLD,
  PRL_S_CLAMP_REF_NEW,
  PRL_S_CLAMP_NEW_OLD,
  PRL_S_TOKEN_WEIGHT,
  PRL_S_VALUE_MEAN,
  PRL_S_VALUE_MSE,
  PRL_S_NUM_NANS,          /* count isnan(token_loss), all positions */
  PRL_S_NUM_OUT,           /* count mask */
  PRL_S_BAD_LP,            /* count non-finite new log-probs, all positions  (assert :209) */
  PRL_S_BAD_LRRN,          /* count non-finite ref-new log ratio             (assert :237) */
  PRL_S_BAD_KL,            /* count non-finite approx KL                     (assert :264) */
  PRL_S_BAD_GT,            /* count group_tokens <= 0 when group-normalising (assert :222) */
  PRL_S_BAD_ID,            /* count target ids outside [0, V)   (torch.gather IndexError :208) */
  PRL_S_MAX_REWARD,        /* masked max/min (NaN-propagating, like torch.max) */
  PRL_S_MIN_REWARD,
  PRL_S_MAX_ADV,
  PRL_S_MIN_ADV,
  PRL_S_MAX_KL,
  PRL_S_MIN_KL,
  PRL_S_MAX_W,
  PRL_S_MIN_W,
  PRL_S_MAX_VALUE,
  PRL_S_MIN_VALUE,
  PRL_NSTAT
};

/* Inputs: a [B, L] batch of packed (B = 1) or padded (B >= 1) rollouts and its logits
 * [B, L, V] (row stride ld elements, batch stride L*ld).  Row t of sequence b is scored
 * against input_ids[b, t+1]; rows t = L-1 carry no loss.  Token fields are the
 * PipelineBatchEncoding tensors (pipelinerl/finetune/types.py:48-75), float32 [B, L]. */
typedef struct PrlGrpoBatch {
  const void* logits;          /* [B, L, V] bf16 or f32 */
  int32_t logits_dtype;        /* PRL_BF16 | PRL_F32 */
  int32_t _pad0;
  int64_t B, L, V, ld;         /* ld = row stride in elements (>= V) */
  const int64_t* input_ids;    /* [B, L] */
  const int64_t* labels;       /* [B, L], -100 = masked */
  const float* rewards;
  const float* advantages;
  const float* ref_logprobs;
  const float* old_logprobs;
  const float* group_tokens;
  const float* num_labels;
  const float* overflow;
  const float* values;         /* [B, L] value-head output or NULL */
} PrlGrpoBatch;

typedef struct PrlGrpoParams {
  int32_t policy_loss;         /* PRL_PPO | PRL_REINFORCE */
  int32_t use_advantages;
  int32_t relu_log_p_weights;
  int32_t group_normalization;
  int32_t overlong_filtering;
  int32_t write_grad;          /* 1: prl_grpo_forward also writes dlogits */
  float epsilon;
  float kl_coef;               /* already linearly decayed (rl/__init__.py:265-266) */
  float entropy_coef;          /* already linearly decayed */
  float clamp_log_ratio;       /* clamp_log_ratio_ref_new_value */
  float temperature;
  float batch_size;            /* token weight = 1 / batch_size unless group-normalised */
  float value_loss_coef;
  float grad_scale;            /* upstream d(final_loss) assumed for dlogits / dvalues (> 0, finite) */
  int32_t pair_spin_ticks;     /* fp32 pair kernel: realtime ticks (100 MHz) a row half waits for its
                                  partner's partial (or the leader's row claim) before going SOLO for
                                  the rest of the launch: its own rows claimed, the other half's
                                  partial and gradient from HBM (the same bits);
                                  0 = the default (20000, 200 us), < 0 = never waits */
  int32_t f32_rows;            /* fp32 logits: 0 = the pair kernel where the row fits two CUs (default),
                                  1 = the part-resident kernel */
} PrlGrpoParams;

/* Outputs.  Per-token arrays have B*(L-1) entries (row q = b*(L-1) + t). */
typedef struct PrlGrpoOutputs {
  float* new_logprobs;
  float* entropy;
  float* lse;                  /* log-sum-exp of logits/temperature (natural log) */
  float* token_loss;           /* (pol - kl_c kl + ent_c H) * w  (unmasked) */
  float* g_lp;                 /* d final / d new_lp  at grad_scale */
  float* g_h;                  /* d final / d entropy at grad_scale */
  float* row_max;              /* reference max m of the row (raw logit units) */
  float* row_log2sum;          /* log2 sum_j 2^((x_j - m) log2(e) / temperature) */
  float* dvalues;              /* [B, L] or NULL (required when values != NULL) */
  void* dlogits;               /* [B, L, V], same dtype/ld as logits, or NULL */
  double* stats;               /* [PRL_NSTAT] */
} PrlGrpoOutputs;

int prl_abi_version(void);
const char* prl_error_string(int code);

/* Bytes of the loss head's device workspace on `device`: the statistics' per-block partial sums
 * and the row kernels' scratch (row counter, fp32 pair hand-off slots, pair fallback counter).
 * Zero-fill it once when allocated (the fallback counter accumulates across launches). */
int prl_grpo_workspace_bytes(int device, size_t* bytes);

/* Fused loss head: log-softmax + gather + entropy over V, importance ratio x advantage
 * policy loss (PPO / REINFORCE), KL-to-reference (Schulman k3), token weights, masked
 * statistics, and (write_grad) dlogits for upstream gradient grad_scale.
 * One read of the logits and (write_grad) one write of dlogits. */
int prl_grpo_forward(const PrlGrpoBatch* batch, const PrlGrpoParams* params,
                     const PrlGrpoOutputs* out, void* workspace, size_t workspace_bytes,
                     void* stream);

/* Row-selected vocab pass (label rows only; chunked lm_head + loss).
 * batch->logits holds n rows [n, ld]; logits row i scores batch row row_ids[i] (device
 * int64, q = b*(L-1) + t, each < B*(L-1)); B and L describe the whole batch, whose token
 * fields are read at those rows.  Per-row outputs land at index row_ids[i] of the
 * B*(L-1)-entry arrays; dlogits (write_grad) is [n, ld] and may alias batch->logits
 * (every row is read before its gradient is stored).  No statistics (out->stats unused).
 * A value head's batch->values (every row) enter only through the advantage, reward - value
 * (rl/__init__.py:239-248); out->dvalues must be given, as for prl_grpo_forward, but the value
 * loss, its statistics and dvalues are written by prl_grpo_stats.  Replaces the [T, V] slice of
 * the ATen chain rl/__init__.py:199-208 for the rows its mask (:152-153) keeps. */
int prl_grpo_forward_rows(const PrlGrpoBatch* batch, const PrlGrpoParams* params,
                          const int64_t* row_ids, int64_t n, const PrlGrpoOutputs* out,
                          void* workspace, size_t workspace_bytes, void* stream);

/* Statistics (rl/__init__.py:315-375) and dvalues from the per-row new_logprobs / entropy
 * arrays over all B*(L-1) rows (batch->logits may be NULL).  Rows never scored must hold
 * finite values (e.g. 0): masked rows only enter num_nans and the finiteness counters. */
int prl_grpo_stats(const PrlGrpoBatch* batch, const PrlGrpoParams* params,
                   const PrlGrpoOutputs* out, void* workspace, size_t workspace_bytes,
                   void* stream);

/* Gradient pass from the per-row max / log2sum / entropy / g_lp / g_h saved by prl_grpo_forward (at
 * params->grad_scale), for an upstream gradient read ON DEVICE from *upstream (NULL = 1.0):
 *   dlogits = (*upstream) * d final / d logits.
 * If params->write_grad is set, dlogits already holds the gradient for upstream ==
 * params->grad_scale (the caller's loss scale, e.g. DeepSpeed's 1/GAS) and the kernel returns
 * without touching memory when *upstream equals it (no host sync needed to decide).  Rows with
 * zero coefficients are written as zeros without reading the logits. */
int prl_grpo_backward(const PrlGrpoBatch* batch, const PrlGrpoParams* params,
                      const float* row_max, const float* row_log2sum, const float* entropy,
                      const float* g_lp, const float* g_h, const float* upstream, void* dlogits,
                      void* stream);

/* Number of statistics (PRL_NSTAT) compiled into the library: bindings check it. */
int prl_grpo_nstat(void);

/* Observability of the pair kernels (fp32 rows, each split over two workgroups): how many rows of
 * launches with this workspace a SOLO half finished alone (its partner's partial or claim had not
 * arrived within PrlGrpoParams.pair_spin_ticks) since the last call; reads and resets the
 * workspace's counter, synchronising the stream. */
int prl_grpo_pair_fallbacks(void* workspace, size_t workspace_bytes, void* stream, uint64_t* count);

/* Weight broadcast staging: copy n tensors (f32 or bf16, contiguous) into one bf16 buffer
 * at the given element offsets (dst_offsets[i], bf16 elements; 8-element aligned for the
 * vector path), converting with round-to-nearest-even; and the inverse into bf16 or f32
 * destinations.  srcs/dsts/dtypes/numels/offsets are HOST arrays of length n. */
int prl_flatten_bf16(const void* const* srcs, const int32_t* dtypes, const int64_t* numels,
                     const int64_t* dst_offsets, int32_t n, void* dst, void* stream);
int prl_unflatten_bf16(const void* src, void* const* dsts, const int32_t* dtypes,
                       const int64_t* numels, const int64_t* src_offsets, int32_t n,
                       void* stream);

/* Weight-gradient scale / accumulate (bf16 destination), the upstream scale read on the device:
 *   t = bf16(float(src[i]) * (*scale));  dst[i] = accumulate ? bf16(float(dst[i]) + float(t)) : t
 * src f32 or bf16, n elements, src / dst 16-B aligned.  In place (dst == src, bf16, accumulate 0)
 * nothing is written when *scale == 1.  Replaces the ATen chain `(dw.float() * g).to(bf16)` +
 * AccumulateGrad's `grad += dw` behind the reference's lm_head weight gradient
 * (pipelinerl/finetune_loop.py:620-629, loss.backward over the lm_head of rl/__init__.py:197). */
int prl_grad_scale_bf16(const void* src, int32_t src_dtype, const float* scale, void* dst, int64_t n,
                        int32_t accumulate, void* stream);

/* Measurement helper, not a product path (bench.py snapshot_overlap): emulates the reads an RCCL
 * broadcast root makes of the buffer it sends (finetune_loop.py:202-205 broadcasts the parameters)
 * when no receiver exists: `blocks` 256-thread workgroups (the communicator's channels) stream
 * `bytes` of `src` (16-B aligned; the tail below 16 B is not read) with nontemporal loads, paced to
 * `gbps` in total against the realtime clock; sink (device, >= blocks words) receives a folded
 * word of workgroup i only when it matches an internal key (keeps the loads; contents unspecified). */
int prl_paced_read(const void* src, int64_t bytes, double gbps, int32_t blocks, uint32_t* sink, void* stream);

/* AdamW step over n tensors (csrc/adamw.hip): params / grads / exp_avgs / exp_avg_sqs are device
 * pointers of `dtype` (PRL_BF16 or PRL_F32, all four alike), steps[i] the device float step count
 * of tensor i (already incremented for this step, as torch's fused AdamW expects it), numels[i] its
 * element count; the pointer arrays themselves are host memory.  grad_scale: NULL, or a device
 * scalar of `dtype` every gradient is multiplied by first (the gradient-clipping coefficient,
 * stored-and-reloaded rounding as torch._foreach_mul_ would leave it; the gradients themselves are
 * not written).  Bit-identical to torch.optim.AdamW(fused=True) after clip_grad_norm_ (ADAMW mode,
 * no amsgrad / maximize).  Every entry is validated before the first launch.  Replaces
 * clip_grad_norm_'s multiply + optimizer.step() at pipelinerl/finetune_loop.py:700-719. */
int prl_adamw_step(int32_t n, void* const* params, const void* const* grads, void* const* exp_avgs,
                   void* const* exp_avg_sqs, const float* const* steps, const int64_t* numels, int32_t dtype,
                   double lr, double beta1, double beta2, double weight_decay, double eps, const void* grad_scale,
                   void* stream);

/* AdamW with fp32 master weights (csrc/adamw.hip): the optimizer state of the reference's default
 * backend, DeepSpeed's bf16 ZeRO optimizer (conf/deepspeed/deepspeed_stage3_bf16.json: fp32 master
 * partitions, fp32 Adam states) and of its FSDP mixed precision (accelerate upcasts the parameters
 * to fp32 in prepare, pipelinerl/finetune_loop.py:355-396).  Per tensor i: grads[i] (grad_dtype,
 * PRL_BF16 or PRL_F32) is read, multiplied in fp32 by *grad_scale (device float; NULL = none: the
 * clip coefficient, as clip_grad_norm_'s foreach_mul_ on fp32 gradients), and the fp32 masters[i],
 * exp_avgs[i], exp_avg_sqs[i] take torch's fused-AdamW fp32 update (ADAMW mode, steps[i] already
 * incremented); params[i] (bf16) receives the round-to-nearest-even of the new master.  One pass:
 * 14 B read + 14 B written per parameter with bf16 gradients.  Host arrays of length n; every
 * entry is validated before the first launch.  Replaces clip_grad_norm_'s multiply +
 * optimizer.step() + the bf16 copy-back at pipelinerl/finetune_loop.py:700-719. */
int prl_adamw_master_step(int32_t n, void* const* params, const void* const* grads, float* const* masters,
                          float* const* exp_avgs, float* const* exp_avg_sqs, const float* const* steps,
                          const int64_t* numels, int32_t grad_dtype, double lr, double beta1, double beta2,
                          double weight_decay, double eps, const float* grad_scale, void* stream);

/* Sum of squares of n device tensors (f32 or bf16) into *out (device f64; overwritten).
 * Deterministic: a fixed 256 partials per tensor (fp64 accumulation) in `workspace`, then one
 * fixed-order fold — no atomics.  workspace: device memory of at least n * 256 * 8 bytes
 * (PRL_E_WORKSPACE otherwise). */
int prl_grad_sqnorm(const void* const* srcs, const int32_t* dtypes, const int64_t* numels,
                    int32_t n, double* out, void* workspace, size_t workspace_bytes,
                    void* stream);

/* ---- Trainer-step model ops (bf16; csrc/model_ops.hip).  One HBM pass each; the forward
 * reproduces the eager HF chains' bf16 roundings (transformers Qwen2RMSNorm.forward,
 * Qwen2MLP.forward act_fn(gate) * up with SiLU, apply_rotary_pos_emb).  Row-major contiguous
 * tensors, 16-B aligned (8-B for RoPE), H and D multiples of 8; PRL_E_UNSUPPORTED otherwise. */

/* y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps))) per row of H; rstd[rows] saved (fp32). */
int prl_rmsnorm_forward(const void* x, const void* w, void* y, float* rstd, int64_t rows, int64_t H,
                        float eps, void* stream);
int prl_rmsnorm_workspace_bytes(int64_t H, size_t* bytes);
/* dx and dw (bf16, dw reduced over all rows through the fp32 workspace); H <= 5120. */
int prl_rmsnorm_backward(const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                         void* dw, void* workspace, size_t workspace_bytes, int64_t rows, int64_t H,
                         void* stream);
/* The decoder's residual add fused with the norm that reads its result (transformers
 * Qwen2DecoderLayer.forward: `hidden = residual + hidden; ... norm(hidden)`): h = bf16(residual
 * + x) written to h, y = rmsnorm(h).  Backward: dx = bf16(bf16(rmsnorm'(dy)) + dh), the gradient
 * of both residual and x (dh = gradient reaching h through the residual stream). */
int prl_add_rmsnorm_forward(const void* residual, const void* x, const void* w, void* h, void* y,
                            float* rstd, int64_t rows, int64_t H, float eps, void* stream);
int prl_add_rmsnorm_backward(const void* dy, const void* dh, const void* h, const void* w,
                             const float* rstd, void* dx, void* dw, void* workspace,
                             size_t workspace_bytes, int64_t rows, int64_t H, void* stream);
/* out = bf16(bf16(silu(gate)) * up) over n elements; backward gives dgate, dup.  counter: a
 * caller-owned device uint32 the kernel's workgroups claim chunks from (zeroed by the call,
 * stream-ordered); NULL = a static chunk stride (the same bits). */
int prl_swiglu_forward(const void* gate, const void* up, void* out, int64_t n, uint32_t* counter, void* stream);
int prl_swiglu_backward(const void* dout, const void* gate, const void* up, void* dgate, void* dup,
                        int64_t n, uint32_t* counter, void* stream);
/* The same over [rows, cols] matrices with row strides (elements; cols and strides multiples of 8,
 * pointers 16-B aligned): gate / up as the column halves of one fused gate_up GEMM output, the
 * backward writing dgate / dup into the halves of one [rows, 2 cols] buffer.  Bit-identical to
 * the contiguous forms.  Replaces Qwen2MLP's act_fn(gate_proj(x)) * up_proj(x) (transformers
 * modeling_qwen2.py) run inside the reference's model forward (finetune_loop.py:620-629). */
int prl_swiglu_forward_rows(const void* gate, const void* up, void* out, int64_t rows, int64_t cols,
                            int64_t ld_gate, int64_t ld_up, int64_t ld_out, void* stream);
int prl_swiglu_backward_rows(const void* dout, const void* gate, const void* up, void* dgate, void* dup,
                             int64_t rows, int64_t cols, int64_t ld_dout, int64_t ld_gate, int64_t ld_up,
                             int64_t ld_dgate, int64_t ld_dup, void* stream);
/* q [tokens, hq, d], k [tokens, hkv, d] token-major; cos / sin [tokens, d] (HF layout:
 * halves repeated).  Out-of-place; backward applies the transposed rotation. */
int prl_rope_forward(const void* q, const void* k, const void* cos, const void* sin, void* q_out,
                     void* k_out, int64_t tokens, int32_t hq, int32_t hkv, int32_t d, void* stream);
/* prl_rope_forward with the inputs' token strides given (elements, multiples of 4): q and k read
 * as column ranges of one fused q/k/v projection output [tokens, ld] (outputs contiguous). */
int prl_rope_forward_strided(const void* q, const void* k, const void* cos, const void* sin, void* q_out,
                             void* k_out, int64_t tokens, int32_t hq, int32_t hkv, int32_t d, int64_t ld_q,
                             int64_t ld_k, void* stream);
int prl_rope_backward(const void* dq_out, const void* dk_out, const void* cos, const void* sin,
                      void* dq, void* dk, int64_t tokens, int32_t hq, int32_t hkv, int32_t d,
                      void* stream);

/* ---- Flash-attention backward for packed causal attention (csrc/attn_bwd.hip), bf16,
 * head_dim 128, GQA (q / dout / dq: heads, k / v / dk / dv: kv_heads, heads % kv_heads == 0).
 * Tensors [tokens, heads, 128] token-major.  lse: the forward's log-sum-exp in torch's varlen layout
 * [nseq][heads][lse_len] (sequence b's row starts at token cu_seqlens[b]; lse_len >= its length).
 * Replaces the backward of torch's varlen flash attention used by the trainer's packed
 * attention (finetune/attention.py; the reference's flash-attn varlen, finetune_loop.py:381). */
/* Forward: out [tokens, heads, 128] bf16 and lse2[heads][tokens] = log2 sum_j exp2(log2(e) s S_tj)
 * (the backward's log-sum-exp input, base 2); q_items as for prl_attn_bwd. */
int prl_attn_fwd(const void* q, const void* k, const void* v, const int32_t* q_items,
                 int32_t n_q_items, void* out, float* lse2, int64_t tokens, int32_t heads,
                 int32_t kv_heads, int32_t head_dim, float scale, void* stream);
/* delta[heads][tokens] = rowsum(out * dout) (fp32), when lse2 comes from prl_attn_fwd. */
int prl_attn_bwd_delta(const void* out, const void* dout, float* delta, int64_t tokens,
                       int32_t heads, int32_t head_dim, void* stream);
/* With torch's forward: lse2 = lse * log2(e), delta = rowsum(out * dout), both fp32 [heads][tokens]. */
int prl_attn_bwd_preprocess(const void* out, const void* dout, const float* lse,
                            const int32_t* cu_seqlens, int32_t nseq, int64_t lse_len, float* lse2,
                            float* delta, int64_t tokens, int32_t heads, int32_t head_dim, void* stream);
/* kv_items / q_items: device int32 triplets (seq_start, seq_end, block_start) covering every
 * sequence in 128-key / 128-query blocks.  Writes dq, dk, dv (bf16). */
int prl_attn_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse2,
                 const float* delta, const int32_t* kv_items, int32_t n_kv_items, const int32_t* q_items,
                 int32_t n_q_items, void* dq, void* dk, void* dv, int64_t tokens, int32_t heads,
                 int32_t kv_heads, int32_t head_dim, float scale, void* stream);
/* prl_attn_bwd with heavy dK/dV work split over the query heads of its group: split_units are
 * int32 7-tuples (seq_start, seq_end, block_start, kv_head, head_lo, head_hi, slot) run before the
 * kv_items (which must then leave those key blocks out); each writes fp32 partial dK / dV to
 * parts + slot * 2 * 128 * 128; split_groups are int32 5-tuples (seq_end, block_start, kv_head,
 * first_slot, n_parts) summed in part order into bf16 dk / dv by a second launch (deterministic). */
int prl_attn_bwd_split(const void* q, const void* k, const void* v, const void* dout, const float* lse2,
                       const float* delta, const int32_t* kv_items, int32_t n_kv_items, const int32_t* q_items,
                       int32_t n_q_items, const int32_t* split_units, int32_t n_split, const int32_t* split_groups,
                       int32_t n_groups, float* parts, void* dq, void* dk, void* dv, int64_t tokens, int32_t heads,
                       int32_t kv_heads, int32_t head_dim, float scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PRL_HIP_H */
