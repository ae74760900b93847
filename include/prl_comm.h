/* prl_comm — C ABI over RCCL (xGMI) for the trainer's two exchange steps.
 *
 * SURVEY.md §8(b) proposes this surface for callers outside PyTorch (e.g. an inference engine
 * receiving the trainer's weights without torch.distributed):
 *   trainer -> actor weight broadcast   pipelinerl/finetune_loop.py:202-205,246-247 (send),
 *                                       pipelinerl/vllm1.py:84-93 (receive),
 *                                       group rendezvous pipelinerl/torch_utils.py:16-65
 *   DP gradient all-reduce              behind pipelinerl/finetune_loop.py:620-656 (DeepSpeed)
 * One communicator per group; every call is asynchronous on the caller's stream; buffers are
 * caller-owned device memory.  Returns 0 on success, PRL_COMM_E_BASE + ncclResult_t for an
 * RCCL error, PRL_COMM_E_INVALID for bad arguments.  Built as libprl_comm.so (links RCCL);
 * libprl_hip.so does not depend on it.
 */
#ifndef PRL_COMM_H
#define PRL_COMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRL_COMM_ID_BYTES 128
#define PRL_COMM_E_INVALID 3001
#define PRL_COMM_E_BASE 3100

enum PrlCommDtype { PRL_COMM_F32 = 0, PRL_COMM_BF16 = 1, PRL_COMM_U8 = 2, PRL_COMM_I64 = 3 };
enum PrlCommOp { PRL_COMM_SUM = 0, PRL_COMM_AVG = 1, PRL_COMM_MAX = 2 };

int prl_comm_abi_version(void);
const char* prl_comm_error_string(int code);

/* Rank 0 creates the id and shares it out of band (the Python side uses the group's TCP
 * store, as torch_utils.init_extra_process_group does). */
int prl_comm_get_unique_id(uint8_t out[PRL_COMM_ID_BYTES]);

/* Collective over `world` ranks: every rank calls it with the same id.  `device` is the HIP
 * device the communicator's buffers live on. */
int prl_comm_init(const uint8_t id[PRL_COMM_ID_BYTES], int rank, int world, int device, void** comm);

/* In-place broadcast of `bytes` bytes from `root`. */
int prl_comm_broadcast(void* comm, void* buf, size_t bytes, int root, void* stream);

/* In-place broadcast of a flat buffer as consecutive `bucket_bytes` pieces inside one RCCL
 * group call (one launch, RCCL pipelines the pieces). */
int prl_comm_broadcast_buckets(void* comm, void* buf, size_t bytes, size_t bucket_bytes, int root,
                               void* stream);

/* In-place all-reduce of `count` elements. */
int prl_comm_allreduce(void* comm, void* buf, size_t count, int dtype, int op, void* stream);

/* This rank / the communicator's size as RCCL reports them (ncclCommUserRank / ncclCommCount). */
int prl_comm_rank(void* comm, int* rank);
int prl_comm_size(void* comm, int* world);
int prl_comm_destroy(void* comm);
/* Abort: frees the communicator without waiting for in-flight collectives, which return (no
 * hang) — the trainer's way out when an actor died mid-broadcast (the reference
 * blocks in NCCL until the process-group timeout, finetune_loop.py:155-172). */
int prl_comm_abort(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* PRL_COMM_H */
