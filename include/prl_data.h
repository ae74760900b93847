/* prl_data — host-side C ABI of the trainer's input path (no device code, libprl_data.so).
 *
 * the training_data stream format and the preprocessing that
 * produces it, in native code.
 *   - JSON micro-batch codec.  The stream carries one JSON document per packed micro-batch
 *     (pipelinerl/streams.py:238-277 writes orjson.dumps(model_dump()), the trainer's loader
 *     thread json-decodes it and builds a PipelineBatchEncoding, pipelinerl/finetune_loop.py:92-115,
 *     pipelinerl/finetune/types.py:48-117).  At 65 536 tokens a line is ~7.7 MB: the Python
 *     decode holds the GIL for ~140 ms per micro-batch in the loader thread.  Here the numeric
 *     arrays are decoded straight into caller-owned (pinned) buffers without the GIL, with the
 *     value semantics of the Python path (numpy.asarray(list) then torch.as_tensor(dtype)).
 *   - populate_rl_data group statistics (pipelinerl/finetune/rl/__init__.py:380-501) and the
 *     packed collation (pipelinerl/finetune/data.py:215-279) over flat arrays.
 * Every function returns 0 or a PRL_DATA_E* code; nothing throws across the ABI; buffers are
 * caller-owned; no global state (every function is reentrant).
 */
#ifndef PRL_DATA_H
#define PRL_DATA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRL_DATA_ABI 1

enum PrlDataDtype { PRL_DT_I64 = 0, PRL_DT_I32 = 1, PRL_DT_F32 = 2, PRL_DT_F64 = 3 };

enum PrlDataError {
  PRL_DATA_OK = 0,
  PRL_DATA_EINVAL = 5001,  /* bad argument */
  PRL_DATA_ESYNTAX = 5002, /* not valid JSON */
  PRL_DATA_ESHAPE = 5003,  /* ragged nesting / more than 8 dimensions */
  PRL_DATA_ETYPE = 5004,   /* an element is not a number (string, object, bool, null) */
  PRL_DATA_ECAP = 5005,    /* output capacity too small */
  PRL_DATA_ERANGE = 5006,  /* a value not representable in the requested type (NaN/inf to int) */
};

#define PRL_JSON_MAX_DIMS 8

int prl_data_abi_version(void);
const char* prl_data_error_string(int code);

/* One member of a top-level JSON object: byte offsets into the document. */
typedef struct {
  int64_t key_off, key_len; /* the key's characters, without the quotes (escapes left as is) */
  int64_t val_off, val_len; /* the value's JSON text */
} PrlJsonMember;

/* Splits `doc` (a JSON object) into members.  *n = member count; PRL_DATA_ECAP when > cap
 * (then *n is the count needed). */
int prl_json_members(const char* doc, int64_t len, PrlJsonMember* out, int32_t cap, int32_t* n);

/* A (nested) JSON array of numbers to decode into a dense row-major buffer. */
typedef struct {
  const char* text; /* the array's JSON text */
  int64_t len;
  int32_t dtype;    /* PrlDataDtype of `out` */
  int32_t ndim;     /* set by prl_json_array_shape */
  int64_t shape[PRL_JSON_MAX_DIMS];
  int32_t has_float; /* some element is not an integer literal: numpy would hold float64 */
  int32_t status;    /* per-array result of the last call */
  void* out;         /* caller-owned, prod(shape) elements of dtype */
} PrlJsonArray;

/* Structure pass: rank, shape (rectangular or PRL_DATA_ESHAPE), whether any element is a
 * float literal.  `[]` has ndim 1 and shape [0]. */
int prl_json_array_shape(PrlJsonArray* a);

/* Value pass over n arrays (each already shaped, out set), up to `threads` OS threads.
 * Semantics of numpy.asarray(list) -> torch.as_tensor(dtype): integers parse exactly; when
 * has_float the whole array goes through float64 first (correctly rounded); float64 -> int
 * truncates toward zero; -> float32 rounds to nearest even from the float64; NaN / Infinity /
 * -Infinity literals accepted (Python json's extension).  Returns the first failing status. */
int prl_json_array_fill(PrlJsonArray* arrays, int32_t n, int32_t threads);

/* Upper bound of the text size prl_json_array_format writes for `count` elements. */
int64_t prl_json_format_bound(int64_t count, int32_t ndim, const int64_t* shape);

/* Writes a dense array as nested JSON lists, floats in shortest round-trip form (Python repr
 * digits; NaN / Infinity / -Infinity as Python json writes them). *written = bytes written. */
int prl_json_array_format(const void* data, int32_t dtype, int32_t ndim, const int64_t* shape, char* out,
                          int64_t cap, int64_t* written);

/* populate_rl_data's per-group statistics (rl/__init__.py:447-468): for rollout i in group
 * group_of[i] (0..n_groups-1): mean of reward0 over the group, sample std (ddof = 1; NaN for a
 * single rollout), mean rollout length.  Outputs per group. Sums in the rollouts' order. */
int prl_rl_group_stats(int64_t n_rollouts, const int64_t* group_of, int64_t n_groups, const double* reward0,
                       const int64_t* length, double* mean, double* std, double* tokens_mean);

/* collate_packed's token layout (data.py:215-279) for n examples of lengths[i] tokens,
 * concatenated in ids / labels: packed ids, labels with the first label of every example after
 * the first set to label_pad, position ids restarting at 0, boundaries[n + 1] (cumsum, int32). */
int prl_collate_packed(int64_t n, const int64_t* lengths, const int64_t* ids, const int64_t* labels, int64_t label_pad,
                       int64_t* out_ids, int64_t* out_labels, int64_t* out_pos, int32_t* boundaries);

#ifdef __cplusplus
}
#endif
#endif /* PRL_DATA_H */
