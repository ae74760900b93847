// prl_comm: thin C ABI over RCCL for the weight broadcast and the gradient all-reduce
// (include/prl_comm.h).  No kernels of its own: RCCL moves the bytes over xGMI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <new>

#include "prl_comm.h"

namespace {

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 0, device = 0;
};

int rc(ncclResult_t r) { return r == ncclSuccess ? 0 : PRL_COMM_E_BASE + (int)r; }

bool dtype_of(int d, ncclDataType_t* out) {
  switch (d) {
    case PRL_COMM_F32: *out = ncclFloat32; return true;
    case PRL_COMM_BF16: *out = ncclBfloat16; return true;
    case PRL_COMM_U8: *out = ncclUint8; return true;
    case PRL_COMM_I64: *out = ncclInt64; return true;
    default: return false;
  }
}

bool op_of(int o, ncclRedOp_t* out) {
  switch (o) {
    case PRL_COMM_SUM: *out = ncclSum; return true;
    case PRL_COMM_AVG: *out = ncclAvg; return true;
    case PRL_COMM_MAX: *out = ncclMax; return true;
    default: return false;
  }
}

}  // namespace

extern "C" {

int prl_comm_abi_version(void) { return 1; }

const char* prl_comm_error_string(int code) {
  if (code == 0) return "ok";
  if (code == PRL_COMM_E_INVALID) return "invalid argument";
  if (code >= PRL_COMM_E_BASE) return ncclGetErrorString(static_cast<ncclResult_t>(code - PRL_COMM_E_BASE));
  return "unknown error";
}

int prl_comm_get_unique_id(uint8_t out[PRL_COMM_ID_BYTES]) {
  if (!out) return PRL_COMM_E_INVALID;
  ncclUniqueId id;
  const int r = rc(ncclGetUniqueId(&id));
  if (r) return r;
  memcpy(out, id.internal, PRL_COMM_ID_BYTES);
  return 0;
}

int prl_comm_init(const uint8_t id[PRL_COMM_ID_BYTES], int rank, int world, int device, void** comm) {
  if (!id || !comm || world < 1 || rank < 0 || rank >= world) return PRL_COMM_E_INVALID;
  if (hipSetDevice(device) != hipSuccess) return PRL_COMM_E_INVALID;
  ncclUniqueId u;
  memcpy(u.internal, id, PRL_COMM_ID_BYTES);
  Comm* c = new (std::nothrow) Comm;
  if (!c) return PRL_COMM_E_INVALID;
  const int r = rc(ncclCommInitRank(&c->comm, world, u, rank));
  if (r) {
    delete c;
    return r;
  }
  c->rank = rank;
  c->world = world;
  c->device = device;
  *comm = c;
  return 0;
}

int prl_comm_broadcast(void* comm, void* buf, size_t bytes, int root, void* stream) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || (!buf && bytes) || root < 0 || root >= c->world) return PRL_COMM_E_INVALID;
  if (!bytes) return 0;
  return rc(ncclBroadcast(buf, buf, bytes, ncclUint8, root, c->comm, static_cast<hipStream_t>(stream)));
}

int prl_comm_broadcast_buckets(void* comm, void* buf, size_t bytes, size_t bucket_bytes, int root, void* stream) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || (!buf && bytes) || root < 0 || root >= c->world || bucket_bytes == 0) return PRL_COMM_E_INVALID;
  if (!bytes) return 0;
  int r = rc(ncclGroupStart());
  if (r) return r;
  char* p = static_cast<char*>(buf);
  for (size_t off = 0; off < bytes; off += bucket_bytes) {
    const size_t n = bytes - off < bucket_bytes ? bytes - off : bucket_bytes;
    r = rc(ncclBroadcast(p + off, p + off, n, ncclUint8, root, c->comm, static_cast<hipStream_t>(stream)));
    if (r) break;
  }
  const int e = rc(ncclGroupEnd());
  return r ? r : e;
}

int prl_comm_allreduce(void* comm, void* buf, size_t count, int dtype, int op, void* stream) {
  Comm* c = static_cast<Comm*>(comm);
  ncclDataType_t dt;
  ncclRedOp_t o;
  if (!c || (!buf && count) || !dtype_of(dtype, &dt) || !op_of(op, &o)) return PRL_COMM_E_INVALID;
  if (!count) return 0;
  return rc(ncclAllReduce(buf, buf, count, dt, o, c->comm, static_cast<hipStream_t>(stream)));
}

// rank / size as RCCL itself reports them (ncclCommUserRank / ncclCommCount), not the values
// the caller passed to prl_comm_init: a census of a running job checks one against the other
int prl_comm_rank(void* comm, int* rank) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || !rank) return PRL_COMM_E_INVALID;
  return rc(ncclCommUserRank(c->comm, rank));
}

int prl_comm_size(void* comm, int* world) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || !world) return PRL_COMM_E_INVALID;
  return rc(ncclCommCount(c->comm, world));
}

int prl_comm_destroy(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return PRL_COMM_E_INVALID;
  const int r = rc(ncclCommDestroy(c->comm));
  delete c;
  return r;
}

int prl_comm_abort(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return PRL_COMM_E_INVALID;
  const int r = rc(ncclCommAbort(c->comm));
  delete c;
  return r;
}

}  // extern "C"
