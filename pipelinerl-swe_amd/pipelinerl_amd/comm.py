"""RcclComm: a communicator of the prl_comm C ABI (include/prl_comm.h, libprl_comm.so).

Selected with ``actor_group_backend: prl_comm`` on the trainer (finetune config) and the
actor (``WorkerExtension.actor_group_backend``): the trainer -> actor weight broadcast then
runs on an RCCL communicator owned by this package instead of a torch.distributed process
group.  Rendezvous mirrors ``init_extra_process_group`` (pipelinerl/torch_utils.py:16-65): a
TCP store at the group's ``init_method`` address, rank 0 publishes the RCCL unique id.

Collectives are enqueued on the caller's current HIP stream and return immediately.  Call
``close()`` on every rank when done (RCCL's destroy is not run from a finalizer).
"""

from __future__ import annotations

import ctypes
import weakref
import os
from datetime import timedelta
from pathlib import Path
from urllib.parse import urlparse

import torch  # loaded first: libprl_comm.so then binds torch's own RCCL (same soname)
import torch.distributed as dist

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["PRL_COMM_LIB"]) if os.environ.get("PRL_COMM_LIB") else _PKG / "libprl_comm.so"
HEADER_PATH = _PKG.parents[1] / "include" / "prl_comm.h"
ID_BYTES = 128
F32, BF16, U8, I64 = 0, 1, 2, 3
OPS = {"sum": 0, "avg": 1, "mean": 1, "max": 2}
_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.uint8: U8, torch.int64: I64}

_lib = None


class CommError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists() and not os.environ.get("PRL_COMM_LIB"):
        try:
            from ._build import build_comm

            build_comm()
        except Exception as e:
            raise CommError(f"libprl_comm.so is missing and could not be built: {e}") from e
    try:
        lib = ctypes.CDLL(str(LIB_PATH))
    except OSError as e:
        raise CommError(f"cannot load {LIB_PATH}: {e}") from e
    c = ctypes
    sig = {
        "prl_comm_abi_version": (c.c_int, []),
        "prl_comm_error_string": (c.c_char_p, [c.c_int]),
        "prl_comm_get_unique_id": (c.c_int, [c.c_void_p]),
        "prl_comm_init": (c.c_int, [c.c_void_p, c.c_int, c.c_int, c.c_int, c.POINTER(c.c_void_p)]),
        "prl_comm_broadcast": (c.c_int, [c.c_void_p, c.c_void_p, c.c_size_t, c.c_int, c.c_void_p]),
        "prl_comm_broadcast_buckets": (c.c_int, [c.c_void_p, c.c_void_p, c.c_size_t, c.c_size_t, c.c_int,
                                                 c.c_void_p]),
        "prl_comm_allreduce": (c.c_int, [c.c_void_p, c.c_void_p, c.c_size_t, c.c_int, c.c_int, c.c_void_p]),
        "prl_comm_rank": (c.c_int, [c.c_void_p, c.POINTER(c.c_int)]),
        "prl_comm_size": (c.c_int, [c.c_void_p, c.POINTER(c.c_int)]),
        "prl_comm_destroy": (c.c_int, [c.c_void_p]),
        "prl_comm_abort": (c.c_int, [c.c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc:
        raise CommError(f"{what} failed: {load().prl_comm_error_string(rc).decode()} (code {rc})")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


_LIVE: "weakref.WeakSet[RcclComm]" = weakref.WeakSet()  # this process's open communicators


def abort_all() -> int:
    """Abort every open prl_comm communicator of this process, so a collective that will never
    complete returns (bench.py's probe deadline); returns how many were aborted."""
    n = 0
    for c in list(_LIVE):
        if c._h:
            try:
                c.abort()
                n += 1
            except CommError:
                pass
    return n


class RcclComm:
    def __init__(self, handle: ctypes.c_void_p, rank: int, world: int, device: torch.device, store=None):
        self._h = handle
        self.rank, self.world, self.device = rank, world, device
        self._store = store  # keeps the rendezvous alive while the communicator exists
        _LIVE.add(self)

    @classmethod
    def create(cls, init_method: str, rank: int, world: int, device: torch.device | str | int,
               timeout_s: float = 1800.0, key: str = "prl_comm/actor") -> "RcclComm":
        """Collective over the `world` ranks that rendezvous at ``init_method`` (tcp://host:port)."""
        lib = load()
        device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if device.type != "cuda":
            raise CommError("RcclComm needs a HIP device")
        u = urlparse(init_method)
        if u.scheme != "tcp" or not u.hostname or not u.port:
            raise ValueError(f"prl_comm rendezvous needs tcp://host:port, got {init_method}")
        store = dist.TCPStore(u.hostname, u.port, world, is_master=rank == 0, timeout=timedelta(seconds=timeout_s))
        if rank == 0:
            buf = (ctypes.c_uint8 * ID_BYTES)()
            _check(lib.prl_comm_get_unique_id(buf), "prl_comm_get_unique_id")
            store.set(key, bytes(buf))
        uid = store.get(key)
        if len(uid) != ID_BYTES:
            raise CommError("malformed RCCL unique id from the rendezvous store")
        idbuf = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        _check(lib.prl_comm_init(idbuf, rank, world, idx, ctypes.byref(h)), "prl_comm_init")
        return cls(h, rank, world, torch.device("cuda", idx), store)

    @classmethod
    def from_group(cls, group, device: torch.device | str | int) -> "RcclComm":
        """Collective over the ranks of an initialised torch process group (e.g. a gloo control
        group): rank 0 of ``group`` creates the RCCL unique id and shares it with
        ``broadcast_object_list``; every rank's communicator rank is its rank in ``group``."""
        lib = load()
        device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if device.type != "cuda":
            raise CommError("RcclComm needs a HIP device")
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [None]
        if rank == 0:
            buf = (ctypes.c_uint8 * ID_BYTES)()
            _check(lib.prl_comm_get_unique_id(buf), "prl_comm_get_unique_id")
            box[0] = bytes(buf)
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if not isinstance(box[0], bytes) or len(box[0]) != ID_BYTES:
            raise CommError("malformed RCCL unique id from the group broadcast")
        idbuf = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(box[0])
        h = ctypes.c_void_p()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        _check(lib.prl_comm_init(idbuf, rank, world, idx, ctypes.byref(h)), "prl_comm_init")
        return cls(h, rank, world, torch.device("cuda", idx))

    def reported_size(self) -> int:
        """The communicator's size as RCCL reports it (ncclCommCount through prl_comm_size)."""
        n = ctypes.c_int(-1)
        _check(load().prl_comm_size(self._h, ctypes.byref(n)), "prl_comm_size")
        return int(n.value)

    def reported_rank(self) -> int:
        """This rank in the communicator as RCCL reports it (ncclCommUserRank)."""
        r = ctypes.c_int(-1)
        _check(load().prl_comm_rank(self._h, ctypes.byref(r)), "prl_comm_rank")
        return int(r.value)

    def broadcast(self, t: torch.Tensor, src: int = 0, bucket_bytes: int = 0) -> None:
        if not t.is_contiguous() or t.device.type != "cuda":
            raise CommError("broadcast needs a contiguous HIP tensor")
        nbytes = t.numel() * t.element_size()
        lib = load()
        if bucket_bytes and nbytes > bucket_bytes:
            _check(lib.prl_comm_broadcast_buckets(self._h, t.data_ptr(), nbytes, bucket_bytes, src, _stream(t)),
                   "prl_comm_broadcast_buckets")
        else:
            _check(lib.prl_comm_broadcast(self._h, t.data_ptr(), nbytes, src, _stream(t)), "prl_comm_broadcast")

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None:
        if not t.is_contiguous() or t.device.type != "cuda" or t.dtype not in _DT:
            raise CommError("all_reduce needs a contiguous f32 / bf16 / u8 / i64 HIP tensor")
        _check(load().prl_comm_allreduce(self._h, t.data_ptr(), t.numel(), _DT[t.dtype], OPS[op], _stream(t)),
               "prl_comm_allreduce")

    def close(self) -> None:
        if self._h:
            _check(load().prl_comm_destroy(self._h), "prl_comm_destroy")
            self._h = None

    def abort(self) -> None:
        """Tear the communicator down without waiting for in-flight collectives (a peer died)."""
        if self._h:
            h, self._h = self._h, None
            _check(load().prl_comm_abort(h), "prl_comm_abort")


def broadcast(t: torch.Tensor, group, src: int = 0, async_op: bool = False):
    """``dist.broadcast`` for a torch process group, the prl_comm call for an RcclComm (always
    stream-ordered, returns None)."""
    if isinstance(group, RcclComm):
        group.broadcast(t, src)
        return None
    return dist.broadcast(t, src=src, group=group, async_op=async_op)
