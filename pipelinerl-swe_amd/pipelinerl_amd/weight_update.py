"""Trainer -> actor weight broadcast, MI355X-first (replaces
pipelinerl/finetune_loop.py:118-256 WeightUpdateManager and its messages).

Protocol (unchanged, so unmodified reference actors keep working):
  1. rank 0 POSTs WeightUpdateRequest{version, parameters_info} to every actor's
     /receive_weight_update (thread pool; the actor answers after it has received everything);
  2. rank 0 broadcasts the parameters, bf16, over the "actor" group (RCCL over xGMI),
     strictly in parameters_info order;
  3. when the broadcast and every HTTP call are done, rank 0 appends
     WeightUpdateSuccess{version} to the ``weight_update_request`` topic.
``version`` is the cumulative number of samples trained (finetune_loop.py:795-801).

What changes:
  * snapshot (``snapshot="zero_copy"``, the default for a bf16 model on one HIP device): at the
    first update every parameter is re-homed into ONE flat bf16 buffer in the broadcast layout
    (``p.data`` becomes a view; a one-time copy), so the broadcast reads the parameters in place:
    no per-update copy at all.  The next optimizer step waits (device-side) until the broadcast has
    read them — one step later, long after it finished.  ``snapshot="copy"`` (and any non-bf16 or
    multi-device model): every parameter is packed into a bf16 staging buffer by the HIP flatten
    kernel (prl_flatten_bf16) on a side stream after the optimizer step; measured on MI355X, that
    5.6 ms copy of 7B's 15.23 GB costs the next step about its own duration (it competes for the
    CUs: ``snapshot_overlap`` in the bench line).  Either way the broadcast runs on a side stream
    while the trainer's next passes run on the main stream — overlapped, not blocking (the
    reference idles the trainer for the whole transfer);
  * transport "per_tensor" (compat: one broadcast per parameter, views into the snapshot)
    or "bucketed" (our actors only: ~256 MiB broadcasts of the flat snapshot, 1 call per
    bucket instead of 339 for 7B).  Layout: parameter i starts at an 8-element (16 B)
    aligned offset of the flat buffer; both ends derive it from parameters_info.
"""

from __future__ import annotations

import ctypes
import functools
import os
import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Any, Callable, Literal

import torch
import torch.distributed as dist
from pydantic import BaseModel, Field

from . import comm

logger = logging.getLogger(__name__)

TRAINER_TOPIC = "weight_update_request"


class ParameterInfo(BaseModel):
    name: str
    shape: list[int]
    dtype: str


class WeightUpdateRequest(BaseModel):
    kind: Literal["weight_update_request"] = "weight_update_request"
    version: int
    parameters_info: list[ParameterInfo]
    timestamp: float = Field(default_factory=time.time)
    # extension fields (pydantic models of reference actors ignore unknown keys)
    transport: Literal["per_tensor", "bucketed"] = "per_tensor"
    bucket_bytes: int = 0


class WeightUpdateSuccess(BaseModel):
    kind: Literal["weight_update_success"] = "weight_update_success"
    version: int
    timestamp: float = Field(default_factory=time.time)


class SamplesProcessed(BaseModel):
    kind: Literal["samples_processed"] = "samples_processed"
    samples_processed: int
    timestamp: float = Field(default_factory=time.time)


TrainerMessage = WeightUpdateRequest | WeightUpdateSuccess | SamplesProcessed

ALIGN = 8  # elements: 16-byte aligned parameter slots in the flat bf16 buffer


@dataclass
class FlatLayout:
    names: list[str]
    shapes: list[list[int]]
    numels: list[int]
    offsets: list[int]
    total: int

    @classmethod
    def from_infos(cls, infos: list[ParameterInfo]) -> "FlatLayout":
        names, shapes, numels, offsets, off = [], [], [], [], 0
        for info in infos:
            n = 1
            for s in info.shape:
                n *= int(s)
            names.append(info.name)
            shapes.append(list(info.shape))
            numels.append(n)
            offsets.append(off)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        return cls(names, shapes, numels, offsets, off)

    def buckets(self, bucket_elems: int) -> list[tuple[int, int]]:
        """Contiguous [start, end) element ranges of at most bucket_elems covering the buffer."""
        bucket_elems = max(ALIGN, bucket_elems // ALIGN * ALIGN)
        return [(a, min(a + bucket_elems, self.total)) for a in range(0, self.total, bucket_elems)]


class HipFlatPacker:
    """Parameters <-> flat bf16 buffer with the HIP kernels (prl_flatten_bf16 / prl_unflatten_bf16)."""

    @staticmethod
    def _tables(tensors, offsets):
        from . import _native

        n = len(tensors)
        for t in tensors:
            if t.device.type != "cuda" or not t.is_contiguous() or t.dtype not in (torch.float32, torch.bfloat16):
                raise RuntimeError("HipFlatPacker needs contiguous f32/bf16 HIP tensors")
        P = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tensors])
        D = (ctypes.c_int32 * n)(*[_native.PRL_BF16 if t.dtype == torch.bfloat16 else _native.PRL_F32 for t in tensors])
        N = (ctypes.c_int64 * n)(*[t.numel() for t in tensors])
        O = (ctypes.c_int64 * n)(*offsets)
        return P, D, N, O

    def flatten(self, tensors: list[torch.Tensor], offsets: list[int], flat: torch.Tensor) -> None:
        from . import _native

        lib = _native.load()
        P, D, N, O = self._tables(tensors, offsets)
        st = torch.cuda.current_stream(flat.device).cuda_stream
        _native.check(lib.prl_flatten_bf16(P, D, N, O, len(tensors), flat.data_ptr(), st), "prl_flatten_bf16")

    def unflatten(self, flat: torch.Tensor, tensors: list[torch.Tensor], offsets: list[int]) -> None:
        from . import _native

        lib = _native.load()
        P, D, N, O = self._tables(tensors, offsets)
        st = torch.cuda.current_stream(flat.device).cuda_stream
        _native.check(lib.prl_unflatten_bf16(flat.data_ptr(), P, D, N, O, len(tensors), st), "prl_unflatten_bf16")
        # written through raw pointers: move the version counters as an in-place copy_ would
        from torch.autograd.graph import increment_version

        from .finetune.model_ops import weights_written

        increment_version(tensors)
        weights_written()


def parameters_info(named: list[tuple[str, torch.Tensor]]) -> list[ParameterInfo]:
    """The request's parameter list (finetune_loop.py:192-196): one entry per named parameter, in
    order, full shape (a sharded parameter reports its global shape, as ZeRO-3's ds_shape does),
    dtype always bf16 (what is broadcast)."""
    return [ParameterInfo(name=n, shape=list(p.shape), dtype=str(torch.bfloat16)) for n, p in named]


def unwrap_model(model):
    m = getattr(model, "module", model)
    return getattr(m, "pretrained_model", m)  # value-head wrapper: broadcast the LM only


def lm_namespace(model, named: list[tuple[str, torch.Tensor]]) -> list[tuple[str, torch.Tensor]]:
    """Names relative to (the FSDP root of) ``model`` -> the language model's own names: under a
    value-head wrapper (sharded as the root, so its units also hold the LM's embedding, norm and
    lm_head) the ``pretrained_model.`` prefix goes and the value head's parameters are dropped."""
    m = getattr(model, "module", model)
    if not hasattr(m, "pretrained_model"):
        return named
    pre = "pretrained_model."
    return [(n[len(pre):], t) for n, t in named if n.startswith(pre)]


class WeightUpdateError(RuntimeError):
    """An actor refused or failed a weight update, or the update did not complete in time."""


def http_post_request(url: str, message: BaseModel, timeout: float | None = 600.0) -> None:
    """POST the request to one actor; raises WeightUpdateError on any HTTP error or timeout.
    The reference logs and carries on (finetune_loop.py:157-166), after which its broadcast waits
    in NCCL for an actor that will never join; here the error reaches the trainer."""
    import requests

    response = None
    try:
        response = requests.post(url + "/receive_weight_update", json=message.model_dump(), timeout=timeout)
        response.raise_for_status()
    except requests.RequestException as e:
        logger.error(f"Error sending weight update request to {url}: {e}")
        detail = f" - {response.status_code} {response.text[:200]}" if response is not None else ""
        if response is not None:
            logger.error(f"Response: {response.status_code} - {response.text}")
        raise WeightUpdateError(f"weight update request to {url} failed: {e}{detail}") from e


class WeightUpdateManager:
    def __init__(self, llm_urls: list[str], accelerated_model, update_stream, actor_update_group, *,
                 transport: str = "per_tensor", bucket_bytes: int = 256 << 20, overlap: bool = True,
                 packer=None, post: Callable[[str, BaseModel], None] | None = None, is_main: bool = True,
                 write_message: Callable[[Any, BaseModel], None] | None = None, timeout_s: float | None = 900.0,
                 http_timeout_s: float | None = 600.0, snapshot: str = "zero_copy"):
        """``snapshot``: "zero_copy" (the parameters are broadcast in place: call
        ``before_optimizer_step()`` before writing them — the trainer loop does, before every
        optimizer step) or "copy" (a staging copy per update; the parameters may be written at once).
        ``timeout_s``: an update (every actor's HTTP answer and the whole broadcast) that has not
        completed this long after its request raises WeightUpdateError from the next ``wait()`` /
        ``send_weight_update()``; so does any actor's HTTP error, as soon as it arrives.  A failed
        update aborts an RcclComm actor group (in-flight broadcasts return) — the trainer exits
        instead of hanging in the collective (failure handling)."""
        if snapshot not in ("zero_copy", "copy"):
            raise ValueError(f"snapshot must be 'zero_copy' or 'copy', got {snapshot!r}")
        self.snapshot = snapshot
        self._flat_params: torch.Tensor | None = None
        self._snapshot_done = None  # event after the staging copy, or (zero-copy) the broadcast's last read
        self._works: list = []  # zero-copy: the in-flight broadcast's works
        self._version: int | None = None
        self._deadline: float | None = None  # the in-flight update's request time + timeout_s
        self.llm_urls = list(llm_urls)
        self.model = accelerated_model
        self.update_stream = update_stream
        self.group = actor_update_group
        self.transport = transport
        self.bucket_bytes = int(bucket_bytes)
        self.overlap = overlap
        self.packer = packer or HipFlatPacker()
        self.post = post or functools.partial(http_post_request, timeout=http_timeout_s)
        self.timeout_s = timeout_s
        self.is_main = is_main
        self.pool = ThreadPoolExecutor(max_workers=max(1, len(self.llm_urls)))
        self._write_message = write_message
        self._staging: torch.Tensor | None = None
        self._stream = None
        self._inflight: threading.Thread | None = None
        self._error: BaseException | None = None
        self.last_latency_s: float | None = None
        self.completed_versions: list[int] = []

    # -- helpers -------------------------------------------------------------------------
    def named_parameters(self) -> list[tuple[str, torch.Tensor]]:
        return list(unwrap_model(self.model).named_parameters())

    def _emit(self, msg: BaseModel) -> None:
        if self._write_message is not None:
            self._write_message(self.update_stream, msg)
            return
        from .streams import write_to_streams

        with write_to_streams(self.update_stream) as w:
            w.write(msg)

    def _zero_copy_flat(self, named, layout: FlatLayout) -> torch.Tensor | None:
        """The flat buffer the parameters live in (re-homed on first use unless the loop already did
        it at load: ``rehome_parameters``), or None when the model cannot be broadcast in place
        (snapshot="copy", a non-bf16 or non-contiguous parameter, or several devices): then the
        staging copy is used."""
        if self.snapshot != "zero_copy" or not named:
            return None
        flat = self._flat_params
        if flat is None or flat_home(named, layout) is None:
            flat = rehome_parameters(self.model)
            if flat is not None:
                logger.info(f"weight updates broadcast the parameters in place ({len(named)} tensors, "
                            f"{2 * layout.total / 1e9:.2f} GB)")
        self._flat_params = flat
        return flat

    def _ensure_staging(self, total: int, device: torch.device) -> torch.Tensor:
        if self._staging is None or self._staging.numel() < total or self._staging.device != device:
            self._staging = torch.empty(total, dtype=torch.bfloat16, device=device)
        return self._staging[:total]

    # -- protocol ------------------------------------------------------------------------
    def send_weight_update(self, version: int) -> None:
        self.wait()
        named = self.named_parameters()
        sharded = _is_sharded(named)
        if not self.is_main and not sharded:
            return
        infos = parameters_info(named)
        layout = FlatLayout.from_infos(infos)
        dev = named[0][1].device
        if sharded:
            # FSDP (finetune_loop.py:222-247 gathers a FULL_STATE_DICT): every rank takes part in
            # one all-gather per FSDP unit, rank 0 packs each unit's parameters into its staging
            # buffer in stream order, so the snapshot precedes the next optimizer step without an event.
            from .finetune.sharding import gather_units

            flat = self._ensure_staging(layout.total, dev) if self.is_main else None
            index = {n: i for i, (n, _) in enumerate(named)}
            seen = set()
            for unit in gather_units(getattr(self.model, "module", self.model)):  # the FSDP root's units
                unit = lm_namespace(self.model, unit)
                seen.update(n for n, _ in unit)
                if self.is_main:
                    self.packer.flatten([t for _, t in unit], [layout.offsets[index[n]] for n, _ in unit], flat)
            if seen != set(index):
                raise RuntimeError(f"FSDP units do not cover the model's parameters: missing {sorted(set(index) - seen)[:4]}, "
                                   f"extra {sorted(seen - set(index))[:4]}")
            if not self.is_main:
                return
        request = WeightUpdateRequest(version=version, parameters_info=infos, transport=self.transport,
                                      bucket_bytes=self.bucket_bytes if self.transport == "bucketed" else 0)
        t0 = time.time()
        self._version = version
        self._deadline = t0 + float(self.timeout_s) if self.timeout_s else None
        futures = [self.pool.submit(self.post, url, request) for url in self.llm_urls]
        logger.info(f"Published weight update request for version {version}")
        params = [p.detach() for _, p in named]
        in_place = None if sharded else self._zero_copy_flat(named, layout)
        if in_place is not None:
            flat = in_place
        elif not sharded:
            flat = self._ensure_staging(layout.total, dev)
        on_gpu = dev.type == "cuda"
        if on_gpu:
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=dev, priority=side_stream_priority(self.group))
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(dev))
            ctx = torch.cuda.stream(self._stream)
        else:
            ctx = _nullcontext()
        works = []
        with ctx:
            if on_gpu:
                self._stream.wait_event(ready)  # snapshot after the optimizer step
            if not sharded and in_place is None:
                self.packer.flatten(params, layout.offsets, flat)
            if on_gpu and in_place is None:
                self._snapshot_done = torch.cuda.Event()
                self._snapshot_done.record(self._stream)
            if self.transport == "bucketed":
                elems = max(ALIGN, self.bucket_bytes // 2)
                for a, b in layout.buckets(elems):
                    works.append(comm.broadcast(flat[a:b], self.group, src=0, async_op=True))
            else:
                for shape, n, off in zip(layout.shapes, layout.numels, layout.offsets):
                    works.append(comm.broadcast(flat[off:off + n].view(shape), self.group, src=0, async_op=True))
            works = [w for w in works if w is not None]  # RcclComm calls are stream-ordered
            done = None
            if on_gpu and self._stream_ordered():
                for w in works:  # RCCL: makes the side stream (not the host) wait for the comm
                    w.wait()
                done = torch.cuda.Event()
                done.record(self._stream)
            # (a gloo group on device tensors — one-GPU tests and rehearsals — completes on gloo's
            # own threads: the watcher and before_optimizer_step poll its works, never a host wait)
            if in_place is not None:  # the parameters are read until the broadcast ends
                self._snapshot_done = done
                self._works = works

        def finish():
            try:
                deadline = None if not self.timeout_s else t0 + float(self.timeout_s)
                fixed = os.environ.get("PRL_WU_POLL_S")  # measurement control: a fixed poll interval
                delay = float(fixed) if fixed else 0.001
                while True:  # an actor's HTTP error ends the wait at once, not the collective
                    for url, f in zip(self.llm_urls, futures):
                        if f.done() and f.exception() is not None:
                            raise f.exception()
                    comm_done = done.query() if done is not None else all(w.is_completed() for w in works)
                    if comm_done and all(f.done() for f in futures):
                        break
                    if deadline is not None and time.time() > deadline:
                        waiting = [u for u, f in zip(self.llm_urls, futures) if not f.done()]
                        raise WeightUpdateError(
                            f"weight update {version} not completed after {self.timeout_s:.0f} s "
                            f"(broadcast {'done' if comm_done else 'in flight'}; actors not answered: {waiting})")
                    time.sleep(delay)
                    delay = delay if fixed else min(delay * 2, 0.02)
                if done is None:
                    for w in works:  # gloo: surfaces a failed work's error
                        w.wait()
                self.last_latency_s = time.time() - t0
                logger.info(f"Finished broadcasting weights for version {version} in {self.last_latency_s:.3f}s")
                self._emit(WeightUpdateSuccess(version=version))
                self.completed_versions.append(version)
            except BaseException as e:  # surfaced on the next wait()
                logger.error(f"weight update {version} failed: {e}")
                self._error = e
                abort = getattr(self.group, "abort", None)
                if callable(abort):  # RcclComm: in-flight broadcasts return instead of hanging
                    try:
                        abort()
                    except Exception as ae:  # noqa: BLE001
                        logger.error(f"aborting the actor group failed: {ae}")

        if self.overlap:
            self._inflight = threading.Thread(target=finish, name=f"weight-update-{version}", daemon=True)
            self._inflight.start()
        else:
            finish()
            self._raise()

    def before_optimizer_step(self) -> None:
        """Order the next in-place parameter update after the snapshot: after the staging copy, or
        (zero-copy) after the broadcast's last read of the parameters.  On a torch group the
        zero-copy wait is bounded: the host polls the broadcast's completion (its event on a device,
        the works of a gloo group) every <= 1 ms between checks of the watcher's error and the
        update's deadline, and raises WeightUpdateError instead of blocking past ``timeout_s`` on an
        actor that never receives.  The broadcast started one step earlier, so it is normally
        complete at the first check and the host goes on at once; the device-side event wait then
        orders the optimizer's writes after its reads.  On an RcclComm group the broadcasts are
        stream-ordered with no host handle: the device-side wait alone orders the writes, and the
        watcher thread bounds it — a failed or timed-out update aborts the communicator
        (``finish`` below), which ends the in-flight broadcast kernels and so the wait."""
        ev = getattr(self, "_snapshot_done", None)
        self._snapshot_done = None
        works, self._works = self._works, []
        if works and ev is not None:  # zero-copy on a device: the broadcast reads the parameters
            self._await_reads(ev.query)
        elif works and not self._stream_ordered():
            self._await_reads(lambda: all(w.is_completed() for w in works))
            for w in works:
                w.wait()  # complete: surfaces a failed work's error
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    def _stream_ordered(self) -> bool:
        """RCCL (an RcclComm or a torch "nccl" group): collectives are ordered on HIP streams."""
        return isinstance(self.group, comm.RcclComm) or "nccl" in str(_backend_of(self.group))

    def _await_reads(self, done: Callable[[], bool]) -> None:
        delay = 0.0002
        while not done():
            self._raise()  # the watcher's error (an actor's HTTP error, its own timeout)
            if self._deadline is not None and time.time() > self._deadline:
                raise WeightUpdateError(f"weight update {self._version} still reading the parameters "
                                        f"{self.timeout_s:.0f} s after its request: the next optimizer step "
                                        "cannot write them (an actor is not receiving)")
            time.sleep(delay)
            delay = min(delay * 2, 0.001)  # at most 1 ms late after the broadcast's last read

    def wait(self) -> None:
        """Block until the in-flight update (if any) has been received by every actor."""
        if self._inflight is not None:
            self._inflight.join()
            self._inflight = None
        self._raise()

    def poll(self) -> None:
        """Raise a failed in-flight update's error now, without waiting for a running one."""
        if self._inflight is not None and not self._inflight.is_alive():
            self._inflight.join()
            self._inflight = None
        self._raise()

    def _raise(self):
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    def close(self) -> None:
        self.wait()
        self.pool.shutdown(wait=True)


def side_stream_priority(group=None) -> int:
    """Priority of the broadcast's side stream (torch: lower is higher): high when the broadcast runs
    on the device (an RCCL group or RcclComm; ``group`` None: assume so), so the runtime maps it to a
    hardware queue of its own (a normal-priority stream may share a hardware queue with the trainer's
    compute stream, and kernels in one hardware queue run in order; tools/queue_probe.py).  A gloo
    group broadcasts from host copies: normal (grad_sync.GradBuckets: several ranks sharing one GPU
    over gloo, each holding high-priority queues, stalled).  PRL_WU_STREAM_PRIORITY=normal: a pool
    stream (A/B)."""
    import os

    if os.environ.get("PRL_WU_STREAM_PRIORITY", "high") == "normal":
        return 0
    if group is not None and isinstance(group, dist.ProcessGroup):
        try:
            if "nccl" not in str(dist.get_backend(group)):
                return 0
        except (RuntimeError, ValueError):
            pass
    return -1


def flat_home(named, layout: FlatLayout) -> torch.Tensor | None:
    """The 1-D bf16 buffer the parameters already live in, laid out as ``layout`` (parameter i at
    element ``layout.offsets[i]``), as a view from parameter 0 on; None when they do not."""
    params = [p for _, p in named]
    if not params or any(p.dtype != torch.bfloat16 or not p.is_contiguous() for p in params):
        return None
    p0 = params[0]
    try:
        st = p0.untyped_storage()
        base = p0.storage_offset()
        if any(p.untyped_storage().data_ptr() != st.data_ptr() or p.storage_offset() - base != off
               for p, off in zip(params, layout.offsets)):
            return None
        if st.nbytes() < (base + layout.total) * 2:
            return None
    except Exception:  # noqa: BLE001 - a tensor without an ordinary storage
        return None
    return p0.detach().as_strided((layout.total,), (1,), base)


def rehome_parameters(model) -> torch.Tensor | None:
    """Put every parameter of (the language model of) ``model`` into ONE bf16 buffer laid out as the
    weight broadcast's flat layout (``FlatLayout`` of ``parameters_info``: named_parameters order,
    16-B aligned slots): ``p.data`` becomes a view of it — the same Parameter objects, optimizer
    state, hooks and ties.  The broadcast then reads the parameters in place (no per-update copy),
    and adjacent projections (gate_proj / up_proj) are one tensor without a concatenation copy
    (finetune/model_ops.py ``_fused_weight``).  Returns the buffer, or None when the model does not
    qualify (FSDP DTensors, a non-bf16 or non-contiguous parameter, several devices).  A one-time
    copy; idempotent (an already re-homed model is returned as it is)."""
    m = unwrap_model(model)
    named = list(m.named_parameters())
    if not named or _is_sharded(named):
        return None
    params = [p for _, p in named]
    dev = params[0].device
    if any(p.dtype != torch.bfloat16 or p.device != dev or not p.is_contiguous() for p in params):
        return None
    layout = FlatLayout.from_infos(parameters_info(named))
    existing = flat_home(named, layout)
    if existing is not None:
        return existing
    from .finetune.model_ops import weights_written

    flat = torch.zeros(layout.total, dtype=torch.bfloat16, device=dev)  # padding gaps stay 0
    with torch.no_grad():
        for p, off in zip(params, layout.offsets):
            view = flat[off:off + p.numel()].view(p.shape)
            view.copy_(p.data)
            p.data = view
    weights_written()
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()  # the old storages are released after the copies
    m._prl_flat_params = True  # checkpoints save host copies (safetensors refuses shared storage)
    return flat


def _backend_of(group) -> str:
    try:
        return dist.get_backend(group)
    except Exception:  # noqa: BLE001 - not a torch process group
        return ""


def _is_sharded(named) -> bool:
    from torch.distributed.tensor import DTensor

    return any(isinstance(p, DTensor) for _, p in named)


class _nullcontext:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
