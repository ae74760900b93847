"""Data-parallel gradient synchronisation for the trainer (replaces Accelerate/DeepSpeed's
gradient all-reduce behind finetune_loop.py:620-656).

Gradients live in flat per-bucket buffers (``param.grad`` are views), so a bucket is reduced
in place by ONE collective.  Buckets follow reverse parameter order (≈ the order backward
produces gradients).  Micro-batches accumulate locally; on the boundary micro-batch of an
optimizer step (``arm()``), a post-accumulate-grad hook launches each bucket's all-reduce on
a side stream the moment its last gradient lands, so the reduction of early buckets
overlaps the rest of the backward — the DP exchange is RCCL over xGMI on MI355X.

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per GPU), and ring collectives are
per-link bound, so buckets are large (default 256 MiB) to amortise the per-call latency;
one step's all-reduce is amortised over every micro-batch of the step.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.distributed as dist


@dataclass
class _Bucket:
    params: list[torch.Tensor]
    flat: torch.Tensor
    pending: int = 0
    work: object = None
    launched: bool = False
    members: set = field(default_factory=set)


class GradBuckets:
    def __init__(self, params, group=None, bucket_bytes: int = 256 << 20, reduce: str = "mean",
                 world: int | None = None):
        """``world``: the group's size when no process group exists (measurement subclasses that
        replace the collective, trainer_probe.EmulatedRingBuckets); else the group's own."""
        if reduce not in ("mean", "sum"):
            raise ValueError("reduce must be 'mean' or 'sum'")
        self.group = group
        self.world = int(world) if world is not None else dist.get_world_size(group)
        self.reduce = reduce
        params = [p for p in params if p.requires_grad]
        self.buckets: list[_Bucket] = []
        cur: list[torch.Tensor] = []
        cur_bytes = 0
        order = list(reversed(params))  # roughly the order the backward produces them
        for p in params:  # a parameter that must sit right after another (rows of one fused GEMM)
            f = getattr(p, "_prl_follows", None)
            if f is not None and any(q is f for q in order):
                order.pop(next(i for i, q in enumerate(order) if q is p))  # by identity (tensor == is elementwise)
                order.insert(next(i for i, q in enumerate(order) if q is f) + 1, p)
        for p in order:
            nbytes = p.numel() * p.element_size()
            if cur and (cur_bytes + nbytes > bucket_bytes or p.dtype != cur[0].dtype or p.device != cur[0].device):
                self._make(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nbytes
        if cur:
            self._make(cur)
        self._owner = {id(p): b for b in self.buckets for p in b.params}
        self.armed = False
        dev = params[0].device if params else torch.device("cpu")
        self.on_gpu = dev.type == "cuda"
        # High priority when the collectives it orders run on the device (RCCL, or their emulation:
        # ``world`` given): a hardware queue of its own — a normal-priority stream created here shares
        # the compute stream's queue (GPU_MAX_HW_QUEUES 4; measured, profiles/r06_queue_probe.json), and
        # the collectives would wait behind the backward's kernels (tools/queue_probe.py).  A gloo group
        # reduces on the host (its device work is two copies), so its stream stays normal: several
        # ranks sharing one GPU over gloo (the one-GPU rehearsals) each holding high-priority queues
        # stalled the 4-rank trainer-step probe for minutes (16 s with normal priority).
        on_device = world is not None or "nccl" in str(dist.get_backend(group))
        self.stream = torch.cuda.Stream(device=dev, priority=-1 if on_device else 0) if self.on_gpu else None
        self._avg = self.on_gpu and world is None and dist.get_backend(group) == "nccl" and reduce == "mean"
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in params]
        for p in params:  # model_ops._wgrad may add into .grad in the GEMM while not armed (no hook due)
            p._prl_grad_buckets = self

    def _make(self, ps: list[torch.Tensor]) -> None:
        total = sum(p.numel() for p in ps)
        flat = torch.zeros(total, dtype=ps[0].dtype, device=ps[0].device)
        off = 0
        for p in ps:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.buckets.append(_Bucket(params=ps, flat=flat, members={id(p) for p in ps}))

    def zero_(self) -> None:
        for b in self.buckets:
            b.flat.zero_()

    def arm(self) -> None:
        """The next backward is the last micro-batch of the step: reduce as gradients land."""
        self.armed = True
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
            b.work = None

    def _launch(self, b: _Bucket) -> None:
        b.launched = True
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        if self.on_gpu:
            self.stream.wait_stream(torch.cuda.current_stream(b.flat.device))
            with torch.cuda.stream(self.stream):
                b.work = dist.all_reduce(b.flat, op=op, group=self.group, async_op=True)
        else:
            b.work = dist.all_reduce(b.flat, op=op, group=self.group, async_op=True)

    def _hook(self, p: torch.Tensor) -> None:
        if not self.armed:
            return
        b = self._owner[id(p)]
        b.pending -= 1
        if b.pending == 0 and not b.launched:
            self._launch(b)

    def finish(self) -> None:
        """Complete every bucket's reduction (buckets whose params got no gradient this pass
        are reduced now) and make the current stream wait for them."""
        if not self.armed:
            return
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        for b in self.buckets:
            b.work.wait()
        if self.on_gpu:
            torch.cuda.current_stream(self.buckets[0].flat.device).wait_stream(self.stream)
        if self.reduce == "mean" and not self._avg and self.world > 1:
            for b in self.buckets:
                b.flat.div_(self.world)
        self.armed = False

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
