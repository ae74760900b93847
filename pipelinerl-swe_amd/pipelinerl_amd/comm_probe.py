"""Measure the two exchange steps of the trainer on the real code paths (bench.py at N > 1).

  grad_allreduce_probe  the DP gradient all-reduce as the trainer runs it: GradBuckets
                        (finetune/grad_sync.py) over gradients shaped like the model's
                        parameters, every bucket launched as if backward had produced it,
                        then finish() (one exchange per optimizer step)
  broadcast_probe       the trainer -> actor weight broadcast: WeightUpdateManager
                        (weight_update.py, rank 0) snapshotting a model-shaped module and
                        broadcasting it; every other rank receives it with
                        WorkerExtension.receive_weight_update (actor.py) into its own module
                        (finetune_loop.py:174-256, vllm1.py:81-94)

Both check their result (the reduced mean, the received bytes) and return timings.  The
parameter shapes are the published Qwen2 layouts.
"""

from __future__ import annotations

import time

import torch
import torch.distributed as dist

QWEN2 = {  # config.json of the published checkpoints
    "0.5b": dict(hidden=896, inter=4864, layers=24, heads=14, kv=2, vocab=151936, tied=True),
    "1.5b": dict(hidden=1536, inter=8960, layers=28, heads=12, kv=2, vocab=151936, tied=True),
    "7b": dict(hidden=3584, inter=18944, layers=28, heads=28, kv=4, vocab=152064, tied=False),
    "32b": dict(hidden=5120, inter=27648, layers=64, heads=40, kv=8, vocab=152064, tied=False),
}


def qwen2_param_shapes(name: str, layers: int | None = None) -> list[tuple[str, tuple[int, ...]]]:
    """named_parameters() order and shapes of Qwen2ForCausalLM (``layers``: only that many decoder
    layers, as trainer_probe.qwen2_model(layers=) builds)."""
    c = dict(QWEN2[name])
    if layers:
        c["layers"] = layers
    H, I, kvd = c["hidden"], c["inter"], c["hidden"] // c["heads"] * c["kv"]
    out = [("model.embed_tokens.weight", (c["vocab"], H))]
    for i in range(c["layers"]):
        p = f"model.layers.{i}."
        out += [(p + "self_attn.q_proj.weight", (H, H)), (p + "self_attn.q_proj.bias", (H,)),
                (p + "self_attn.k_proj.weight", (kvd, H)), (p + "self_attn.k_proj.bias", (kvd,)),
                (p + "self_attn.v_proj.weight", (kvd, H)), (p + "self_attn.v_proj.bias", (kvd,)),
                (p + "self_attn.o_proj.weight", (H, H)),
                (p + "mlp.gate_proj.weight", (I, H)), (p + "mlp.up_proj.weight", (I, H)),
                (p + "mlp.down_proj.weight", (H, I)),
                (p + "input_layernorm.weight", (H,)), (p + "post_attention_layernorm.weight", (H,))]
    out.append(("model.norm.weight", (H,)))
    if not c["tied"]:
        out.append(("lm_head.weight", (c["vocab"], H)))
    return out


class ShapedModule(torch.nn.Module):
    """A module whose named_parameters() are the given (dotted) names and shapes."""

    def __init__(self, shapes, dtype=torch.bfloat16, device="cpu", fill: float | None = None, seed: int = 0):
        super().__init__()
        self._names = []
        g = torch.Generator(device="cpu").manual_seed(seed)
        for name, shape in shapes:
            t = torch.empty(shape, dtype=dtype, device=device)
            if fill is not None:
                t.fill_(fill)
            elif t.numel() < (1 << 22):
                t.copy_(torch.randn(shape, generator=g, dtype=torch.float32).to(dtype))
            else:
                t.uniform_(-1, 1)
            self.register_parameter(name.replace(".", "__"), torch.nn.Parameter(t))
            self._names.append(name)

    def named_parameters(self, *a, **k):  # the dotted names, in declaration order
        for name in self._names:
            yield name, getattr(self, name.replace(".", "__"))


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def group_census(groups: dict, device) -> dict:
    """The size every communicator of a multi-rank run reports, against the intended rank count.

    ``groups``: name -> (torch process group | comm.RcclComm | None for the default group,
    intended ranks).  Per entry: the size the communicator itself reports (``ncclCommCount`` /
    ``ncclCommUserRank`` through prl_comm for an RcclComm; ``dist.get_world_size(group)`` and the
    backend for a torch group) and the sum of an all-reduce of ones over it, i.e. the ranks that
    actually took part.  Collective over each group's members (non-members pass the group's entry
    as absent).  Raises AssertionError when any reported size or participant count differs from
    the intended one (launch.py:147-150 / world.py:184: the actor group is 1 + actor GPUs)."""
    from .comm import RcclComm

    out = {}
    for name, (group, intended) in groups.items():
        ones = torch.ones(1, dtype=torch.float32, device=device)
        if isinstance(group, RcclComm):
            entry = {"kind": "prl_comm (RCCL)", "reported": group.reported_size(), "rank": group.reported_rank()}
            group.all_reduce(ones)
        else:
            entry = {"kind": f"torch {dist.get_backend(group)}", "reported": dist.get_world_size(group),
                     "rank": dist.get_rank(group)}
            dist.all_reduce(ones, group=group)
        _sync(torch.device(device))
        entry.update(intended=int(intended), participants=int(ones.item()))
        entry["ok"] = entry["reported"] == entry["participants"] == int(intended)
        out[name] = entry
    bad = {k: v for k, v in out.items() if not v["ok"]}
    assert not bad, f"communicator sizes differ from the intended rank counts: {bad}"
    return out


def grad_allreduce_probe(shapes, device, iters: int = 5, bucket_bytes: int = 256 << 20, group=None,
                         dtype=torch.bfloat16) -> dict:
    from .finetune.grad_sync import GradBuckets

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    params = [torch.nn.Parameter(torch.empty(s, dtype=dtype, device=device)) for _, s in shapes]
    gb = GradBuckets(params, group=group, bucket_bytes=bucket_bytes, reduce="mean")
    nbytes = sum(b.flat.numel() * b.flat.element_size() for b in gb.buckets)
    times = []
    for it in range(iters + 1):
        for b in gb.buckets:
            b.flat.fill_(float(rank + 1))
        _sync(device)
        dist.barrier(group)
        t0 = time.perf_counter()
        gb.arm()
        for p in reversed(params):  # the order backward produces gradients
            gb._hook(p)
        gb.finish()
        _sync(device)
        if it:  # first iteration warms the communicator
            times.append(time.perf_counter() - t0)
    want = (world + 1) / 2.0
    ok = all(bool((b.flat.float() == want).all()) for b in gb.buckets)
    gb.remove()
    t = torch.tensor([sum(times) / len(times)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    sec = float(t)
    return {"bytes": nbytes, "buckets": len(gb.buckets), "bucket_mb": bucket_bytes >> 20, "ms": round(sec * 1e3, 3),
            "algbw_GBps": round(nbytes / sec / 1e9, 1),
            "busbw_GBps": round(nbytes * 2 * (world - 1) / world / sec / 1e9, 1), "correct": ok}


def broadcast_probe(shapes, device, iters: int = 3, bucket_bytes: int = 256 << 20, group=None,
                    packer=None, transport: str = "bucketed") -> dict:
    """Rank 0 sends with WeightUpdateManager, ranks 1.. receive with WorkerExtension."""
    from .actor import StandaloneWorker
    from .weight_update import ParameterInfo, WeightUpdateManager, WeightUpdateRequest

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    group = group or dist.group.WORLD
    infos = [ParameterInfo(name=n, shape=list(s), dtype=str(torch.bfloat16)) for n, s in shapes]
    if rank == 0:
        module = ShapedModule(shapes, device=device, seed=1)
        mgr = WeightUpdateManager([], module, None, group, transport=transport, bucket_bytes=bucket_bytes,
                                  overlap=True, packer=packer, write_message=lambda s, m: None)
    else:
        worker = StandaloneWorker(ShapedModule(shapes, device=device, fill=0.0), rank=0, device=device)
        worker.process_group = group
    times = []
    for v in range(iters + 1):
        _sync(device)
        dist.barrier(group)
        t0 = time.perf_counter()
        if rank == 0:
            mgr.send_weight_update(v)
            mgr.wait()
        else:
            worker.receive_weight_update(WeightUpdateRequest(version=v, parameters_info=infos, transport=transport,
                                                             bucket_bytes=bucket_bytes if transport == "bucketed"
                                                             else 0))
        _sync(device)
        if v:
            times.append(time.perf_counter() - t0)
    # checksum of what every rank now holds (sender's module vs each receiver's)
    src = module if rank == 0 else worker.model_runner.model.module
    cs = torch.zeros(1, dtype=torch.float64, device=device)
    for _, p in src.named_parameters():
        cs += p.detach().double().sum()
    cs_all = [torch.zeros_like(cs) for _ in range(world)]
    dist.all_gather(cs_all, cs, group=group)
    ok = all(bool(c == cs_all[0]) for c in cs_all)
    if rank == 0:
        mgr.close()
    t = torch.tensor([sum(times) / len(times)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    nbytes = sum(2 * int(torch.Size(s).numel()) for _, s in shapes)
    sec = float(t)
    return {"bytes": nbytes, "tensors": len(shapes), "receivers": world - 1, "transport": transport,
            "ms": round(sec * 1e3, 3), "GBps": round(nbytes / sec / 1e9, 1), "correct": ok}
