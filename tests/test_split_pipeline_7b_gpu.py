"""BASELINE configs[3] (C4) at its own size on ONE GPU: a Qwen2.5-7B trainer rank and an actor rank
share cuda:0 over gloo (cuda tensors).  The trainer runs two optimizer steps of the product path
(patched HIP model ops, HIP attention, label-row lm_head + HIP loss head, native AdamW at lr 1e-3
so every version differs) and after each one WeightUpdateManager snapshots the 339 tensors /
15.23 GB with the HIP flatten kernel and broadcasts them (finetune_loop.py:174-256); the actor
receives them through WorkerExtension.receive_weight_update (vllm1.py:81-94) — per_tensor, then
bucketed (256 MiB buckets, HIP unflatten into its parameters).  After each transport the actor's
weights must equal the trainer's bit for bit (bf16 bit-pattern digests of every tensor), and the
request's parameters_info must follow F4's rule (named_parameters order, full shapes, bf16).
RCCL needs one GPU per rank: the driver's multi-GPU run measures that transport."""

import os
import socket
import sys
import time
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest(named) -> dict:
    """Two integer sums over each tensor's bf16 bit patterns (plain and position-weighted)."""
    out = {}
    for n, p in named:
        x = p.detach().reshape(-1).view(torch.int16)
        s0 = s1 = 0
        for a in range(0, x.numel(), 1 << 26):
            c = x[a:a + (1 << 26)].to(torch.int64)
            w = torch.arange(a, a + c.numel(), device=c.device, dtype=torch.int64) % 1000003 + 1
            s0 += int(c.sum())
            s1 += int((c * w).sum())
        out[n] = (s0, s1)
    return out


def _log(rank, msg):
    print(f"[c4-7b r{rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _run(rank, port, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist

    from pipelinerl_amd.actor import StandaloneWorker
    from pipelinerl_amd.trainer_probe import TrainerStep, qwen2_model
    from pipelinerl_amd.weight_update import WeightUpdateManager, WeightUpdateRequest, parameters_info

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    dp_group = dist.new_group([0])
    bc_group = dist.new_group([0, 1])
    report = {"transports": {}}
    if rank == 0:
        ts = TrainerStep("7b", tokens=2048, seq=1024, prompt=128, micro_batches=1, device=dev, group=dp_group)
        for grp in ts.opt.param_groups:
            grp["lr"] = 1e-3
        named = list(ts.model.named_parameters())
        infos = parameters_info(named)
        report["infos"] = [(i.name, list(i.shape), i.dtype) for i in infos]
        report["named"] = [(n, list(p.shape)) for n, p in named]
        dist.broadcast_object_list([[i.model_dump() for i in infos]], src=0, group=bc_group)
        _log(rank, f"trainer ready: {len(infos)} tensors")
        version = 0
        for transport in ("per_tensor", "bucketed"):
            wum = WeightUpdateManager([], ts.model, None, bc_group, transport=transport, bucket_bytes=256 << 20,
                                      overlap=True, write_message=lambda s, m: None)
            digests = []
            for _ in range(2):
                version += 1
                ts.step(wum=wum, version=version)  # snapshot + broadcast after the optimizer step
                wum.wait()
                torch.cuda.synchronize()
                digests.append(_digest(ts.model.named_parameters()))
                _log(rank, f"{transport}: version {version} sent ({wum.last_latency_s:.1f} s)")
            wum.close()
            report["transports"][transport] = {"digests": digests, "latency_s": wum.last_latency_s}
    else:
        holder = [None]
        dist.broadcast_object_list(holder, src=0, group=bc_group)
        from pipelinerl_amd.weight_update import ParameterInfo

        infos = [ParameterInfo(**d) for d in holder[0]]
        module = qwen2_model("7b", dev, fused_ops=False)
        worker = StandaloneWorker(module, rank=0, device=dev)
        worker.process_group = bc_group
        version = 0
        for transport in ("per_tensor", "bucketed"):
            with torch.no_grad():
                for p in module.parameters():
                    p.zero_()
            digests = []
            for _ in range(2):
                version += 1
                worker.receive_weight_update(WeightUpdateRequest(
                    version=version, parameters_info=infos, transport=transport,
                    bucket_bytes=(256 << 20) if transport == "bucketed" else 0))
                torch.cuda.synchronize()
                digests.append(_digest(module.named_parameters()))
                _log(rank, f"{transport}: version {version} received")
            report["transports"][transport] = {"digests": digests}
    torch.save(report, Path(out) / f"r{rank}.pt")
    dist.barrier(group=bc_group)
    dist.destroy_process_group()


def test_split_pipeline_7b_one_gpu(tmp_path):
    mp.spawn(_run, args=(_free_port(), str(tmp_path)), nprocs=2, join=True)
    tr, ac = (torch.load(tmp_path / f"r{r}.pt") for r in range(2))
    infos = tr["infos"]
    # F4's rule (tests/golden/f4_weight_update.json, finetune_loop.py:192-196): one entry per
    # named parameter, in named_parameters order, full shape, dtype bf16
    assert [(n, s) for n, s, _ in infos] == [tuple(x) for x in tr["named"]]
    assert all(d == str(torch.bfloat16) for _, _, d in infos)
    assert len(infos) == 339
    nbytes = sum(2 * torch.Size(s).numel() for _, s, _ in infos)
    assert abs(nbytes - 15.23e9) < 0.01e9, nbytes
    for transport in ("per_tensor", "bucketed"):
        t, a = tr["transports"][transport]["digests"], ac["transports"][transport]["digests"]
        assert len(t) == len(a) == 2
        for v in range(2):
            bad = [n for n in t[v] if t[v][n] != a[v][n]]
            assert not bad, (transport, v, bad[:5])
        # the two versions differ (the optimizer moved the weights): a stale update would be caught
        # (all but the RMSNorm weights: at 1.0 a 1e-3 step is below half a bf16 ulp)
        assert sum(t[0][n] != t[1][n] for n in t[0]) >= 339 - 57, transport
