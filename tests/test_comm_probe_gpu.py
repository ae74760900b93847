"""The bench's exchange probes with their device-side paths (HIP flatten / unflatten staging,
GradBuckets side stream) on one MI355X: two ranks share cuda:0 over gloo, since RCCL needs one
GPU per rank; the driver's multi-GPU bench runs the same code over RCCL."""

import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu
SHAPES = [("model.embed_tokens.weight", (4096, 64)), ("model.layers.0.mlp.up_proj.weight", (333, 64)),
          ("model.layers.0.input_layernorm.weight", (64,)), ("model.norm.weight", (7,))]


def _run(rank, port, world, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    import torch.distributed as dist
    from pipelinerl_amd import comm_probe

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ar = comm_probe.grad_allreduce_probe(SHAPES, dev, iters=2, bucket_bytes=64 << 10)
    bc = comm_probe.broadcast_probe(SHAPES, dev, iters=2, bucket_bytes=100 << 10)
    torch.save({"ar": ar, "bc": bc}, Path(out) / f"r{rank}.pt")
    dist.destroy_process_group()


def test_probes_on_device(tmp_path):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), 2, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"r{r}.pt")
        assert res["ar"]["correct"] and res["ar"]["buckets"] >= 2, res
        assert res["bc"]["correct"], res
