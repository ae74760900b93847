"""The bench's exchange-step probes (comm_probe.py) on a world-size-2 gloo group on CPU:
the DP gradient all-reduce through GradBuckets and the trainer -> actor weight broadcast
through WeightUpdateManager / WorkerExtension, each verifying its own result; the communicator
census (every group reports, and carries, the intended number of ranks; a wrong size fails)."""

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
SHAPES = [("model.embed_tokens.weight", (64, 16)), ("model.layers.0.mlp.up_proj.weight", (40, 16)),
          ("model.layers.0.input_layernorm.weight", (16,)), ("model.norm.weight", (16,))]


def _run(rank, port, world, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from pipelinerl_amd import comm_probe
    from test_weight_update_cpu import TorchFlatPacker

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cpu")
    ar = comm_probe.grad_allreduce_probe(SHAPES, dev, iters=2, bucket_bytes=2048)
    bc = comm_probe.broadcast_probe(SHAPES, dev, iters=2, bucket_bytes=1000, packer=TorchFlatPacker())
    pt = comm_probe.broadcast_probe(SHAPES, dev, iters=1, packer=TorchFlatPacker(), transport="per_tensor")
    ctrl = dist.new_group(backend="gloo")
    sub = dist.new_group([0, world - 1])
    groups = {"dp": (None, world), "ctrl": (ctrl, world)}
    if rank in (0, world - 1):
        groups["actor"] = (sub, 2)
    census = comm_probe.group_census(groups, dev)
    try:  # a group that is not the size it should be fails the census on every member
        comm_probe.group_census({"dp": (None, world + 1)}, dev)
        wrong = None
    except AssertionError as e:
        wrong = str(e)
    torch.save({"ar": ar, "bc": bc, "pt": pt, "census": census, "wrong": wrong}, Path(out) / f"r{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_probes_gloo(tmp_path, world):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), world, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt")
        assert res["ar"]["correct"] and res["ar"]["buckets"] >= 2
        assert res["bc"]["correct"] and res["pt"]["correct"]
        assert res["bc"]["receivers"] == world - 1
        assert res["ar"]["bytes"] == sum(2 * torch.Size(s).numel() for _, s in SHAPES)
        c = res["census"]
        assert set(c) == ({"dp", "ctrl", "actor"} if r in (0, world - 1) else {"dp", "ctrl"})
        for name, e in c.items():
            assert e["ok"] and e["reported"] == e["participants"] == e["intended"], (name, e)
            assert e["kind"] == "torch gloo"
        assert c["dp"]["intended"] == world and ("actor" not in c or c["actor"]["reported"] == 2)
        assert res["wrong"] and "intended" in res["wrong"]


def test_qwen2_shapes_match_survey():
    sys.path[:0] = [str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd.comm_probe import qwen2_param_shapes

    for name, n, params in (("0.5b", 290, 0.494e9), ("1.5b", 338, 1.544e9), ("7b", 339, 7.616e9),
                            ("32b", 771, 32.764e9)):
        s = qwen2_param_shapes(name)
        assert len(s) == n
        assert abs(sum(torch.Size(x).numel() for _, x in s) - params) < 1e-3 * params
