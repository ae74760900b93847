"""Where the trainer's collectives run (torch_utils.collective_options, finetune_loop.Dist,
grad_sync.GradBuckets, weight_update.side_stream_priority): RCCL groups are created with
high-priority streams so their kernels get hardware queues of their own instead of sharing the
compute stream's (measured on MI355X: tools/queue_probe.py, profiles/r06_queue_probe.json)."""

import json
from pathlib import Path

import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]


def test_collective_options_are_high_priority_for_rccl_only():
    from pipelinerl_amd.torch_utils import collective_options

    o = collective_options("nccl")
    assert o is not None and o.is_high_priority_stream
    assert collective_options("nccl", high_priority=False) is None
    assert collective_options("gloo") is None and collective_options(None) is None
    assert collective_options("cpu:gloo,cuda:nccl").is_high_priority_stream


def test_dp_group_is_created_with_the_options(monkeypatch):
    from pipelinerl_amd import finetune_loop

    calls = []
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    monkeypatch.setattr(dist, "init_process_group", lambda be, **kw: calls.append((be, kw)))
    d = finetune_loop.Dist("nccl")
    (be, kw), = calls
    assert be == "nccl" and kw["pg_options"].is_high_priority_stream and d.pg_options is kw["pg_options"]
    calls.clear()
    finetune_loop.Dist("nccl", high_priority_collectives=False)
    assert calls[0][1]["pg_options"] is None
    calls.clear()
    finetune_loop.Dist("gloo")
    assert calls[0][1]["pg_options"] is None


def test_weight_update_side_stream_is_high_priority_by_default(monkeypatch):
    from pipelinerl_amd.weight_update import side_stream_priority

    monkeypatch.delenv("PRL_WU_STREAM_PRIORITY", raising=False)
    assert side_stream_priority() == -1
    monkeypatch.setenv("PRL_WU_STREAM_PRIORITY", "normal")
    assert side_stream_priority() == 0


def test_host_collectives_keep_normal_priority_streams(monkeypatch):
    """A gloo group reduces / broadcasts from host copies: its side streams stay normal priority
    (several ranks sharing one GPU over gloo, each holding high-priority queues, stalled the 4-rank
    rehearsal's trainer-step probe); an RCCL group (or none named) gets high priority."""
    import os

    import torch.distributed as dist

    from pipelinerl_amd.weight_update import side_stream_priority

    monkeypatch.delenv("PRL_WU_STREAM_PRIORITY", raising=False)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        assert side_stream_priority(dist.group.WORLD) == 0
        assert side_stream_priority(None) == -1
        from pipelinerl_amd.comm import RcclComm

        assert side_stream_priority(RcclComm(None, 0, 1, None)) == -1
    finally:
        dist.destroy_process_group()


def test_queue_probe_record_shows_collectives_off_the_compute_queue():
    """The committed rocprofv3 evidence: no collective-carrying stream shares the compute queue,
    while a normal-priority pool stream does (the hazard the options remove)."""
    rec = json.loads((ROOT / "profiles" / "r06_queue_probe.json").read_text())
    assert rec["collective_streams_off_compute_queue"] is True
    for role in ("grad_buckets", "dp_collective", "actor_collective", "wu_side", "rccl"):
        assert rec["shares_compute_queue"][role] is False, role
    assert rec["run"]["gpu_max_hw_queues"] == "4"
