"""Data-parallel trainer loop on CPU (gloo, world sizes 1 and 2) with the test-only torch loss.

Checks the reference protocol (finetune_loop.py:567-719): lockstep sample counts with
sentinel batches, optimizer step exactly when the global count reaches samples_per_step,
SamplesProcessed messages, checkpoint layout, and that the bucketed gradient all-reduce
keeps replicas identical and (reduce=sum) equals one rank training on all the data.
"""

import json
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, exp, steps, passes, extra):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    import torch.distributed as dist

    from cpu_rl_step import cpu_rl_step
    from loop_helpers import loop_cfg
    from pipelinerl_amd.finetune_loop import run_finetuning_loop
    from pipelinerl_amd.streams import reset_streams_backend

    reset_streams_backend()
    exp = Path(exp)
    cfg = loop_cfg(exp, exp / "tiny_qwen2", world, passes, steps, **extra)
    captured = {}

    def step(model, batch, cur, mx, config):
        captured["model"] = model
        return cpu_rl_step(model, batch, cur, mx, config)

    m = run_finetuning_loop(cfg, step_fn=step)
    torch.save({n: p.detach().clone() for n, p in captured["model"].named_parameters()},
               exp / f"params_w{world}_r{rank}.pt")
    (exp / f"metrics_w{world}_r{rank}.json").write_text(json.dumps({"steps": m.completed_steps, "samples": m.samples,
                                                                    "passes": m.passes}))
    if dist.is_initialized():
        dist.destroy_process_group()


def _setup(tmp: Path, world: int, n_groups=4, attempts=4, seq_length=28, tail_groups=0):
    """``tail_groups``: groups written after the two steps' data (never trained on) so the packer
    finishes the second step's last round of writes — with finite data the protocol's round ends
    only when more samples arrive (preprocess.py:557-626), which at 4 and 8 ranks starves the
    ranks after the last write."""
    sys.path[:0] = [str(ROOT / "tests")]
    from loop_helpers import rollouts, tiny_model_dir, write_training_data
    from pipelinerl_amd.streams import reset_streams_backend, set_streams_backend

    reset_streams_backend()
    set_streams_backend("files")
    tiny_model_dir(tmp)
    data = rollouts(n_groups + tail_groups, attempts)  # the first n_groups groups as rollouts(n_groups)
    total = n_groups * attempts
    per_step = total // 2  # two optimizer steps
    writes = write_training_data(tmp, data, world, seq_length, per_step // world)
    reset_streams_backend()
    return per_step, writes


@pytest.mark.parametrize("world", [2, 8])
def test_dp_loop_matches_single_rank(tmp_path, world):
    """The DP loop at world 2 and 8 (the driver's N = 8 scaling run has 8 ranks in lockstep:
    sample quotas, sentinels, per-pass exchange) ends with the parameters of one rank trained on
    all the data."""
    exp2 = tmp_path / f"w{world}"
    exp2.mkdir()
    ng = max(4, 2 * world)  # 4 samples per rank and optimizer step
    per_step, writes = _setup(exp2, world, n_groups=ng, tail_groups=ng)
    if world == 2:
        assert any(b.sentinel for _, b in writes), "the packing should have produced sentinel batches"
    mp.spawn(_rank_main, args=(world, free_port(), str(exp2), 2, per_step, {}), nprocs=world, join=True)
    p0 = torch.load(exp2 / f"params_w{world}_r0.pt")
    for r in range(1, world):
        pr = torch.load(exp2 / f"params_w{world}_r{r}.pt")
        for n in p0:
            assert torch.equal(p0[n], pr[n]), (r, n)  # replicas stay identical
    m0 = json.loads((exp2 / f"metrics_w{world}_r0.json").read_text())
    assert m0["steps"] == 2 and m0["samples"] == 2 * per_step
    # world-1 run on the same rollouts
    exp1 = tmp_path / "w1"
    exp1.mkdir()
    _setup(exp1, 1, n_groups=ng, tail_groups=ng)
    mp.spawn(_rank_main, args=(1, free_port(), str(exp1), 2, per_step, {}), nprocs=1, join=True)
    q = torch.load(exp1 / "params_w1_r0.pt")
    worst = max(float((p0[n] - q[n]).abs().max()) for n in q)
    assert worst < 2e-5, worst
    # protocol outputs
    msgs = [json.loads(x) for x in (exp2 / "streams" / "weight_update_request" / "0" / "0" / "0.jsonl").read_text()
            .splitlines()]
    counts = [m["samples_processed"] for m in msgs if m["kind"] == "samples_processed"]
    assert counts[0] == 0 and counts == sorted(counts) and counts[-1] == 2 * per_step
    fin = exp2 / "finetune"
    assert (fin / "current" / "config.json").exists() and (fin / "training_state" / "training_state.pt").exists()
    summary = json.loads((fin / "summary.json").read_text())
    assert summary["completed_steps"] == 2 and summary["samples"] == 2 * per_step
    lines = [json.loads(x) for x in (fin / "logs" / "metrics.jsonl").read_text().splitlines()]
    assert {"rl/ess", "throughput/tokens_per_sec", "stats/grad_norm", "rl/loss"} <= set(lines[-1])


def test_resume_from_training_state(tmp_path):
    exp = tmp_path / "r"
    exp.mkdir()
    per_step, _ = _setup(exp, 1)
    mp.spawn(_rank_main, args=(1, free_port(), str(exp), 1, per_step, {}), nprocs=1, join=True)
    m = json.loads((exp / "metrics_w1_r0.json").read_text())
    assert m["steps"] == 1
    state = torch.load(exp / "finetune" / "training_state" / "training_state.pt", weights_only=True)
    assert state["completed_steps"] == 1 and "optimizer_state" in state


def _grad_capture_main(rank, world, port, exp, steps, passes, extra):
    """_rank_main with torch.nn.utils.clip_grad_norm_ wrapped to record the gradients just
    before and just after clipping at every optimizer step."""
    import torch.nn.utils as nnu

    orig = nnu.clip_grad_norm_
    rec = []

    def clip(params, max_norm, *a, **k):
        params = list(params)
        before = torch.cat([p.grad.detach().reshape(-1).clone() for p in params if p.grad is not None])
        n = orig(params, max_norm, *a, **k)
        after = torch.cat([p.grad.detach().reshape(-1).clone() for p in params if p.grad is not None])
        rec.append({"before": before, "after": after, "norm": float(n)})
        return n

    nnu.clip_grad_norm_ = clip
    try:
        _rank_main(rank, world, port, exp, steps, passes, extra)
    finally:
        nnu.clip_grad_norm_ = orig
    torch.save(rec, Path(exp) / f"grads_r{rank}.pt")


def test_deepspeed_grad_scale_convention(tmp_path):
    """finetune.grad_scale: deepspeed divides every micro-batch loss by GAS =
    seq_parallel * gradient_accumulation_passes / world (DeepSpeed's engine.backward with the
    gradient_accumulation_steps the reference injects, finetune_loop.py:306-312); accelerate
    (GAS 1) sums them.  The gradient the clip sees — and so the clip decision at 0.3 — differs
    by exactly 1/GAS; after clipping both are the clipped form of their own gradient."""
    world = 2
    runs = {}
    for mode in ("accelerate", "deepspeed"):
        exp = tmp_path / mode
        exp.mkdir()
        per_step, _ = _setup(exp, world)
        # (master_weights off: the capture wraps torch's clip_grad_norm_, which PrlAdamW's fp32 norm skips)
        extra = {"grad_scale": mode, "master_weights": False}
        mp.spawn(_grad_capture_main, args=(world, free_port(), str(exp), 1, per_step, extra),
                 nprocs=world, join=True)
        runs[mode] = torch.load(exp / "grads_r0.pt")
    gas = per_step // world
    assert gas > 1
    acc, ds = runs["accelerate"][0], runs["deepspeed"][0]
    rel = float((ds["before"] * gas - acc["before"]).abs().max() / acc["before"].abs().max())
    assert rel < 1e-5, rel
    assert abs(ds["norm"] * gas - acc["norm"]) <= 1e-5 * acc["norm"]
    for r in (acc, ds):
        want = r["before"] * min(1.0, 0.3 / (r["norm"] + 1e-6))
        assert torch.allclose(r["after"], want, rtol=1e-5, atol=1e-9)


def test_grad_scale_convention_follows_the_backend():
    from pipelinerl_amd.config import Cfg
    from pipelinerl_amd.finetune_loop import grad_scale_convention, micro_batch_loss_scale

    assert grad_scale_convention(Cfg.wrap({"finetune": {}})) == "accelerate"
    assert grad_scale_convention(Cfg.wrap({"use_deepspeed": True, "finetune": {}})) == "deepspeed"
    assert grad_scale_convention(Cfg.wrap({"use_deepspeed": True, "use_fsdp": True, "finetune": {}})) == "accelerate"
    assert grad_scale_convention(Cfg.wrap({"use_deepspeed": True, "finetune": {"grad_scale": "accelerate"}})) \
        == "accelerate"
    with pytest.raises(ValueError):
        grad_scale_convention(Cfg.wrap({"finetune": {"grad_scale": "zero3"}}))
    args = Cfg.wrap({"seq_parallel": 1, "gradient_accumulation_passes": 1024})
    assert micro_batch_loss_scale(args, 4, "deepspeed") == 1 / 256
    assert micro_batch_loss_scale(args, 4, "accelerate") == 1.0


def test_launch_without_deepspeed_warns_about_the_grad_scale(caplog):
    """The reference config (conf/base.yaml:94-95: use_deepspeed true, deepspeed_config named)
    launched with the documented use_deepspeed=false (launch.py:272-277 then drops --use_deepspeed):
    one WARNING that the default gradient convention changed, naming the override; both explicit
    conventions resolve silently, and a config without deepspeed_config does not warn."""
    import logging

    from pipelinerl_amd.config import Cfg
    from pipelinerl_amd.finetune_loop import grad_scale_convention

    ref_default = {"use_deepspeed": False, "deepspeed_config": "deepspeed_stage3_bf16", "finetune": {}}
    with caplog.at_level(logging.WARNING, logger="pipelinerl_amd.finetune_loop"):
        assert grad_scale_convention(Cfg.wrap(ref_default)) == "accelerate"
    warns = [r for r in caplog.records if r.levelno == logging.WARNING]
    assert len(warns) == 1 and "finetune.grad_scale=deepspeed" in warns[0].getMessage()
    for mode in ("deepspeed", "accelerate"):
        caplog.clear()
        with caplog.at_level(logging.WARNING, logger="pipelinerl_amd.finetune_loop"):
            cfg = dict(ref_default, finetune={"grad_scale": mode})
            assert grad_scale_convention(Cfg.wrap(cfg)) == mode
        assert not caplog.records
    caplog.clear()
    with caplog.at_level(logging.WARNING, logger="pipelinerl_amd.finetune_loop"):
        assert grad_scale_convention(Cfg.wrap({"use_deepspeed": False, "finetune": {}})) == "accelerate"
        assert grad_scale_convention(Cfg.wrap({"use_deepspeed": True, "deepspeed_config": "x", "finetune": {}})) \
            == "deepspeed"
    assert not caplog.records


def test_phase_trace_metrics(tmp_path):
    """finetune.trace_gpu_phases: per-step trace/<phase>_ms for forward, backward, all-reduce wait,
    clip and optimizer (summed over the step's micro-batches) and trace/gpu_step_ms in the logged
    metrics (wall-clock marks on a CPU device, HIP events on a GPU); the phases add up to the step."""
    exp = tmp_path / "t"
    exp.mkdir()
    per_step, _ = _setup(exp, 1)
    mp.spawn(_rank_main, args=(1, free_port(), str(exp), 1, per_step, {"trace_gpu_phases": True}), nprocs=1, join=True)
    lines = [json.loads(x) for x in (exp / "finetune" / "logs" / "metrics.jsonl").read_text().splitlines()]
    keys = {f"trace/{p}_ms" for p in ("forward", "backward", "allreduce_wait", "clip", "optimizer")}
    assert keys | {"trace/gpu_step_ms"} <= set(lines[-1])
    parts = sum(lines[-1][k] for k in keys)
    assert lines[-1]["trace/forward_ms"] > 0 and lines[-1]["trace/backward_ms"] > 0
    assert parts <= lines[-1]["trace/gpu_step_ms"] + 1e-6


def test_phase_trace_unit():
    from pipelinerl_amd.finetune.trace import PhaseTrace

    t = PhaseTrace(torch.device("cpu"))
    t.start()
    for _ in range(3):
        t.mark("forward")
        t.mark("backward")
    t.mark("optimizer")
    out = t.collect()
    assert set(out) == {"trace/forward_ms", "trace/backward_ms", "trace/optimizer_ms", "trace/gpu_step_ms"}
    assert abs(sum(v for k, v in out.items() if k != "trace/gpu_step_ms") - out["trace/gpu_step_ms"]) < 1e-6
    assert t.collect() == {}  # collect() resets
    off = PhaseTrace(torch.device("cpu"), enabled=False)
    off.start()
    off.mark("forward")
    assert off.collect() == {}


def test_freeze_setup_heap(monkeypatch):
    """hostgc.freeze_setup_heap moves the set-up heap to the permanent generation (no
    generation-2 walk over it mid-step); PRL_GC_FREEZE=0 leaves the collector alone; objects made
    after the freeze are still collected."""
    import gc

    from pipelinerl_amd.hostgc import freeze_setup_heap

    try:
        monkeypatch.setenv("PRL_GC_FREEZE", "0")
        gc.unfreeze()
        assert not freeze_setup_heap() and gc.get_freeze_count() == 0
        monkeypatch.setenv("PRL_GC_FREEZE", "1")
        assert freeze_setup_heap() and gc.get_freeze_count() > 1000
        a, b = [], []
        a.append(b)
        b.append(a)  # a reference cycle made after the freeze
        del a, b
        assert gc.collect() >= 2
    finally:
        gc.unfreeze()


def test_prl_adamw_cpu_falls_back_to_torch():
    """PrlAdamW on CPU parameters takes torch's fused step, with clip_grad_norm's deferred
    multiply applied first: identical to clip_grad_norm_ + torch.optim.AdamW(fused=True)."""
    from pipelinerl_amd.finetune.optim import PrlAdamW, clip_grad_norm

    g = torch.Generator().manual_seed(0)
    pa = [torch.nn.Parameter(torch.randn(s, generator=g)) for s in ((5, 7), (11,))]
    pb = [torch.nn.Parameter(p.detach().clone()) for p in pa]
    ref = torch.optim.AdamW(pa, lr=1e-2, fused=True)
    opt = PrlAdamW(pb, lr=1e-2)
    for step in range(3):
        grads = [torch.randn(p.shape, generator=g) * 5 for p in pa]
        for p, q, gr in zip(pa, pb, grads):
            p.grad, q.grad = gr.clone(), gr.clone()
        na = torch.nn.utils.clip_grad_norm_(pa, 0.3)
        nb = clip_grad_norm(pb, 0.3, opt)
        assert torch.equal(na, nb)
        ref.step()
        opt.step()
    for p, q in zip(pa, pb):
        assert torch.equal(p, q)
    assert isinstance(clip_grad_norm(pa, 1.0, ref), torch.Tensor)  # any other optimizer: torch's clip


def test_resume_refuses_a_deepspeed_training_state(tmp_path, monkeypatch):
    """The reference resumes whenever finetune/training_state/ exists (finetune_loop.py:416-418),
    including DeepSpeed's tag layout (finetune/checkpoints.py:169-180: <dir>/deepspeed/ + latest).
    This trainer cannot read ZeRO shards, so it raises instead of restarting at samples=0."""
    sys.path[:0] = [str(ROOT / "tests")]
    from cpu_rl_step import cpu_rl_step
    from loop_helpers import loop_cfg
    from pipelinerl_amd.finetune_loop import TrainingStateError, check_training_state_layout, run_finetuning_loop
    from pipelinerl_amd.streams import reset_streams_backend

    exp = tmp_path / "ds"
    exp.mkdir()
    per_step, _ = _setup(exp, 1)
    state = exp / "finetune" / "training_state"
    (state / "deepspeed").mkdir(parents=True)
    (state / "latest").write_text("deepspeed")
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    reset_streams_backend()
    cfg = loop_cfg(exp, exp / "tiny_qwen2", 1, per_step, 1, dist_backend=None)
    with pytest.raises(TrainingStateError, match="DeepSpeed"):
        run_finetuning_loop(cfg, step_fn=cpu_rl_step)
    # an empty training_state/ fails too (the reference's torch.load of training_state.pt would)
    empty = tmp_path / "empty_state"
    empty.mkdir()
    with pytest.raises(TrainingStateError, match="no training_state.pt"):
        check_training_state_layout(empty)
    (empty / "training_state.pt").write_bytes(b"")
    check_training_state_layout(empty)  # the layout this trainer writes: accepted
