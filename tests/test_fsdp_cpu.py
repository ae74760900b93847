"""FSDP trainer path (finetune/sharding.py) on CPU with gloo, world size 2.

  * the sharded loop (use_fsdp, grad_reduce=sum) ends with the same parameters as one
    unsharded rank trained on all the data, and writes full HF weights + a sharded optimizer
    checkpoint that resumes;
  * the weight snapshot of a sharded model (every trainer rank joins the all-gathers, rank 0
    broadcasts on the "actor" group) reaches an actor bit-exactly.
"""

import json
import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _loop_rank(rank, world, port, exp, steps, passes, extra):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from torch.distributed.tensor import DTensor

    from cpu_rl_step import cpu_rl_step
    from loop_helpers import loop_cfg
    from pipelinerl_amd.finetune_loop import run_finetuning_loop
    from pipelinerl_amd.streams import reset_streams_backend

    reset_streams_backend()
    exp = Path(exp)
    cfg = loop_cfg(exp, exp / "tiny_qwen2", world, passes, steps, **extra)
    captured = {}

    def step(model, batch, cur, mx, config):
        if "model" not in captured:
            from pipelinerl_amd.finetune.sharding import decoder_layers

            def at_final_norm(mod, inp):  # every decoder layer's forward is done, no backward yet
                captured["unsharded_at_norm"] = [not any(isinstance(p, DTensor) for p in layer.parameters())
                                                 for layer in decoder_layers(model)]

            norm = next(m for n, m in model.named_modules() if n.endswith("model.norm"))
            norm.register_forward_pre_hook(at_final_norm)
        captured["model"] = model
        return cpu_rl_step(model, batch, cur, mx, config)

    m = run_finetuning_loop(cfg, step_fn=step)
    full = {n: (p.full_tensor() if isinstance(p, DTensor) else p).detach().clone()
            for n, p in captured["model"].named_parameters()}
    torch.save(full, exp / f"params_w{world}_r{rank}.pt")
    from pipelinerl_amd.finetune.sharding import decoder_layers

    flags = [bool(getattr(layer, "gradient_checkpointing", False)) for layer in decoder_layers(captured["model"])]
    (exp / f"metrics_w{world}_r{rank}.json").write_text(json.dumps({
        "steps": m.completed_steps, "samples": m.samples, "ckpt_flags": flags,
        "unsharded_at_norm": captured.get("unsharded_at_norm")}))
    if dist.is_initialized():
        dist.destroy_process_group()


def _setup(tmp: Path, world: int):
    sys.path[:0] = [str(ROOT / "tests")]
    from test_finetune_loop_cpu import _setup as dp_setup

    return dp_setup(tmp, world)


def test_fsdp_loop_matches_single_rank_and_resumes(tmp_path):
    from test_finetune_loop_cpu import _rank_main, free_port

    exp2 = tmp_path / "fsdp"
    exp2.mkdir()
    per_step, _ = _setup(exp2, 2)
    mp.spawn(_loop_rank, args=(2, free_port(), str(exp2), 2, per_step, {"sharding": "fsdp"}), nprocs=2, join=True)
    p0 = torch.load(exp2 / "params_w2_r0.pt")
    p1 = torch.load(exp2 / "params_w2_r1.pt")
    for n in p0:
        assert torch.equal(p0[n], p1[n]), n
    exp1 = tmp_path / "single"
    exp1.mkdir()
    _setup(exp1, 1)
    mp.spawn(_rank_main, args=(1, free_port(), str(exp1), 2, per_step, {}), nprocs=1, join=True)
    q = torch.load(exp1 / "params_w1_r0.pt")
    assert set(q) == set(p0)
    worst = max(float((p0[n] - q[n]).abs().max()) for n in q)
    assert worst < 2e-5, worst
    # full HF weights written by rank 0 from the gathered state dict
    from safetensors.torch import load_file

    saved = load_file(str(exp2 / "finetune" / "current" / "model.safetensors"))
    for n, t in saved.items():
        assert torch.equal(t, p0[n]), n
    assert (exp2 / "finetune" / "training_state" / "optim").is_dir()
    # resume: one more step from the sharded training state
    mp.spawn(_loop_rank, args=(2, free_port(), str(exp2), 3, per_step, {"sharding": "fsdp"}), nprocs=2, join=True)
    m = json.loads((exp2 / "metrics_w2_r0.json").read_text())
    assert m["steps"] == 3


def _bcast_rank(rank, port_default, port_actor, exp, value_head=False):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from loop_helpers import tiny_model_dir
    from test_weight_update_cpu import TorchFlatPacker
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd import torch_utils
    from pipelinerl_amd.weight_update import ParameterInfo, WeightUpdateManager, WeightUpdateRequest

    exp = Path(exp)
    torch.manual_seed(0)
    model = AutoModelForCausalLM.from_config(AutoConfig.from_pretrained(tiny_model_dir(exp)))
    names = [(n, list(p.shape)) for n, p in model.named_parameters()]
    if rank < 2:  # the two trainer ranks
        from pipelinerl_amd.finetune.sharding import shard_model

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port_default}", rank=rank, world_size=2)
        lm = model
        if value_head:  # the root FSDP unit is the wrapper: it holds the LM's embedding / norm / lm_head
            from pipelinerl_amd.finetune.value_model import AutoModelForCausalLMWithValueHead

            model = AutoModelForCausalLMWithValueHead(model)
        shard_model(model)
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
        pg = None
        if rank == 0:
            pg = torch_utils.init_extra_process_group(group_name="actor", backend="gloo",
                                                      init_method=f"tcp://127.0.0.1:{port_actor}", rank=0,
                                                      world_size=2)
        mgr = WeightUpdateManager([], model, None, pg, transport="bucketed", bucket_bytes=4096, overlap=True,
                                  packer=TorchFlatPacker(), is_main=rank == 0, write_message=lambda s, m: None)
        mgr.send_weight_update(5)
        mgr.close()
        from torch.distributed.tensor import DTensor

        full = {n: p.full_tensor().detach().clone() if isinstance(p, DTensor) else p.detach().clone()
                for n, p in lm.named_parameters()}
        if rank == 0:
            torch.save(full, exp / "trainer.pt")
        dist.destroy_process_group()
    else:
        from pipelinerl_amd.actor import StandaloneWorker

        worker = StandaloneWorker(model.to(torch.bfloat16), rank=0, device="cpu", backend="gloo")
        worker.init_actor_update_group(0, 1, f"tcp://127.0.0.1:{port_actor}", 2)
        infos = [ParameterInfo(name=n, shape=s, dtype=str(torch.bfloat16)) for n, s in names]
        worker.receive_weight_update(WeightUpdateRequest(version=5, parameters_info=infos, transport="bucketed",
                                                         bucket_bytes=4096))
        torch.save({n: p.detach().clone() for n, p in worker.model_runner.model.params.items()}, exp / "actor.pt")


@pytest.mark.parametrize("value_head", [False, True], ids=["lm", "value_head"])
def test_sharded_weight_snapshot_reaches_actor(tmp_path, value_head):
    """With a value-head wrapper (reference conf/finetune/ppo.yaml) the wrapper is the FSDP root:
    the snapshot gathers its units, maps them into the LM's names and leaves the value head out."""
    from test_weight_update_cpu import free_port

    mp.spawn(_bcast_rank, args=(free_port(), free_port(), str(tmp_path), value_head), nprocs=3, join=True)
    want = torch.load(tmp_path / "trainer.pt")
    got = torch.load(tmp_path / "actor.pt")
    assert set(got) == set(want)
    for n in want:
        assert torch.equal(got[n], want[n].to(torch.bfloat16)), n


def test_fsdp_loop_with_partial_recompute_matches(tmp_path):
    """gradient_checkpointing with the last 1 of 2 decoder layers keeping its activations
    (finetune.gradient_checkpointing_keep_layers, checkpoints.keep_activations) under the FSDP2
    loop: the same parameters as the FSDP loop without checkpointing."""
    from test_finetune_loop_cpu import free_port

    runs = {}
    for name, extra in (("plain", {"sharding": "fsdp"}),
                        ("ckpt", {"sharding": "fsdp", "gradient_checkpointing": True,
                                  "gradient_checkpointing_keep_layers": 1})):
        exp = tmp_path / name
        exp.mkdir()
        per_step, _ = _setup(exp, 2)
        mp.spawn(_loop_rank, args=(2, free_port(), str(exp), 2, per_step, extra), nprocs=2, join=True)
        runs[name] = torch.load(exp / "params_w2_r0.pt")
        flags = json.loads((exp / "metrics_w2_r0.json").read_text())["ckpt_flags"]
        assert flags == ([False, False] if name == "plain" else [True, False]), (name, flags)
    worst = max(float((runs["plain"][n] - runs["ckpt"][n]).abs().max()) for n in runs["plain"])
    assert worst < 2e-6, worst


def test_fsdp_loop_keeps_planned_layers_gathered(tmp_path):
    """finetune.fsdp_keep_gathered_layers (finetune/recompute.py plan_fsdp_gathering -> shard_model):
    the last decoder layer keeps its unsharded parameters from its forward to its backward (seen
    from a hook at the final norm: every forward done, no backward yet), the first one is resharded
    as FSDP2 does by default; the parameters after two steps are bit-identical to the default wrap
    (the same all-gathered values feed the same computation)."""
    from test_finetune_loop_cpu import free_port

    runs = {}
    for name, extra in (("plain", {"sharding": "fsdp"}),
                        ("gathered", {"sharding": "fsdp", "fsdp_keep_gathered_layers": 1})):
        exp = tmp_path / name
        exp.mkdir()
        per_step, _ = _setup(exp, 2)
        mp.spawn(_loop_rank, args=(2, free_port(), str(exp), 2, per_step, extra), nprocs=2, join=True)
        runs[name] = torch.load(exp / "params_w2_r0.pt")
        seen = json.loads((exp / "metrics_w2_r0.json").read_text())["unsharded_at_norm"]
        assert seen == ([False, False] if name == "plain" else [False, True]), (name, seen)
    for n in runs["plain"]:
        assert torch.equal(runs["plain"][n], runs["gathered"][n]), n


def _toggle_rank(rank, port, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from torch.distributed.tensor import DTensor
    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd.finetune.sharding import decoder_layers, set_kept_gathered, shard_model

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    torch.manual_seed(0)
    cfg = Qwen2Config(vocab_size=64, hidden_size=32, intermediate_size=64, num_hidden_layers=4,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
    model = shard_model(AutoModelForCausalLM.from_config(cfg, dtype=torch.float32))
    seen = []
    model.model.norm.register_forward_pre_hook(lambda m, a: seen.append(
        [not any(isinstance(p, DTensor) for p in layer.parameters()) for layer in decoder_layers(model)]))
    ids = torch.randint(0, 64, (1, 12), generator=torch.Generator().manual_seed(rank))
    res = []
    for keep in (0, 2, 4, 0):
        res.append(set_kept_gathered(model, keep))
        model(input_ids=ids, labels=ids).loss.backward()
    if rank == 0:
        Path(out).write_text(json.dumps({"returned": res, "seen": seen}))
    dist.destroy_process_group()


def test_set_kept_gathered_toggles_at_run_time(tmp_path):
    """sharding.set_kept_gathered on an already sharded model (the bench's fsdp_32b A/B): the last
    ``keep`` layers hold their unsharded parameters at the final norm, the rest are resharded."""
    from test_weight_update_cpu import free_port

    out = tmp_path / "seen.json"
    mp.spawn(_toggle_rank, args=(free_port(), str(out)), nprocs=2, join=True)
    r = json.loads(out.read_text())
    assert r["returned"] == [0, 2, 4, 0]
    F, T = False, True
    assert r["seen"] == [[F, F, F, F], [F, F, T, T], [T, T, T, T], [F, F, F, F]], r["seen"]
