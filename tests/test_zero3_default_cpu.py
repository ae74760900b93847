"""The reference's default backend, DeepSpeed bf16 ZeRO-3 (conf/base.yaml:94-96: use_deepspeed true,
deepspeed_config deepspeed_stage3_bf16), under the build (finetune/sharding.py sharding_mode /
decide_sharding, finetune/optim.py master_weights_requested).

  * the layout decision on the reference's own default exp_config at the published Qwen2.5 shapes
    (meta device, a 288 GB MI355X): 32B selects FSDP (its model state, 524 GB with fp32 masters,
    cannot be replicated), 7B keeps replicas (its 122 GB state fits beside the activations);
    ``finetune.sharding`` overrides both ways; stage names and plain DDP map as documented;
  * a gloo world-2 loop under the default config — the auto layout (replicas on CPU) and the
    ZeRO-3 layout forced (FSDP2 with fp32 master shards) — ends with the parameters of one rank
    trained on all the data, bf16 weights loaded as the reference loads them, fp32 masters."""

import json
import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
GB = 10 ** 9
DEFAULT_TOP = {"use_deepspeed": True, "deepspeed_config": "deepspeed_stage3_bf16", "use_fsdp": False}


def _meta(name):
    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd.trainer_probe import QWEN

    with torch.device("meta"):
        return AutoModelForCausalLM.from_config(Qwen2Config(**QWEN[name]), dtype=torch.bfloat16)


def test_reference_default_config_selects_the_layout():
    from pipelinerl_amd.config import load_config
    from pipelinerl_amd.finetune.optim import master_weights_requested
    from pipelinerl_amd.finetune.sharding import decide_sharding, sharding_mode, zero_stage

    cfg = load_config(ROOT / "tests" / "golden", "exp_config_math_grpo")
    args = cfg.finetune
    assert zero_stage(cfg) == 3 and sharding_mode(cfg, args) == "auto" and master_weights_requested(cfg)
    cuda = torch.device("cuda")
    shard, why = decide_sharding(cfg, args, _meta("32b"), cuda, 4, True, device_bytes=288 * GB)
    assert shard and "ZeRO-3" in why and "FSDP" in why, why
    shard, why = decide_sharding(cfg, args, _meta("7b"), cuda, 4, True, device_bytes=288 * GB)
    assert not shard and "fits" in why, why
    # overrides, one rank, and the other backends
    args_f = dict(args, sharding="fsdp")
    assert decide_sharding(cfg, args_f, _meta("7b"), cuda, 4, True, device_bytes=288 * GB)[0]
    args_n = dict(args, sharding="none")
    assert not decide_sharding(cfg, args_n, _meta("32b"), cuda, 4, True, device_bytes=288 * GB)[0]
    assert not decide_sharding(cfg, args, _meta("7b"), cuda, 1, True, device_bytes=288 * GB)[0]
    assert decide_sharding(cfg, args_f, _meta("7b"), cuda, 1, True, device_bytes=288 * GB)[0]  # asked for
    with pytest.raises(ValueError):
        sharding_mode(cfg, dict(args, sharding="zero3"))


@pytest.mark.parametrize("top,stage,mode", [
    ({"use_deepspeed": True, "deepspeed_config": "deepspeed_stage3_bf16"}, 3, "auto"),
    ({"use_deepspeed": True, "deepspeed_config": "deepspeed_stage3_bf16_group4"}, 3, "auto"),
    ({"use_deepspeed": True, "deepspeed_config": "deepspeed_stage2_bf16"}, 2, "auto"),
    ({"use_deepspeed": True, "deepspeed_config": "deepspeed_stage1"}, 1, "auto"),
    ({"use_deepspeed": False, "use_fsdp": True}, None, "fsdp"),
    ({"use_deepspeed": False, "use_fsdp": False}, None, "none"),
])
def test_backend_to_layout(top, stage, mode):
    from pipelinerl_amd.config import Cfg
    from pipelinerl_amd.finetune.sharding import sharding_mode, zero_stage

    cfg = Cfg.wrap({**top, "finetune": {}})
    assert zero_stage(cfg) == stage
    assert sharding_mode(cfg, cfg.finetune) == mode


def test_zero_stage_read_from_a_json_file(tmp_path):
    from pipelinerl_amd.config import Cfg
    from pipelinerl_amd.finetune.sharding import zero_stage

    f = tmp_path / "custom.json"
    f.write_text(json.dumps({"zero_optimization": {"stage": 2}}))
    assert zero_stage(Cfg.wrap({"use_deepspeed": True, "deepspeed_config": str(f)})) == 2


def _rank(rank, world, port, exp, steps, passes, finetune, top):
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
    cfg = loop_cfg(exp, exp / "tiny_qwen2", world, passes, steps, **finetune)
    cfg.update(top)
    captured = {}

    def step(model, batch, cur, mx, config):
        if "init" not in captured:  # before the first optimizer step
            captured["init"] = {n: (p.full_tensor() if isinstance(p, DTensor) else p).detach().float().clone()
                                for n, p in model.named_parameters()}
        captured["model"] = model
        return cpu_rl_step(model, batch, cur, mx, config)

    m = run_finetuning_loop(cfg, step_fn=step)
    model = captured["model"]
    torch.save(captured["init"], exp / f"init_w{world}_r{rank}.pt")
    full = {n: (p.full_tensor() if isinstance(p, DTensor) else p).detach().clone() for n, p in model.named_parameters()}
    dtypes = sorted({str(p.dtype) for p in model.parameters()})
    torch.save(full, exp / f"params_w{world}_r{rank}.pt")
    (exp / f"info_w{world}_r{rank}.json").write_text(json.dumps({
        "steps": m.completed_steps, "sharded": any(isinstance(p, DTensor) for p in model.parameters()),
        "dtypes": dtypes}))
    if dist.is_initialized():
        dist.destroy_process_group()


def test_default_config_loop_world2_equals_one_rank(tmp_path):
    from test_finetune_loop_cpu import _setup, free_port

    # the reference default: bf16 weights loaded (load_as_bf16), DeepSpeed's mean over ranks and
    # 1/GAS loss scale (finetune.grad_scale follows use_deepspeed), fp32 masters (auto)
    ft = {"load_as_bf16": True, "grad_reduce": "mean"}
    runs = {}
    for name, world, extra in (("one", 1, {}), ("auto", 2, {}), ("zero3", 2, {"sharding": "fsdp"})):
        exp = tmp_path / name
        exp.mkdir()
        ng = 4
        per_step, _ = _setup(exp, world, n_groups=ng, tail_groups=ng)
        mp.spawn(_rank, args=(world, free_port(), str(exp), 2, per_step, {**ft, **extra}, DEFAULT_TOP), nprocs=world,
                 join=True)
        runs[name] = (torch.load(exp / f"params_w{world}_r0.pt"), json.loads((exp / f"info_w{world}_r0.json").read_text()),
                      torch.load(exp / f"init_w{world}_r0.pt"))
        if world == 2:
            p1 = torch.load(exp / "params_w2_r1.pt")
            for n, t in runs[name][0].items():
                assert torch.equal(t, p1[n]), (name, n)  # ranks agree
        # the default config's checkpoint keeps the loaded dtype (DeepSpeed's 16-bit gather on save)
        from safetensors.torch import load_file

        saved = load_file(str(exp / "finetune" / "current" / "model.safetensors"))
        assert {t.dtype for t in saved.values()} == {torch.bfloat16}, name
    one, auto, zero3 = runs["one"], runs["auto"], runs["zero3"]
    assert one[1]["steps"] == auto[1]["steps"] == zero3[1]["steps"] == 2
    assert not auto[1]["sharded"] and zero3[1]["sharded"]
    assert one[1]["dtypes"] == auto[1]["dtypes"] == ["torch.bfloat16"]
    assert zero3[1]["dtypes"] == ["torch.float32"]  # the fp32 master shards themselves
    init = one[2]
    for n in init:  # the same seeded bf16 initialisation in every run
        assert torch.equal(init[n], auto[2][n]) and torch.equal(init[n], zero3[2][n]), n
    # one rank's fp32 masters, from its training_state.pt (param_groups: decay, then no-decay)
    from pipelinerl_amd.finetune.optim import NO_DECAY

    st = torch.load(tmp_path / "one" / "finetune" / "training_state" / "training_state.pt", weights_only=True)
    names = list(init)
    order = [n for n in names if not any(k in n for k in NO_DECAY)] + [n for n in names if any(k in n for k in NO_DECAY)]
    masters = {n: st["optimizer_state"]["state"][i]["master"] for i, n in enumerate(order)}
    assert all(m.dtype == torch.float32 for m in masters.values())
    assert all(torch.equal(masters[n].to(torch.bfloat16), one[0][n]) for n in names)  # weights = rounded masters
    errs = {}
    for name, (params, _, _) in (("auto", auto), ("zero3", zero3)):
        # the two steps' update against one rank's, over all weights (for zero3, whose shards are
        # the fp32 masters, against one rank's masters): they differ by the gradient reduction's
        # summation order on bf16 gradients, which Adam amplifies on elements whose gradient is near
        # zero (measured 0.025 / 0.023)
        num = den = 0.0
        ref = one[0] if name == "auto" else masters  # the ZeRO-3 shards are masters: compare masters
        for n, t in ref.items():
            d_one, d_got = t.float() - init[n], params[n].float() - init[n]
            num += float(((d_got - d_one) ** 2).sum())
            den += float((d_one ** 2).sum())
        errs[name] = (num / den) ** 0.5
    print(json.dumps({"update_rel_err_vs_one_rank": errs}))
    assert errs["auto"] < 0.05 and errs["zero3"] < 0.05, errs
