"""fp32 master weights on the host side: which configs turn them on (``finetune.master_weights``,
finetune/optim.py master_weights_requested, following the reference's backend: DeepSpeed bf16
ZeRO-3 by default, conf/base.yaml:94-95), the CPU step (torch's fused fp32 AdamW on the masters,
used by the gloo rehearsals) against the fp32-master reference, and the checkpoint round trip."""

import io

import pytest
import torch

from pipelinerl_amd.config import Cfg, load_config
from pipelinerl_amd.finetune.optim import PrlAdamW, clip_grad_norm, get_optimizer, master_weights_requested


@pytest.mark.parametrize("cfg,expected", [
    ({"use_deepspeed": True, "deepspeed_config": "deepspeed_stage3_bf16"}, True),  # the reference default
    ({"use_deepspeed": False, "use_fsdp": True}, True),  # FSDP mixed precision
    ({"use_deepspeed": False, "use_fsdp": False}, False),  # plain DDP: bf16 weights trained directly
    ({}, True),  # no backend named: the reference default's
    ({"use_deepspeed": True, "finetune": {"master_weights": False}}, False),
    ({"use_deepspeed": False, "finetune": {"master_weights": True}}, True),
])
def test_master_weights_follow_the_reference_backend(cfg, expected):
    cfg = Cfg.wrap({"finetune": {}, **cfg})
    assert master_weights_requested(cfg) is expected


def test_master_weights_rejects_unknown_mode():
    with pytest.raises(ValueError):
        master_weights_requested(Cfg.wrap({"finetune": {"master_weights": "sometimes"}}))


def test_reference_default_config_selects_master_weights():
    """The reference's own default exp_config (tests/golden/exp_config_math_grpo.yaml, composed
    from conf/base.yaml) keeps fp32 masters."""
    from pathlib import Path

    cfg = load_config(Path(__file__).parent / "golden", "exp_config_math_grpo")
    assert cfg.use_deepspeed is True
    assert master_weights_requested(cfg)


def _model(seed=0):
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(64, 96), torch.nn.Linear(96, 33)).to(torch.bfloat16)
    return m


def _grads(ps, step):
    g = torch.Generator().manual_seed(step)
    return [torch.randn(p.shape, generator=g).to(torch.bfloat16) for p in ps]


def test_cpu_master_step_matches_fp32_master_reference():
    model = _model()
    ps = list(model.parameters())
    masters = [torch.nn.Parameter(p.detach().float().clone()) for p in ps]
    opt = get_optimizer("adamw_torch", model, 1e-4, 0.01, master_weights=True)
    assert isinstance(opt, PrlAdamW) and opt.master_weights
    # the same decay / no-decay grouping as get_grouped_params (".bias" -> no decay)
    names = [n for n, _ in model.named_parameters()]
    groups = [{"params": [m for n, m in zip(names, masters) if "bias" not in n], "weight_decay": 0.01},
              {"params": [m for n, m in zip(names, masters) if "bias" in n], "weight_decay": 0.0}]
    ref = torch.optim.AdamW(groups, lr=1e-4, fused=True)
    for step in range(3):
        gs = _grads(ps, step)
        for p, m, g in zip(ps, masters, gs):
            p.grad = g.clone()
            m.grad = g.float()
        na = torch.nn.utils.clip_grad_norm_(masters, 0.3)
        nb = clip_grad_norm(ps, 0.3, opt)
        assert torch.equal(na, nb)
        ref.step()
        opt.step()
        for p, m in zip(ps, masters):
            assert torch.equal(opt.state[p]["master"], m.detach())
            assert torch.equal(p.detach(), m.detach().to(torch.bfloat16))
            assert torch.equal(opt.state[p]["exp_avg_sq"], ref.state[m]["exp_avg_sq"])


def test_cpu_master_state_dict_round_trip_keeps_fp32():
    model = _model(1)
    ps = list(model.parameters())
    opt = get_optimizer("adamw_torch", model, 1e-4, 0.01, master_weights=True)
    for step in range(2):
        for p, g in zip(ps, _grads(ps, step)):
            p.grad = g
        opt.step()
    buf = io.BytesIO()
    torch.save(opt.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    opt2 = get_optimizer("adamw_torch", model, 1e-4, 0.01, master_weights=True)
    opt2.load_state_dict(sd)
    for p in ps:
        a, b = opt.state[p], opt2.state[p]
        for k in ("master", "exp_avg", "exp_avg_sq"):
            assert b[k].dtype == torch.float32 and torch.equal(a[k], b[k])
    # without master weights the saved masters are dropped and the moments follow the parameters
    from pipelinerl_amd.finetune.optim import get_grouped_params

    opt3 = PrlAdamW(get_grouped_params(model, 0.01), lr=1e-4, master_weights=False)
    opt3.load_state_dict(sd)
    assert all("master" not in opt3.state[p] for p in ps)


def test_memory_plan_counts_master_state():
    """With master weights the plan's model state is weight + gradient (bf16) + master + two
    moments (fp32): 16 B per parameter instead of 8."""
    from types import SimpleNamespace

    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    cfg = SimpleNamespace(hidden_size=64, intermediate_size=128, num_attention_heads=4, num_key_value_heads=2,
                          num_hidden_layers=2, vocab_size=100, tie_word_embeddings=False)
    model = torch.nn.Linear(1000, 1000, bias=False).to(torch.bfloat16)
    model.config = cfg
    base = {"gradient_checkpointing": True, "seq_length": 128}
    p_bf16 = plan_gradient_checkpointing({**base, "master_weights": False}, model, torch.device("cpu"),
                                         device_bytes=200 << 30)
    p_master = plan_gradient_checkpointing({**base, "master_weights": True}, model, torch.device("cpu"),
                                           device_bytes=200 << 30)
    assert p_bf16.state_bytes == 8 * 1000 * 1000
    assert p_master.state_bytes == 16 * 1000 * 1000


def test_fsdp_master_shards_reduce_in_fp32():
    """fp32 master shards computed in bf16: the gradients are reduce-scattered in fp32 (the reference's
    fsdp reduce_dtype, conf/base.yaml:97-100).  FSDP2 reduces in param_dtype when reduce_dtype is None,
    so the policy must name fp32 even though it equals the shards' dtype (a round-6 build left it None
    and reduced in bf16: the 32B-shaped GPU test then matched a bf16 model's gradients bit for bit)."""
    import os

    import torch
    import torch.distributed as dist
    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd.finetune.sharding import shard_model

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        cfg = Qwen2Config(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                          num_key_value_heads=2, vocab_size=256)
        model = shard_model(AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16), master_weights=True)
        assert {p.dtype for p in model.parameters()} == {torch.float32}
        for unit in [model, *model.model.layers]:
            mp = unit._get_fsdp_state()._mp_policy
            assert mp.param_dtype == torch.bfloat16 and mp.reduce_dtype == torch.float32, mp
    finally:
        dist.destroy_process_group()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
