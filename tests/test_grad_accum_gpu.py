"""Weight gradients accumulated in place (finetune/model_ops.py _wgrad, rl/fused_linear.py
_weight_grad, csrc/flat_pack.hip prl_grad_scale_bf16) against autograd's own accumulation over
the same micro-batches, on the GPU: the patched decoder's linear layers (wgrad GEMM with
beta = 1), the fused lm_head (one scale / accumulate pass), and the DP loop's gradient buckets
(hooks still fire on the armed boundary micro-batch)."""

import copy
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bits(t):
    """Bit patterns with every NaN canonicalised (a NaN's payload / sign is not a result)."""
    b = t.contiguous().view(torch.int16).clone()
    b[torch.isnan(t)] = 0x7FC0
    return b


@pytest.mark.parametrize("src_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("scale", [1.0, 0.37, 0.0])
def test_grad_scale_kernel_bit_exact(src_dtype, scale):
    """prl_grad_scale_bf16 == the ATen chain it replaces: (src.float() * g).to(bf16), and the
    AccumulateGrad add grad + that (bf16 + bf16 in fp32, rounded once)."""
    from pipelinerl_amd import _native

    lib = _native.load()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=DEV).manual_seed(1)
    n = 8 * 4099 + 5  # ragged tail
    src = (torch.randn(n, generator=g, device=DEV) * 3).to(src_dtype)
    src[:3] = torch.tensor([float("nan"), float("inf"), -0.0])
    grad = (torch.randn(n, generator=g, device=DEV)).to(torch.bfloat16)
    s = torch.tensor([scale], device=DEV)
    dt = _native.PRL_F32 if src_dtype == torch.float32 else _native.PRL_BF16
    want = (src.float() * s).to(torch.bfloat16)
    out = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    _native.check(lib.prl_grad_scale_bf16(src.data_ptr(), dt, s.data_ptr(), out.data_ptr(), n, 0, st), "scale")
    assert torch.equal(_bits(out), _bits(want))
    acc = grad.clone()
    _native.check(lib.prl_grad_scale_bf16(src.data_ptr(), dt, s.data_ptr(), acc.data_ptr(), n, 1, st), "acc")
    assert torch.equal(_bits(acc), _bits(grad + want))
    if src_dtype == torch.bfloat16:  # in place: nothing written at scale 1
        ip = src.clone()
        _native.check(lib.prl_grad_scale_bf16(ip.data_ptr(), dt, s.data_ptr(), ip.data_ptr(), n, 0, st), "in place")
        assert torch.equal(_bits(ip), _bits(want))
    assert lib.prl_grad_scale_bf16(src.data_ptr(), 7, s.data_ptr(), out.data_ptr(), n, 0, st) != 0
    assert lib.prl_grad_scale_bf16(None, dt, s.data_ptr(), out.data_ptr(), n, 0, st) == 1001


def _tiny(tmp_path):
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd.finetune.attention import register

    cfg = AutoConfig.from_pretrained(tiny_model_dir(tmp_path, vocab=512))
    cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.num_key_value_heads = 256, 512, 4, 2
    torch.manual_seed(0)
    return AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16, attn_implementation=register()).to(DEV)


def _micro_batches(n, T=96):
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 512, (1, T), generator=g).to(DEV)
        pos = torch.cat([torch.arange(40), torch.arange(T - 40)])[None].to(DEV)
        out.append((ids, pos))
    return out


def _run(model, batches, kw_of, fuse: bool, monkeypatch, on_pass=None):
    from pipelinerl_amd.finetune import model_ops

    monkeypatch.setattr(model_ops, "_FUSE_GRAD_ACCUM", fuse)
    for i, (ids, pos) in enumerate(batches):
        if on_pass is not None:
            on_pass(i)
        lg = model(input_ids=ids, position_ids=pos, **kw_of(pos)).logits
        lg.float().pow(2).mean().backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def _packed_kw(pos):
    from pipelinerl_amd.finetune.attention import packed_kwargs

    batch = type("B", (), {"seq_boundaries": torch.tensor([0, 40, pos.shape[1]]), "position_ids": pos})()
    return packed_kwargs(batch, DEV)


def _compare(a, b, rel=2e-2):
    for n in a:
        err = float((a[n].float() - b[n].float()).abs().max())
        assert err <= rel * float(a[n].float().abs().max()) + 1e-6, (n, err)


def test_linear_wgrad_accumulates_in_the_gemm(tmp_path, monkeypatch):
    """Three micro-batches through a patched Qwen2: the fused accumulation (every wgrad after the
    first added by the GEMM, beta = 1) == autograd's AccumulateGrad adds, to bf16 rounding; the
    fused run really took the beta = 1 path."""
    from pipelinerl_amd import gemm
    from pipelinerl_amd.finetune.model_ops import patch_model

    base = _tiny(tmp_path)
    try:
        models = [copy.deepcopy(base) for _ in range(2)]
        for m in models:
            patch_model(m)
        batches = _micro_batches(3)
        ref = _run(models[0], batches, _packed_kw, False, monkeypatch)
        calls = []
        orig = gemm.linear_wgrad

        def spy(dy, x, out=None, accumulate=False):
            calls.append(accumulate and out is not None and out.dtype == torch.bfloat16)
            return orig(dy, x, out=out, accumulate=accumulate)

        monkeypatch.setattr(gemm, "linear_wgrad", spy)
        got = _run(models[1], batches, _packed_kw, True, monkeypatch)
    finally:
        from transformers.models.qwen2 import modeling_qwen2 as mq

        f = mq.apply_rotary_pos_emb
        if getattr(f, "_prl_fused", False):
            mq.apply_rotary_pos_emb = f._prl_orig
    nl = base.config.num_hidden_layers
    from pipelinerl_amd.finetune import model_ops

    # q/k/v (one fused GEMM or three), o, gate/up (one or two), down per layer
    per_layer = (1 if model_ops._FUSED_QKV else 3) + 1 + (1 if model_ops._FUSED_GATE_UP else 2) + 1
    assert sum(calls) == 2 * (per_layer * nl + 1)  # micro-batches 2 and 3, + lm_head
    _compare(ref, got)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_grad_buckets_hooks_fire_on_the_armed_pass(tmp_path, monkeypatch):
    """With the DP loop's GradBuckets (grads are views of flat buckets, never None): passes before
    the boundary accumulate in the GEMM (no hook due), the armed boundary pass goes through
    autograd so every bucket's hook fires and its all-reduce launches from the backward; the
    reduced gradients equal the unfused run's (world 1, gloo)."""
    import torch.distributed as dist

    from pipelinerl_amd.finetune.grad_sync import GradBuckets
    from pipelinerl_amd.finetune.model_ops import patch_model

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    try:
        base = _tiny(tmp_path)
        batches = _micro_batches(3)
        results = []
        for fuse in (False, True):
            m = copy.deepcopy(base)
            patch_model(m)
            gb = GradBuckets(list(m.parameters()), bucket_bytes=1 << 20)
            launched = []
            orig_launch = gb._launch
            monkeypatch.setattr(gb, "_launch", lambda b, _o=orig_launch: (launched.append(b), _o(b)))
            grads = _run(m, batches, _packed_kw, fuse, monkeypatch,
                         on_pass=lambda i, gb=gb: gb.arm() if i == len(batches) - 1 else None)
            # every bucket launched from a hook during the armed backward, none left for finish()
            assert len(launched) == len(gb.buckets)
            gb.finish()
            torch.cuda.synchronize()
            grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
            results.append(grads)
        _compare(results[0], results[1])
    finally:
        dist.destroy_process_group()
        from transformers.models.qwen2 import modeling_qwen2 as mq

        f = mq.apply_rotary_pos_emb
        if getattr(f, "_prl_fused", False):
            mq.apply_rotary_pos_emb = f._prl_orig


def test_fused_lm_head_weight_grad_accumulates(tmp_path, monkeypatch):
    """rl_step with the label-row lm_head over two micro-batches: lm_head.weight.grad with the
    in-place accumulation (second micro-batch) == the sum autograd forms (two separate runs
    added), and a sentinel-style x0 upstream adds exact zeros."""
    import types

    from loop_helpers import rollouts
    from pipelinerl_amd.finetune import model_ops
    from pipelinerl_amd.finetune.data import collate_packed
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    base = _tiny(tmp_path)
    base.config.tie_word_embeddings = False
    base.lm_head.weight = torch.nn.Parameter(base.lm_head.weight.detach().clone())
    cfg = RLConfig(policy_loss="ppo", epsilon=4.0, batch_size=8)
    tok = types.SimpleNamespace(eos_token_id=511)
    bs = [collate_packed(rollouts(2, 4, seed=s, vocab=512), tok, 1).to_device(DEV) for s in (3, 4)]

    def grads(batches, fuse, scale_last=1.0):
        monkeypatch.setattr(model_ops, "_FUSE_GRAD_ACCUM", fuse)
        m = copy.deepcopy(base)
        for i, b in enumerate(batches):
            loss, _ = rl_step(m, b, 0, 10, cfg)
            (loss * scale_last if i == len(batches) - 1 else loss).backward()
        torch.cuda.synchronize()
        return m.lm_head.weight.grad.detach().clone()

    sep = [grads([b], True) for b in bs]
    both = grads(bs, True)
    ref = grads(bs, False)
    assert torch.equal(_bits(both), _bits(ref))  # same two roundings as AccumulateGrad's add
    assert torch.equal(_bits(both), _bits(sep[0] + sep[1]))
    zero = grads(bs, True, scale_last=0.0)
    assert torch.equal(_bits(zero), _bits(sep[0]))
