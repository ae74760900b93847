"""Fused model ops (csrc/model_ops.hip) against the eager HF chains they replace, on the GPU.
Forward: bit-identical to the eager bf16 chain.  Backward: against torch autograd through the
same chain and against an fp32 reference of the op."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _eager_rmsnorm(x, w, eps):  # transformers Qwen2RMSNorm.forward
    h = x.to(torch.float32)
    var = h.pow(2).mean(-1, keepdim=True)
    h = h * torch.rsqrt(var + eps)
    return w * h.to(x.dtype)


def _close(a, b, rtol, atol=0.0):
    err = (a.float() - b.float()).abs()
    lim = atol + rtol * b.float().abs()
    return bool((err <= lim).all()), float(err.max())


@pytest.mark.parametrize("H", [896, 1536, 3584, 5120])
def test_rmsnorm(H):
    from pipelinerl_amd.finetune.model_ops import RMSNormFn

    g = torch.Generator(device=DEV).manual_seed(H)
    x = (torch.randn((3, 701, H), generator=g, device=DEV) * 2).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, generator=g, device=DEV)).to(torch.bfloat16)
    dy = torch.randn((3, 701, H), generator=g, device=DEV).to(torch.bfloat16)
    xa, wa = x.clone().requires_grad_(), w.clone().requires_grad_()
    ya = _eager_rmsnorm(xa, wa, 1e-6)
    ya.backward(dy)
    xb, wb = x.clone().requires_grad_(), w.clone().requires_grad_()
    yb = RMSNormFn.apply(xb, wb, 1e-6)
    yb.backward(dy)
    # forward: same roundings; rstd from a different fp32 summation order may flip a last bit
    diff = (ya.float() != yb.float()).float().mean().item()
    assert diff < 1e-3, diff
    assert _close(yb, ya, 1.6e-2)[0]  # <= 2 bf16 ulps where a last bit of rstd flips
    ok, err = _close(xb.grad, xa.grad, 2e-2, 1e-3)
    assert ok, err
    # fp32 reference of the op for the weight gradient (both bf16 paths reduce 2103 rows)
    xf, wf = x.float().requires_grad_(), w.float().requires_grad_()
    (_eager_rmsnorm(xf, wf, 1e-6) * dy.float()).sum().backward()
    ok, err = _close(wb.grad, wf.grad, 2e-2, 1e-2 * float(wf.grad.abs().max()))
    assert ok, err


@pytest.mark.parametrize("shape", [(5, 333, 1024), (1, 77, 4864), (1, 61, 27648)])  # toy, 0.5B, 32B widths
def test_swiglu(shape):
    from pipelinerl_amd.finetune.model_ops import SwiGLUFn

    g0 = torch.Generator(device=DEV).manual_seed(1)
    gate = (torch.randn(shape, generator=g0, device=DEV) * 3).to(torch.bfloat16)
    up = torch.randn(shape, generator=g0, device=DEV).to(torch.bfloat16)
    dh = torch.randn(shape, generator=g0, device=DEV).to(torch.bfloat16)
    ga, ua = gate.clone().requires_grad_(), up.clone().requires_grad_()
    ha = torch.nn.functional.silu(ga) * ua
    ha.backward(dh)
    gb, ub = gate.clone().requires_grad_(), up.clone().requires_grad_()
    hb = SwiGLUFn.apply(gb, ub)
    hb.backward(dh)
    assert torch.equal(ha, hb)
    assert torch.equal(ua.grad, ub.grad)
    ok, err = _close(gb.grad, ga.grad, 8e-3, 1e-6)
    assert ok, err


def test_swiglu_phased_chunks_claimed_and_static():
    """The phased kernels at a size with many chunks per workgroup (4096 x 8960: 4480 forward chunks
    for a 256-workgroup grid): chunks claimed from the caller's counter (the default) and the static
    stride (no counter) give bit-identical outputs, equal to the eager forward."""
    from pipelinerl_amd.finetune import model_ops
    from pipelinerl_amd.finetune.model_ops import SwiGLUFn

    g0 = torch.Generator(device=DEV).manual_seed(2)
    gate = (torch.randn((4096, 8960), generator=g0, device=DEV) * 3).to(torch.bfloat16)
    up = torch.randn((4096, 8960), generator=g0, device=DEV).to(torch.bfloat16)
    dh = torch.randn((4096, 8960), generator=g0, device=DEV).to(torch.bfloat16)
    outs = {}
    orig = model_ops._chunk_counter
    for arm in ("claim", "static"):
        if arm == "static":
            model_ops._chunk_counter = lambda t: None
        try:
            gb, ub = gate.clone().requires_grad_(), up.clone().requires_grad_()
            hb = SwiGLUFn.apply(gb, ub)
            hb.backward(dh)
            torch.cuda.synchronize()
        finally:
            model_ops._chunk_counter = orig
        outs[arm] = (hb.detach(), gb.grad, ub.grad)
    for a, b in zip(outs["claim"], outs["static"]):
        assert torch.equal(a, b)
    assert torch.equal(outs["claim"][0], torch.nn.functional.silu(gate) * up)


@pytest.mark.parametrize("heads", [(12, 2), (14, 2), (28, 4), (40, 8)])  # 1.5B, 0.5B, 7B, 32B
def test_rope_matches_hf(heads):
    from transformers.models.qwen2 import modeling_qwen2 as mq

    from pipelinerl_amd.finetune.model_ops import RopeFn

    B, T, D = 2, 97, 128
    hq, hkv = heads
    g = torch.Generator(device=DEV).manual_seed(3)
    qp = torch.randn((B, T, hq * D), generator=g, device=DEV).to(torch.bfloat16)
    kp = torch.randn((B, T, hkv * D), generator=g, device=DEV).to(torch.bfloat16)
    pos = torch.arange(T, device=DEV)[None].expand(B, T) + torch.tensor([[0], [5]], device=DEV)
    inv = 1.0 / (1e6 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    fr = pos[..., None].float() * inv
    emb = torch.cat([fr, fr], -1)
    cos, sin = emb.cos().to(torch.bfloat16), emb.sin().to(torch.bfloat16)
    dq = torch.randn((B, hq, T, D), generator=g, device=DEV).to(torch.bfloat16)
    dk = torch.randn((B, hkv, T, D), generator=g, device=DEV).to(torch.bfloat16)

    def views(a, b):
        a = a.clone().requires_grad_()
        b = b.clone().requires_grad_()
        return a, b, a.view(B, T, hq, D).transpose(1, 2), b.view(B, T, hkv, D).transpose(1, 2)

    qa0, ka0, qa, ka = views(qp, kp)
    oqa, oka = mq.apply_rotary_pos_emb(qa, ka, cos, sin)
    torch.autograd.backward([oqa, oka], [dq, dk])
    qb0, kb0, qb, kb = views(qp, kp)
    oqb, okb = RopeFn.apply(qb, kb, cos, sin)
    torch.autograd.backward([oqb, okb], [dq, dk])
    assert torch.equal(oqa, oqb) and torch.equal(oka, okb)
    assert oqb.transpose(1, 2).is_contiguous()
    assert torch.equal(qa0.grad, qb0.grad) and torch.equal(ka0.grad, kb0.grad)


@pytest.mark.parametrize("shape", [(16384, 1536, 256), (4096, 1536, 1536), (3000, 64, 96), (37, 8, 24)])
def test_prl_linear(shape):
    """PrlLinearFn: torch's forward (bit-identical), backward GEMMs through prl_gemm within bf16
    rounding of the fp32 products (the same bound torch's own backward meets)."""
    from pipelinerl_amd.finetune.model_ops import PrlLinearFn

    T, K, N = shape
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn((1, T, K), generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn((N, K), generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=DEV).to(torch.bfloat16)
    dy = torch.randn((1, T, N), generator=g, device=DEV).to(torch.bfloat16)
    ga = [t.clone().requires_grad_() for t in (x, w, b)]
    gb = [t.clone().requires_grad_() for t in (x, w, b)]
    ya = torch.nn.functional.linear(*ga)
    ya.backward(dy)
    yb = PrlLinearFn.apply(*gb)
    yb.backward(dy)
    assert torch.equal(ya, yb)
    refs = (dy[0].float() @ w.float(), dy[0].float().t() @ x[0].float(), dy[0].float().sum(0))
    for i, ref in enumerate(refs):
        tol = 1e-2 * float(ref.abs().max())
        for got in (ga[i].grad, gb[i].grad):
            assert float((got.reshape(ref.shape).float() - ref).abs().max()) <= tol, (i, shape)


@pytest.mark.parametrize("H", [256, 1536, 3584])
def test_add_rmsnorm(H):
    """AddRMSNormFn: h and y bit-identical to eager `residual + x` then Qwen2RMSNorm; gradients
    of residual, x and w vs eager autograd (which sums the residual-stream and norm gradients
    in a separate bf16 add), with and without a gradient reaching h directly."""
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RMSNorm

    from pipelinerl_amd.finetune.model_ops import AddRMSNormFn, RMSNormFn

    T = 777
    g = torch.Generator(device=DEV).manual_seed(11)
    r = torch.randn((1, T, H), generator=g, device=DEV).to(torch.bfloat16)
    x = torch.randn((1, T, H), generator=g, device=DEV).to(torch.bfloat16)
    norm = Qwen2RMSNorm(H, eps=1e-6).to(DEV, torch.bfloat16)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.1 * torch.randn(H, generator=g, device=DEV))
    dh = torch.randn((1, T, H), generator=g, device=DEV).to(torch.bfloat16)
    dy = torch.randn((1, T, H), generator=g, device=DEV).to(torch.bfloat16)
    for with_dh in (True, False):
        ra, xa, wa = (t.detach().clone().requires_grad_() for t in (r, x, norm.weight))
        rb, xb, wb = (t.detach().clone().requires_grad_() for t in (r, x, norm.weight))
        ha = ra + xa
        ya = Qwen2RMSNorm.forward(type("N", (), {"weight": wa, "variance_epsilon": 1e-6})(), ha)  # eager, weight wa
        hb, yb = AddRMSNormFn.apply(rb, xb, wb, 1e-6)
        assert torch.equal(ha, hb)
        # y: the same kernel as RMSNormFn on h (bit-identical to it); vs eager up to a last-bit
        # rstd flip (test_rmsnorm)
        assert torch.equal(yb, RMSNormFn.apply(hb.detach(), wb.detach(), 1e-6))
        assert (ya.float() != yb.float()).float().mean().item() < 1e-3 and _close(yb, ya, 1.6e-2)[0]
        outs_a, outs_b = ([ha, ya], [dh, dy]), ([hb, yb], [dh, dy])
        if not with_dh:
            outs_a, outs_b = ([ya], [dy]), ([yb], [dy])
        torch.autograd.backward(*outs_a)
        torch.autograd.backward(*outs_b)
        for ga, gb in ((ra.grad, rb.grad), (xa.grad, xb.grad), (wa.grad, wb.grad)):
            err = float((ga.float() - gb.float()).abs().max())
            assert err <= 2e-2 * float(ga.float().abs().max()) + 1e-6, (H, with_dh, err)


@pytest.mark.parametrize("bias", [True, False])
def test_shared_input_linear(bias):
    """SharedInputLinearFn (q/k/v-shaped: 3 layers on one input, dgrads summed in the GEMM
    epilogue with beta = 1): outputs equal separate linears, gradients within bf16 rounding of
    the fp32 products; a layer whose output is unused contributes nothing."""
    from pipelinerl_amd.finetune.model_ops import SharedInputLinearFn

    T, K, Ns = 1000, 512, (512, 128, 128)
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn((1, T, K), generator=g, device=DEV).to(torch.bfloat16)
    ws = [(torch.randn((n, K), generator=g, device=DEV) * 0.05).to(torch.bfloat16) for n in Ns]
    bs = [torch.randn(n, generator=g, device=DEV).to(torch.bfloat16) if bias else None for n in Ns]
    dys = [torch.randn((1, T, n), generator=g, device=DEV).to(torch.bfloat16) for n in Ns]
    for used in ((0, 1, 2), (0, 2)):
        xa = x.clone().requires_grad_()
        wa = [w.clone().requires_grad_() for w in ws]
        ba = [b.clone().requires_grad_() if b is not None else None for b in bs]
        ys = SharedInputLinearFn.apply(xa, *[t for p in zip(wa, ba) for t in p])
        for i, y in enumerate(ys):
            assert torch.equal(y, torch.nn.functional.linear(x, ws[i], bs[i]))
        torch.autograd.backward([ys[i] for i in used], [dys[i] for i in used])
        dx = sum(dys[i][0].float() @ ws[i].float() for i in used)
        assert float((xa.grad[0].float() - dx).abs().max()) <= 1e-2 * float(dx.abs().max())
        for i in range(3):
            if i not in used:
                assert wa[i].grad is None
                continue
            ref = dys[i][0].float().t() @ x[0].float()
            assert float((wa[i].grad.float() - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
            if bias:
                ref = dys[i][0].float().sum(0)
                assert float((ba[i].grad.float() - ref).abs().max()) <= 1e-2 * float(ref.abs().max())


# toy, then two decoder layers of the 7B (C3 / C4) and 32B (C5) shapes: head dim 128 (the HIP
# attention), GQA groups of 7 and 5, the wide MLPs
@pytest.mark.parametrize("shape", [(256, 512, 4, 2), (3584, 18944, 28, 4), (5120, 27648, 40, 8)])
def test_patched_qwen2_matches_eager(tmp_path, shape):
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd.finetune.attention import packed_kwargs, register
    from pipelinerl_amd.finetune.model_ops import patch_model

    cfg = AutoConfig.from_pretrained(tiny_model_dir(tmp_path, vocab=512))
    cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.num_key_value_heads = shape
    cfg.num_hidden_layers = 2
    torch.manual_seed(0)
    eager = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16, attn_implementation=register()).to(DEV)
    fused = copy.deepcopy(eager)
    T = 96
    ids = torch.randint(0, 512, (1, T), device=DEV)
    pos = torch.cat([torch.arange(40), torch.arange(56)])[None].to(DEV)
    batch = type("B", (), {"seq_boundaries": torch.tensor([0, 40, 96]), "position_ids": pos})()
    kw = packed_kwargs(batch, DEV)
    outs = []
    try:
        for m in (eager, fused):
            if m is fused:  # patch after the eager pass: the RoPE patch is module-wide
                counts = patch_model(fused)
                assert counts["rmsnorm"] == 2 * cfg.num_hidden_layers + 1
                assert counts["swiglu_mlp"] == cfg.num_hidden_layers and counts["rope_modules"] == 1
                assert counts["prl_linear"] == 7 * cfg.num_hidden_layers + 1  # + lm_head
                assert counts["qkv_groups"] == cfg.num_hidden_layers
                assert counts["add_norm_layers"] == cfg.num_hidden_layers
            lg = m(input_ids=ids, position_ids=pos, **kw).logits
            lg.float().pow(2).mean().backward()
            outs.append(lg.detach())
    finally:
        from transformers.models.qwen2 import modeling_qwen2 as mq

        f = mq.apply_rotary_pos_emb
        if getattr(f, "_prl_fused", False):  # leave the module as other tests expect it
            mq.apply_rotary_pos_emb = f._prl_orig
    assert (outs[0].float() - outs[1].float()).abs().max() <= 5e-2 * outs[0].float().abs().max()
    for (n, p), (_, q) in zip(eager.named_parameters(), fused.named_parameters()):
        err = float((p.grad.float() - q.grad.float()).abs().max())
        assert err <= 5e-2 * float(p.grad.float().abs().max()) + 1e-6, (n, err)


@pytest.mark.parametrize("reentrant", [False, True])
def test_patched_qwen2_gradient_checkpointing(tmp_path, reentrant):
    """The decoder fusions under HF gradient checkpointing (the layer forward runs twice; the
    cross-layer norm hand-over is skipped): patched + checkpointed == eager + checkpointed."""
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd.finetune.attention import packed_kwargs, register
    from pipelinerl_amd.finetune.model_ops import patch_model

    cfg = AutoConfig.from_pretrained(tiny_model_dir(tmp_path, vocab=512))
    cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.num_key_value_heads = 256, 512, 4, 2
    torch.manual_seed(0)
    eager = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16, attn_implementation=register()).to(DEV)
    fused = copy.deepcopy(eager)
    T = 96
    ids = torch.randint(0, 512, (1, T), device=DEV)
    pos = torch.cat([torch.arange(40), torch.arange(56)])[None].to(DEV)
    batch = type("B", (), {"seq_boundaries": torch.tensor([0, 40, 96]), "position_ids": pos})()
    kw = packed_kwargs(batch, DEV)
    outs = []
    try:
        for m in (eager, fused):
            if m is fused:
                patch_model(fused)
            m.train()
            m.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": reentrant})
            if reentrant:  # the reentrant form needs an input that requires grad to build a graph
                m.enable_input_require_grads()
            lg = m(input_ids=ids, position_ids=pos, use_cache=False, **kw).logits
            lg.float().pow(2).mean().backward()
            outs.append(lg.detach())
    finally:
        from transformers.models.qwen2 import modeling_qwen2 as mq

        f = mq.apply_rotary_pos_emb
        if getattr(f, "_prl_fused", False):
            mq.apply_rotary_pos_emb = f._prl_orig
    assert (outs[0].float() - outs[1].float()).abs().max() <= 5e-2 * outs[0].float().abs().max()
    for (n, p), (_, q) in zip(eager.named_parameters(), fused.named_parameters()):
        err = float((p.grad.float() - q.grad.float()).abs().max())
        assert err <= 5e-2 * float(p.grad.float().abs().max()) + 1e-6, (n, err)
    assert all(m.__dict__.get("_prl_pending") is None for m in fused.modules())


def test_varlen_gqa_native_matches_repeated():
    """torch's varlen flash attention takes GQA (Hkv < Hq) directly: forward and gradients equal
    the repeated-k/v form the attention path used before (finetune/attention.py)."""
    from torch.nn.attention.varlen import varlen_attn

    T, hq, hkv, D = 256, 12, 2, 128
    g = torch.Generator(device=DEV).manual_seed(0)
    q, k, v = (torch.randn((T, h, D), generator=g, device=DEV).to(torch.bfloat16) for h in (hq, hkv, hkv))
    do = torch.randn((T, hq, D), generator=g, device=DEV).to(torch.bfloat16)
    cu = torch.tensor([0, 100, 256], dtype=torch.int32, device=DEV)
    grads = []
    for rep in (False, True):
        qq, kk, vv = (t.clone().requires_grad_() for t in (q, k, v))
        kx, vx = (kk.repeat_interleave(hq // hkv, 1), vv.repeat_interleave(hq // hkv, 1)) if rep else (kk, vv)
        out = varlen_attn(qq, kx, vx, cu, cu, 156, 156, is_causal=True)
        out.backward(do)
        grads.append((out.detach(), qq.grad, kk.grad, vv.grad))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    for a, b in zip(grads[0][2:], grads[1][2:]):  # dk / dv: group sums in a different order
        assert float((a.float() - b.float()).abs().max()) <= 2e-2 * float(b.float().abs().max())
