"""HIP flash attention (csrc/attn_bwd.hip: forward and backward) for packed causal attention vs
torch's varlen flash attention and an fp32 per-sequence reference."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(bounds, hq=12, hkv=2, D=128, seed=0):
    T = bounds[-1]
    g = torch.Generator(device=DEV).manual_seed(seed)
    q = torch.randn((T, hq, D), generator=g, device=DEV).to(torch.bfloat16)
    k = torch.randn((T, hkv, D), generator=g, device=DEV).to(torch.bfloat16)
    v = torch.randn((T, hkv, D), generator=g, device=DEV).to(torch.bfloat16)
    do = torch.randn((T, hq, D), generator=g, device=DEV).to(torch.bfloat16)
    return q, k, v, do


def _run(fn, q, k, v, do):
    qq, kk, vv = (t.clone().requires_grad_() for t in (q, k, v))
    out = fn(qq, kk, vv)
    out.backward(do)
    return out.detach(), qq.grad, kk.grad, vv.grad


def _fp32_ref(q, k, v, do, bounds):
    rep = q.shape[1] // k.shape[1]
    qq, kk, vv = (t.float().clone().requires_grad_() for t in (q, k, v))
    outs = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        qi = qq[a:b].transpose(0, 1)
        ki = kk[a:b].repeat_interleave(rep, 1).transpose(0, 1)
        vi = vv[a:b].repeat_interleave(rep, 1).transpose(0, 1)
        outs.append(torch.nn.functional.scaled_dot_product_attention(qi, ki, vi, is_causal=True).transpose(0, 1))
    out = torch.cat(outs)
    out.backward(do.float())
    return out.detach(), qq.grad, kk.grad, vv.grad


@pytest.mark.parametrize("fwd", ["hip", "torch"])
@pytest.mark.parametrize("bounds", [[0, 2048, 4096], [0, 1, 37, 300, 531, 1024, 1151], [0, 129, 130, 3000]])
def test_hip_backward_matches(bounds, fwd, monkeypatch):
    monkeypatch.setenv("PRL_ATTN_FWD", fwd)
    from torch.nn.attention.varlen import varlen_attn

    from pipelinerl_amd.finetune.attention import PackedCausalAttention

    q, k, v, do = _inputs(bounds)
    rep = q.shape[1] // k.shape[1]
    cu = torch.tensor(bounds, dtype=torch.int32, device=DEV)
    mx = max(b - a for a, b in zip(bounds[:-1], bounds[1:]))

    def ours(qq, kk, vv):  # GQA native: k / v keep their 2 heads
        return PackedCausalAttention.apply(qq, kk, vv, cu, mx, bounds)

    def lib(qq, kk, vv):
        return varlen_attn(qq, kk.repeat_interleave(rep, 1), vv.repeat_interleave(rep, 1), cu, cu, mx, mx,
                           is_causal=True)

    a = _run(ours, q, k, v, do)
    b = _run(lib, q, k, v, do)
    ref = _fp32_ref(q, k, v, do, bounds)
    if fwd == "torch":
        assert torch.equal(a[0], b[0])  # the library's forward
    else:  # HIP forward: as close to the fp32 reference as the library's
        scale = float(ref[0].abs().max())
        err_ours = float((a[0].float() - ref[0]).abs().max()) / scale
        err_lib = float((b[0].float() - ref[0]).abs().max()) / scale
        assert err_ours <= max(1e-2, 2 * err_lib), ("out", err_ours, err_lib)
    for name, x, y, r in zip(("dq", "dk", "dv"), a[1:], b[1:], ref[1:]):
        scale = float(r.abs().max())
        err_ours = float((x.float() - r).abs().max()) / scale
        err_lib = float((y.float() - r).abs().max()) / scale
        assert err_ours <= max(1e-2, 2 * err_lib), (name, err_ours, err_lib)
    c = _run(ours, q, k, v, do)  # deterministic: no atomics
    assert all(torch.equal(x, y) for x, y in zip(a[1:], c[1:]))


@pytest.mark.parametrize("heads", [(12, 2), (28, 4)])
@pytest.mark.parametrize("bounds", [[0, 4096], [0, 3000, 3400, 3500], [0, 3160, 6443]])
def test_split_heavy_key_blocks(bounds, heads, monkeypatch):
    """Heavy dK/dV key blocks split over query heads (prl_attn_bwd_split, the default): dq
    bit-identical to the unsplit launch, dk / dv within the unsplit kernel's error of the fp32
    reference (the partial sums change the fp32 summation order), runs bitwise repeatable, and the
    plan does split these packings."""
    from pipelinerl_amd.finetune.attention import PackedCausalAttention, split_plan

    assert split_plan(bounds, *heads, torch.cuda.get_device_properties(0).multi_processor_count)[1]
    q, k, v, do = _inputs(bounds, *heads, seed=4)
    cu = torch.tensor(bounds, dtype=torch.int32, device=DEV)
    mx = max(b - a for a, b in zip(bounds[:-1], bounds[1:]))

    def ours(qq, kk, vv):
        return PackedCausalAttention.apply(qq, kk, vv, cu, mx, bounds)

    monkeypatch.setenv("PRL_ATTN_SPLIT", "0")
    a = _run(ours, q, k, v, do)
    monkeypatch.setenv("PRL_ATTN_SPLIT", "1")
    b = _run(ours, q, k, v, do)
    c = _run(ours, q, k, v, do)
    ref = _fp32_ref(q, k, v, do, bounds)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])  # out, dq
    for name, x, y, r in zip(("dk", "dv"), a[2:], b[2:], ref[2:]):
        scale = float(r.abs().max())
        err_split = float((y.float() - r).abs().max()) / scale
        err_one = float((x.float() - r).abs().max()) / scale
        assert err_split <= max(1e-2, 1.5 * err_one), (name, err_split, err_one)
    assert all(torch.equal(x, y) for x, y in zip(b, c))


@pytest.mark.parametrize("heads", [(14, 2), (40, 8)])
@pytest.mark.parametrize("bounds", [[0, 4096], [0, 3000, 3400, 3500], [0, 1, 700, 2900, 3100]])
def test_reference_model_gqa_ratios(bounds, heads):
    """The query / kv head counts of the other BASELINE models (C1 Qwen2.5-0.5B: 14 / 2, C5
    Qwen2.5-32B: 40 / 8, a group of 5 — the XCD remap's and the split plan's non-power-of-two
    case) through the HIP forward and the default (split) backward: within the bf16 error of the
    fp32 per-sequence reference, and bitwise repeatable."""
    from pipelinerl_amd.finetune.attention import PackedCausalAttention

    q, k, v, do = _inputs(bounds, *heads, seed=7)
    cu = torch.tensor(bounds, dtype=torch.int32, device=DEV)
    mx = max(b - a for a, b in zip(bounds[:-1], bounds[1:]))

    def ours(qq, kk, vv):
        return PackedCausalAttention.apply(qq, kk, vv, cu, mx, bounds)

    a = _run(ours, q, k, v, do)
    ref = _fp32_ref(q, k, v, do, bounds)
    for name, x, r in zip(("out", "dq", "dk", "dv"), a, ref):
        scale = float(r.abs().max())
        err = float((x.float() - r).abs().max()) / scale
        assert err <= 1e-2, (name, err)
    b = _run(ours, q, k, v, do)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
