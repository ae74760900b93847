"""The HIP AdamW step (csrc/adamw.hip through finetune/optim.py PrlAdamW) against torch's fused
AdamW, with and without the gradient-clipping multiply folded in (clip_grad_norm): parameters,
both moments and the step counts bit for bit over several steps, on bf16 and fp32 parameters,
ragged sizes (vector body + scalar tail), a misaligned parameter (scalar path), a parameter
without a gradient on one step, and a torch-written state_dict loaded mid-run."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(1000, 64), (3584,), (1001,), (7,), (256, 264), (3, 5, 17)]


def _bits(t):
    return t.contiguous().view(torch.int16 if t.dtype == torch.bfloat16 else torch.int32)


def _params(dtype, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    ps = [torch.nn.Parameter((torch.randn(s, generator=g, device=DEV) * 0.1).to(dtype)) for s in SHAPES]
    base = (torch.randn(1025, generator=g, device=DEV) * 0.1).to(dtype)
    ps.append(torch.nn.Parameter(base[1:]))  # storage offset of one element: not 16-B aligned
    return ps


def _groups(ps, wd=0.01):
    return [{"params": ps[0::2], "weight_decay": wd}, {"params": ps[1::2], "weight_decay": 0.0}]


def _grads(ps, step, dtype, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(100 + step)
    return [(torch.randn(p.shape, generator=g, device=DEV) * scale).to(dtype) for p in ps]


def _assert_same(pa, pb, oa, ob):
    for a, b in zip(pa, pb):
        assert torch.equal(_bits(a.detach()), _bits(b.detach()))
        sa, sb = oa.state[a], ob.state[b]
        assert torch.equal(sa["step"], sb["step"])
        assert torch.equal(_bits(sa["exp_avg"]), _bits(sb["exp_avg"]))
        assert torch.equal(_bits(sa["exp_avg_sq"]), _bits(sb["exp_avg_sq"]))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("max_norm", [None, 0.3])
def test_adamw_matches_torch_fused(dtype, max_norm):
    from pipelinerl_amd.finetune.optim import PrlAdamW, clip_grad_norm

    pa, pb = _params(dtype), _params(dtype)
    ref = torch.optim.AdamW(_groups(pa), lr=3e-4, fused=True)
    opt = PrlAdamW(_groups(pb), lr=3e-4)
    for step in range(4):
        for ps in (pa, pb):
            for p, g in zip(ps, _grads(ps, step, dtype, scale=1.0 + step)):
                p.grad = None if (step == 2 and p is ps[3]) else g.clone()
        if max_norm is not None:
            na = torch.nn.utils.clip_grad_norm_(pa, max_norm)
            nb = clip_grad_norm(pb, max_norm, opt)
            assert torch.equal(na, nb) and float(na) > max_norm  # the clip is active
        ref.step()
        opt.step()
        for g in ref.param_groups:
            g["lr"] *= 0.9  # a scheduler between steps
        for g in opt.param_groups:
            g["lr"] *= 0.9
        _assert_same(pa, pb, ref, opt)
    assert float(opt.state[pb[3]]["step"]) == 3.0  # skipped on the step it had no gradient


def _checkpoint(sd):
    """Through torch.save / torch.load, as training_state.pt (a state_dict() aliases the live
    state tensors, which load_state_dict would otherwise share between the two optimizers)."""
    import io

    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def test_adamw_resumes_from_torch_state_dict():
    """A checkpoint written by torch's AdamW loads into PrlAdamW (same state keys) and the run
    continues bit for bit; and the other way round."""
    from pipelinerl_amd.finetune.optim import PrlAdamW

    dtype = torch.bfloat16
    pa, pb = _params(dtype, 1), _params(dtype, 1)
    ref = torch.optim.AdamW(_groups(pa), lr=1e-3, fused=True)
    for step in range(2):
        for p, g in zip(pa, _grads(pa, step, dtype)):
            p.grad = g
        ref.step()
    with torch.no_grad():
        for a, b in zip(pa, pb):
            b.copy_(a)
    opt = PrlAdamW(_groups(pb), lr=1e-3)
    opt.load_state_dict(_checkpoint(ref.state_dict()))
    for step in range(2, 4):
        for ps in (pa, pb):
            for p, g in zip(ps, _grads(ps, step, dtype)):
                p.grad = g.clone()
        ref.step()
        opt.step()
    _assert_same(pa, pb, ref, opt)
    back = torch.optim.AdamW(_groups(pa), lr=1e-3, fused=True)
    back.load_state_dict(_checkpoint(opt.state_dict()))
    assert torch.equal(back.state_dict()["state"][0]["exp_avg"], opt.state_dict()["state"][0]["exp_avg"])


def test_adamw_unsupported_group_takes_torch_step():
    """amsgrad is not in the kernel: the step is torch's own, with the deferred clip applied."""
    from pipelinerl_amd.finetune.optim import PrlAdamW, clip_grad_norm

    dtype = torch.bfloat16
    pa, pb = _params(dtype, 2), _params(dtype, 2)
    ref = torch.optim.AdamW(_groups(pa), lr=1e-3, amsgrad=True, fused=True)
    opt = PrlAdamW(_groups(pb), lr=1e-3, amsgrad=True)
    for step in range(2):
        for ps in (pa, pb):
            for p, g in zip(ps, _grads(ps, step, dtype, 4.0)):
                p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(pa, 0.5)
        clip_grad_norm(pb, 0.5, opt)
        ref.step()
        opt.step()
    for a, b in zip(pa, pb):
        assert torch.equal(_bits(a.detach()), _bits(b.detach()))


def test_adamw_abi_rejects_bad_arguments():
    import ctypes

    from pipelinerl_amd import _native

    lib = _native.load()
    p = torch.zeros(8, device=DEV, dtype=torch.bfloat16)
    s = torch.zeros((), device=DEV)
    ptrs = (ctypes.c_uint64 * 1)(p.data_ptr())
    nul = (ctypes.c_uint64 * 1)(0)
    steps = (ctypes.c_uint64 * 1)(s.data_ptr())
    n = (ctypes.c_int64 * 1)(8)
    st = torch.cuda.current_stream().cuda_stream
    args = (1e-3, 0.9, 0.999, 0.0, 1e-8, None, st)
    assert lib.prl_adamw_step(1, ptrs, nul, ptrs, ptrs, steps, n, 1, *args) == 1001
    assert lib.prl_adamw_step(1, ptrs, ptrs, ptrs, ptrs, steps, n, 7, *args) == 1002
    assert lib.prl_adamw_step(0, None, None, None, None, None, None, 1, *args) == 0
