"""fp32 master weights (csrc/adamw.hip prl_adamw_master_step through finetune/optim.py PrlAdamW
with ``master_weights=True``) against the optimizer state of the reference's default backend.

The reference trains with DeepSpeed's bf16 ZeRO-3 optimizer (conf/base.yaml:94-95,
conf/deepspeed/deepspeed_stage3_bf16.json) or FSDP mixed precision: fp32 master weights and fp32
AdamW moments, updated from the fp32 gradients, the model's bf16 weights a rounding of the masters.
The reference here: fp32 copies of the parameters, their gradients = the bf16 gradients widened,
``clip_grad_norm_`` + ``torch.optim.AdamW(fused=True)`` on them, then ``p.copy_(master)``.  The
product must match it bit for bit — masters, both moments, step counts and the bf16 parameters —
over ragged sizes (whole 8192-element chunks, partial chunks, scalar tails), a misaligned tensor,
a skipped gradient and lr changes; and at the reference's own lr (5e-7, conf/finetune/base.yaml:35)
over 50 steps, where a pure-bf16 AdamW (the negative control) stays several bf16 ulps behind."""

import io

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(1000, 64), (3584,), (1001,), (7,), (256, 264), (3, 20000), (3, 5, 17), (8192 * 3,)]


def _bits(t):
    return t.contiguous().view(torch.int16 if t.dtype == torch.bfloat16 else torch.int32)


def _params(seed=0, std=0.1):
    g = torch.Generator(device=DEV).manual_seed(seed)
    ps = [torch.nn.Parameter((torch.randn(s, generator=g, device=DEV) * std).to(torch.bfloat16)) for s in SHAPES]
    base = (torch.randn(1025, generator=g, device=DEV) * std).to(torch.bfloat16)
    ps.append(torch.nn.Parameter(base[1:]))  # storage offset of one element: not 16-B aligned
    return ps


def _groups(ps, wd=0.01):
    return [{"params": ps[0::2], "weight_decay": wd}, {"params": ps[1::2], "weight_decay": 0.0}]


def _grads(ps, step, scale=1.0, bias=None):
    g = torch.Generator(device=DEV).manual_seed(100 + step)
    out = []
    for i, p in enumerate(ps):
        x = torch.randn(p.shape, generator=g, device=DEV) * scale
        if bias is not None:  # a consistent direction across steps (a trend the optimizer follows)
            x = x + bias[i]
        out.append(x.to(torch.bfloat16))
    return out


class Fp32MasterReference:
    """The reference default's optimizer state: fp32 masters + torch's fused fp32 AdamW."""

    def __init__(self, ps, lr):
        self.ps = ps
        self.masters = [torch.nn.Parameter(p.detach().float().clone()) for p in ps]
        self.opt = torch.optim.AdamW(_groups(self.masters), lr=lr, fused=True)

    def step(self, grads, max_norm):
        for m, g in zip(self.masters, grads):
            m.grad = None if g is None else g.float()
        norm = torch.nn.utils.clip_grad_norm_(self.masters, max_norm) if max_norm is not None else None
        self.opt.step()
        with torch.no_grad():
            for p, m in zip(self.ps, self.masters):
                p.copy_(m)
        return norm

    def set_lr(self, f):
        for g in self.opt.param_groups:
            g["lr"] *= f


def _assert_state_equal(ref, pb, opt):
    for a, m, b in zip(ref.ps, ref.masters, pb):
        assert torch.equal(_bits(a.detach()), _bits(b.detach()))
        sa, sb = ref.opt.state[m], opt.state[b]
        if not sa:
            assert "master" not in sb or float(sb["step"]) == 0
            continue
        assert sb["master"].dtype == torch.float32 and sb["exp_avg"].dtype == torch.float32
        assert torch.equal(sa["step"], sb["step"])
        assert torch.equal(_bits(m.detach()), _bits(sb["master"]))
        assert torch.equal(_bits(sa["exp_avg"]), _bits(sb["exp_avg"]))
        assert torch.equal(_bits(sa["exp_avg_sq"]), _bits(sb["exp_avg_sq"]))


@pytest.mark.parametrize("max_norm", [None, 0.3])
def test_master_step_matches_fp32_master_reference(max_norm):
    from pipelinerl_amd.finetune.optim import PrlAdamW, clip_grad_norm

    pa, pb = _params(), _params()
    ref = Fp32MasterReference(pa, lr=3e-4)
    opt = PrlAdamW(_groups(pb), lr=3e-4, master_weights=True)
    for step in range(4):
        grads = _grads(pb, step, scale=1.0 + step)
        if step == 2:
            grads[3] = None  # no gradient this step: not stepped
        for p, g in zip(pb, grads):
            p.grad = None if g is None else g.clone()
        na = ref.step(grads, max_norm)
        if max_norm is not None:
            nb = clip_grad_norm(pb, max_norm, opt)
            assert torch.equal(na, nb) and float(na) > max_norm  # fp32 norm, the clip active
        opt.step()
        ref.set_lr(0.9)  # a scheduler between steps
        for g in opt.param_groups:
            g["lr"] *= 0.9
        _assert_state_equal(ref, pb, opt)
    assert float(opt.state[pb[3]]["step"]) == 3.0


def test_master_weights_train_at_the_reference_lr():
    """lr 5e-7 (the reference's), 50 clipped steps with a consistent gradient direction: the bf16
    parameters stay bit-identical to the fp32-master reference's rounding (so within one bf16 ulp),
    while pure-bf16 AdamW — the negative control, the build's optimizer before master weights —
    drifts several ulps away: its updates are below half a bf16 ulp and round away."""
    from pipelinerl_amd.finetune.optim import PrlAdamW, clip_grad_norm

    lr, steps = 5e-7, 50
    pa, pb, pc = _params(3, 0.02), _params(3, 0.02), _params(3, 0.02)
    start = [p.detach().clone() for p in pb]
    g0 = torch.Generator(device=DEV).manual_seed(7)
    bias = [torch.randn(p.shape, generator=g0, device=DEV) * 2.0 for p in pb]
    ref = Fp32MasterReference(pa, lr=lr)
    opt = PrlAdamW(_groups(pb), lr=lr, master_weights=True)
    ctl = PrlAdamW(_groups(pc), lr=lr, master_weights=False)
    for step in range(steps):
        grads = _grads(pb, step, bias=bias)
        for ps in (pb, pc):
            for p, g in zip(ps, grads):
                p.grad = g.clone()
        ref.step(grads, 0.3)
        clip_grad_norm(pb, 0.3, opt)
        clip_grad_norm(pc, 0.3, ctl)
        opt.step()
        ctl.step()
    _assert_state_equal(ref, pb, opt)

    def ulps(x, y):  # bf16 ulps between same-sign neighbours (the weights barely move)
        return (_bits(x).int() - _bits(y).int()).abs()

    worst_ctl = max(int(ulps(a.detach(), c.detach()).max()) for a, c in zip(pa, pc))
    frac_ctl = sum(int((ulps(a.detach(), c.detach()) > 1).sum()) for a, c in zip(pa, pc)) / sum(p.numel() for p in pa)
    assert worst_ctl >= 3 and frac_ctl > 0.01, (worst_ctl, frac_ctl)  # the control fails the 1-ulp bound
    moved = sum(float((p.detach().float() - s.float()).abs().sum()) for p, s in zip(pb, start))
    moved_ctl = sum(float((p.detach().float() - s.float()).abs().sum()) for p, s in zip(pc, start))
    assert moved > 5 * moved_ctl, (moved, moved_ctl)


def _checkpoint(sd):
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def test_master_state_resumes_bit_for_bit():
    """state_dict -> torch.save -> load into a fresh PrlAdamW: the fp32 masters and moments stay
    fp32 (torch's load would round them to the parameters' bf16) and the run continues bit for bit;
    a checkpoint written without master weights resumes with masters = its bf16 parameters."""
    from pipelinerl_amd.finetune.optim import PrlAdamW

    pa, pb = _params(5), _params(5)
    ref = Fp32MasterReference(pa, lr=1e-4)
    opt = PrlAdamW(_groups(pb), lr=1e-4, master_weights=True)
    for step in range(2):
        grads = _grads(pb, step)
        for p, g in zip(pb, grads):
            p.grad = g.clone()
        ref.step(grads, None)
        opt.step()
    sd = _checkpoint(opt.state_dict())
    assert sd["state"][0]["master"].dtype == torch.float32 and sd["state"][0]["exp_avg"].dtype == torch.float32
    opt2 = PrlAdamW(_groups(pb), lr=1e-4, master_weights=True)
    opt2.load_state_dict(sd)
    for step in range(2, 4):
        grads = _grads(pb, step)
        for p, g in zip(pb, grads):
            p.grad = g.clone()
        ref.step(grads, None)
        opt2.step()
    _assert_state_equal(ref, pb, opt2)

    # from a bf16-state checkpoint (torch AdamW on the bf16 parameters)
    pc = _params(6)
    plain = torch.optim.AdamW(_groups(pc), lr=1e-4, fused=True)
    for p, g in zip(pc, _grads(pc, 0)):
        p.grad = g
    plain.step()
    opt3 = PrlAdamW(_groups(pc), lr=1e-4, master_weights=True)
    opt3.load_state_dict(_checkpoint(plain.state_dict()))
    st = opt3.state[pc[0]]
    assert st["master"].dtype == torch.float32 and torch.equal(st["master"], pc[0].detach().float())
    assert st["exp_avg"].dtype == torch.float32
    assert torch.equal(st["exp_avg"], plain.state[pc[0]]["exp_avg"].float())


def test_master_abi_rejects_bad_arguments():
    import ctypes

    from pipelinerl_amd import _native

    lib = _native.load()
    p = torch.zeros(8, device=DEV, dtype=torch.bfloat16)
    f = torch.zeros(8, device=DEV)
    s = torch.zeros((), device=DEV)
    pp = (ctypes.c_uint64 * 1)(p.data_ptr())
    fp = (ctypes.c_uint64 * 1)(f.data_ptr())
    nul = (ctypes.c_uint64 * 1)(0)
    steps = (ctypes.c_uint64 * 1)(s.data_ptr())
    n = (ctypes.c_int64 * 1)(8)
    st = torch.cuda.current_stream().cuda_stream
    args = (1e-3, 0.9, 0.999, 0.0, 1e-8, None, st)
    assert lib.prl_adamw_master_step(1, pp, pp, nul, fp, fp, steps, n, 1, *args) == 1001
    assert lib.prl_adamw_master_step(1, pp, pp, fp, fp, fp, steps, n, 7, *args) == 1002
    assert lib.prl_adamw_master_step(0, None, None, None, None, None, None, None, 1, *args) == 0
