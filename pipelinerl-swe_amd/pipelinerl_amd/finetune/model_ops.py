"""Fused HIP kernels for the trainer model's element-wise chains (csrc/model_ops.hip), patched
into an HF Qwen2 / Llama-style decoder.

``patch_model(model)`` rebinds, on that model only:
  * every ``*RMSNorm`` module (``weight``, ``variance_epsilon``)  -> prl_rmsnorm_forward / _backward
  * every ``*MLP`` with gate/up/down projections and SiLU         -> prl_swiglu_forward / _backward
  * every decoder ``nn.Linear`` (q/k/v/o, gate/up/down) and the    -> backward GEMMs through
    ``lm_head``                                                        prl_gemm (ROCm hipBLASLt)
  * the decoder module's ``apply_rotary_pos_emb``                  -> prl_rope_forward / _backward
    (q and k in one launch; outputs laid out token-major [B, T, H, D] and returned as the
    [B, H, T, D] views HF expects, so the varlen attention's ``.contiguous()`` is free)

The forward reproduces the eager chains' bf16 roundings (transformers
modeling_qwen2.py: Qwen2RMSNorm.forward, Qwen2MLP.forward, apply_rotary_pos_emb), so a patched
model's forward is bit-identical to the unpatched one; backward matches to bf16 rounding.
Inputs the kernels do not take (non-bf16, unaligned, other layouts) go through the original
HF code on the same device.
"""

from __future__ import annotations

import ctypes
import logging
import os
import sys
import types

import torch

from .. import _native, gemm

logger = logging.getLogger(__name__)

_WS: dict[tuple[int, int], torch.Tensor] = {}


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ok(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts)


class RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps: float):
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        lib = _native.load()
        _native.check(lib.prl_rmsnorm_forward(x2.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), rows, H,
                                              float(eps), _stream(x)), "prl_rmsnorm_forward")
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        H = x2.shape[1]
        dy2 = dy.reshape(-1, H).contiguous()
        dx = torch.empty_like(x2)
        dw = torch.empty_like(w)
        lib = _native.load()
        key = (x2.device.index or 0, H)
        ws = _WS.get(key)
        if ws is None:
            n = ctypes.c_size_t(0)
            _native.check(lib.prl_rmsnorm_workspace_bytes(H, ctypes.byref(n)), "prl_rmsnorm_workspace_bytes")
            ws = _WS[key] = torch.empty(n.value, dtype=torch.uint8, device=x2.device)
        _native.check(lib.prl_rmsnorm_backward(dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                               dx.data_ptr(), dw.data_ptr(), ws.data_ptr(), ws.numel(), x2.shape[0],
                                               H, _stream(x2)), "prl_rmsnorm_backward")
        return dx.view(ctx.shape), dw, None


class SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, u):
        h = torch.empty_like(g)
        _native.check(_native.load().prl_swiglu_forward(g.data_ptr(), u.data_ptr(), h.data_ptr(), g.numel(),
                                                        _stream(g)), "prl_swiglu_forward")
        ctx.save_for_backward(g, u)
        return h

    @staticmethod
    def backward(ctx, dh):
        g, u = ctx.saved_tensors
        dh = dh.contiguous()
        dg, du = torch.empty_like(g), torch.empty_like(u)
        _native.check(_native.load().prl_swiglu_backward(dh.data_ptr(), g.data_ptr(), u.data_ptr(), dg.data_ptr(),
                                                         du.data_ptr(), g.numel(), _stream(g)), "prl_swiglu_backward")
        return dg, du


class RopeFn(torch.autograd.Function):
    """q [B, Hq, T, D] / k [B, Hkv, T, D] given as views of token-major [B, T, H, D] memory."""

    @staticmethod
    def forward(ctx, q, k, cos, sin):
        B, hq, T, D = q.shape
        hkv = k.shape[1]
        qt, kt = q.transpose(1, 2), k.transpose(1, 2)  # contiguous [B, T, H, D]
        qo, ko = torch.empty_like(qt), torch.empty_like(kt)
        _native.check(_native.load().prl_rope_forward(qt.data_ptr(), kt.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                                                      qo.data_ptr(), ko.data_ptr(), B * T, hq, hkv, D, _stream(q)),
                      "prl_rope_forward")
        ctx.save_for_backward(cos, sin)
        ctx.dims = (B, T, hq, hkv, D)
        return qo.transpose(1, 2), ko.transpose(1, 2)

    @staticmethod
    def backward(ctx, dqo, dko):
        cos, sin = ctx.saved_tensors
        B, T, hq, hkv, D = ctx.dims
        dqt = dqo.transpose(1, 2).contiguous() if dqo is not None else torch.zeros((B, T, hq, D), dtype=cos.dtype,
                                                                                    device=cos.device)
        dkt = dko.transpose(1, 2).contiguous() if dko is not None else torch.zeros((B, T, hkv, D), dtype=cos.dtype,
                                                                                    device=cos.device)
        dq, dk = torch.empty_like(dqt), torch.empty_like(dkt)
        _native.check(_native.load().prl_rope_backward(dqt.data_ptr(), dkt.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                                                       dq.data_ptr(), dk.data_ptr(), B * T, hq, hkv, D,
                                                       _stream(cos)), "prl_rope_backward")
        return dq.transpose(1, 2), dk.transpose(1, 2), None, None


class PrlLinearFn(torch.autograd.Function):
    """F.linear whose GEMMs run through prl_gemm (the ROCm hipBLASLt, include/prl_gemm.h).

    Backward (dX = dY W, dW = dY^T X) always: 1.3-2.9x faster weight gradients and 1.05-1.15x
    faster input gradients than torch's bundled library with the library heuristic alone
    (tools/gemm_sweep.py, profiles/r01_gemm_sweep.jsonl), more with the swept solutions of
    gemm_solutions.json.  Forward only where gemm_solutions.json routes the shape (a swept solution,
    or the heuristic where it measured faster than torch; bias in the GEMM epilogue); elsewhere
    torch's F.linear, which the heuristic does not generally beat.  bf16 only."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        T = x.numel() // x.shape[-1]
        sol = gemm.solution_for("fwd", T, w.shape[0], w.shape[1])
        if sol is not None and (b is None or (b.dtype == torch.bfloat16 and b.is_contiguous())):
            return gemm.linear_fwd(x, w, b, solution=sol)
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy if dy.is_contiguous() else dy.contiguous()
        dx = gemm.linear_dgrad(dy, w) if ctx.needs_input_grad[0] else None
        dw = gemm.linear_wgrad(dy, x) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0, dtype=torch.float32).to(dy.dtype)
        return dx, dw, db


def _linear_ok(x, w) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
            and x.dim() >= 2 and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0)


def _prl_linear_forward(self, x):
    if _linear_ok(x, self.weight):
        return PrlLinearFn.apply(x, self.weight, self.bias)
    return torch.nn.functional.linear(x, self.weight, self.bias)


# ------------------------------------------------------------------------------------------
# patching

def _rmsnorm_forward(self, hidden_states):
    w = self.weight
    H = hidden_states.shape[-1]
    if _ok(hidden_states, w) and H % 8 == 0 and H <= 5120:
        return RMSNormFn.apply(hidden_states, w, self.variance_epsilon)
    return self._prl_orig_forward(hidden_states)


def _mlp_forward(self, x):
    g, u = self.gate_proj(x), self.up_proj(x)
    if _ok(g, u) and g.numel() % 8 == 0:
        return self.down_proj(SwiGLUFn.apply(g, u))
    return self.down_proj(self.act_fn(g) * u)


def _rope_ok(q, k, cos, sin) -> bool:
    if q.dim() != 4 or k.dim() != 4 or cos.dim() != 3:
        return False
    qt, kt = q.transpose(1, 2), k.transpose(1, 2)
    B, hq, T, D = q.shape
    return (_ok(qt, kt, cos, sin) and D % 8 == 0 and cos.shape == (B, T, D) and sin.shape == (B, T, D)
            and k.shape[0] == B and k.shape[2] == T and k.shape[3] == D)


def _make_rope(orig):
    def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1):
        if unsqueeze_dim == 1 and _rope_ok(q, k, cos, sin):
            return RopeFn.apply(q, k, cos, sin)
        return orig(q, k, cos, sin, unsqueeze_dim)

    apply_rotary_pos_emb._prl_fused = True
    apply_rotary_pos_emb._prl_orig = orig
    return apply_rotary_pos_emb


_SILU = ("SiLU", "SiLUActivation")  # torch.nn.SiLU / transformers ACT2FN["silu"] (both F.silu)


def patch_model(model) -> dict:
    """Patch ``model`` in place; returns counts of patched modules."""
    _native.load()  # fail loudly here, not on the first forward
    if any(p.is_cuda for p in model.parameters()):
        gemm.library()  # opens the ROCm hipBLASLt now: raises if it cannot
    n_norm = n_mlp = n_linear = 0
    mods = set()
    for m in model.modules():
        name = type(m).__name__
        if name.endswith("RMSNorm") and hasattr(m, "weight") and hasattr(m, "variance_epsilon"):
            if not hasattr(m, "_prl_orig_forward"):
                m._prl_orig_forward = m.forward
                m.forward = types.MethodType(_rmsnorm_forward, m)
            n_norm += 1
        elif (name.endswith("MLP") and all(hasattr(m, a) for a in ("gate_proj", "up_proj", "down_proj"))
              and type(getattr(m, "act_fn", None)).__name__ in _SILU):
            m.forward = types.MethodType(_mlp_forward, m)
            n_mlp += 1
        elif name.endswith("Attention"):
            mods.add(type(m).__module__)
    # PRL_LINEAR_GEMM=torch keeps torch's own linear layers (A/B measurements)
    for mname, lin in (model.named_modules() if os.environ.get("PRL_LINEAR_GEMM", "") != "torch" else ()):
        if isinstance(lin, torch.nn.Linear) and (".layers." in f".{mname}" or mname.endswith("lm_head")):
            if not getattr(lin, "_prl_linear", False):
                lin.forward = types.MethodType(_prl_linear_forward, lin)
                lin._prl_linear = True
            n_linear += 1
    n_rope = 0
    for modname in mods:
        mod = sys.modules.get(modname)
        f = getattr(mod, "apply_rotary_pos_emb", None)
        if f is not None and not getattr(f, "_prl_fused", False):
            mod.apply_rotary_pos_emb = _make_rope(f)
        if f is not None:
            n_rope += 1
    counts = {"rmsnorm": n_norm, "swiglu_mlp": n_mlp, "rope_modules": n_rope, "prl_linear": n_linear}
    logger.info(f"fused model ops patched: {counts}")
    return counts
