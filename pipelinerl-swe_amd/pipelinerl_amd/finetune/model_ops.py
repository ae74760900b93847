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
import inspect
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
        ws = _norm_ws(x2.device, H)
        _native.check(lib.prl_rmsnorm_backward(dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                               dx.data_ptr(), dw.data_ptr(), ws.data_ptr(), ws.numel(), x2.shape[0],
                                               H, _stream(x2)), "prl_rmsnorm_backward")
        return dx.view(ctx.shape), dw, None


def _norm_ws(dev: torch.device, H: int) -> torch.Tensor:
    key = (dev.index or 0, H)
    ws = _WS.get(key)
    if ws is None:
        n = ctypes.c_size_t(0)
        _native.check(_native.load().prl_rmsnorm_workspace_bytes(H, ctypes.byref(n)), "prl_rmsnorm_workspace_bytes")
        ws = _WS[key] = torch.empty(n.value, dtype=torch.uint8, device=dev)
    return ws


class AddRMSNormFn(torch.autograd.Function):
    """h = residual + x and y = rmsnorm(h) in one pass (the decoder's residual add fused with the
    norm that reads it); returns (h, y).  Backward: the gradient reaching h through the residual
    stream is added inside the norm's backward kernel, so no separate add runs in either
    direction.  Forward bit-identical to the eager `residual + x` then Qwen2RMSNorm."""

    @staticmethod
    def forward(ctx, residual, x, w, eps: float):
        H = x.shape[-1]
        x2, r2 = x.reshape(-1, H), residual.reshape(-1, H)
        rows = x2.shape[0]
        h, y = torch.empty_like(x2), torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        _native.check(_native.load().prl_add_rmsnorm_forward(r2.data_ptr(), x2.data_ptr(), w.data_ptr(), h.data_ptr(),
                                                             y.data_ptr(), rstd.data_ptr(), rows, H, float(eps),
                                                             _stream(x)), "prl_add_rmsnorm_forward")
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(h, w, rstd)
        ctx.shape = x.shape
        return h.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, dh, dy):
        h, w, rstd = ctx.saved_tensors
        H = h.shape[1]
        if dy is None:
            return dh, dh, None, None
        dy2 = dy.reshape(-1, H).contiguous()
        dx = torch.empty_like(h)
        dw = torch.empty_like(w)
        ws = _norm_ws(h.device, H)
        lib = _native.load()
        if dh is None:
            rc = lib.prl_rmsnorm_backward(dy2.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                          dw.data_ptr(), ws.data_ptr(), ws.numel(), h.shape[0], H, _stream(h))
        else:
            dh2 = dh.reshape(-1, H).contiguous()
            rc = lib.prl_add_rmsnorm_backward(dy2.data_ptr(), dh2.data_ptr(), h.data_ptr(), w.data_ptr(),
                                              rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(), ws.data_ptr(), ws.numel(),
                                              h.shape[0], H, _stream(h))
        _native.check(rc, "prl_add_rmsnorm_backward")
        dx = dx.view(ctx.shape)
        return dx, dx, dw, None


def _chunk_counter(t: torch.Tensor) -> int:
    """The phased SwiGLU kernels' chunk counter for ``t``'s device and current stream (caller-owned
    scratch, include/prl_hip.h: the library zeroes it per launch)."""
    return _native.stream_scratch("swiglu_ctr", 16, t.device, _stream(t)).data_ptr()


class SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, u):
        h = torch.empty_like(g)
        _native.check(_native.load().prl_swiglu_forward(g.data_ptr(), u.data_ptr(), h.data_ptr(), g.numel(),
                                                        _chunk_counter(g), _stream(g)), "prl_swiglu_forward")
        ctx.save_for_backward(g, u)
        return h

    @staticmethod
    def backward(ctx, dh):
        g, u = ctx.saved_tensors
        dh = dh.contiguous()
        dg, du = torch.empty_like(g), torch.empty_like(u)
        _native.check(_native.load().prl_swiglu_backward(dh.data_ptr(), g.data_ptr(), u.data_ptr(), dg.data_ptr(),
                                                         du.data_ptr(), g.numel(), _chunk_counter(g), _stream(g)),
                      "prl_swiglu_backward")
        return dg, du


class RopeFn(torch.autograd.Function):
    """q [B, Hq, T, D] / k [B, Hkv, T, D] given as views of token-major [B, T, H, D] memory."""

    @staticmethod
    def forward(ctx, q, k, cos, sin):
        B, hq, T, D = q.shape
        hkv = k.shape[1]
        qt, kt = q.transpose(1, 2), k.transpose(1, 2)  # [B, T, H, D]: contiguous, or token-strided (fused qkv)
        qo = torch.empty((B, T, hq, D), dtype=q.dtype, device=q.device)
        ko = torch.empty((B, T, hkv, D), dtype=k.dtype, device=k.device)
        _native.check(_native.load().prl_rope_forward_strided(qt.data_ptr(), kt.data_ptr(), cos.data_ptr(),
                                                              sin.data_ptr(), qo.data_ptr(), ko.data_ptr(), B * T, hq,
                                                              hkv, D, qt.stride(1), kt.stride(1), _stream(q)),
                      "prl_rope_forward_strided")
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


# Weight-gradient accumulation in the wgrad GEMM's epilogue: when a weight already holds a
# gradient (the micro-batches after the first of an optimizer step, or the DP loop's gradient
# buckets, which are never None), dW = dY^T X is added into it by the GEMM (beta = 1) instead of
# being written to a new tensor that autograd's AccumulateGrad then adds with a separate bf16 add
# kernel (a [N, K] read-read-write per weight per micro-batch: ~2 % of a 7B C3 step).  The sum is
# rounded to bf16 once instead of twice.  Not used when a post-accumulate hook must see the
# gradient (an armed GradBuckets, any other hook) or under FSDP (shard_model switches it off):
# there autograd accumulates as before.
_FUSE_GRAD_ACCUM = True


def disable_fused_grad_accumulation() -> None:
    global _FUSE_GRAD_ACCUM
    _FUSE_GRAD_ACCUM = False


def _accum_target(w):
    if not _FUSE_GRAD_ACCUM or not isinstance(w, torch.nn.Parameter):
        return None
    g = w.grad
    if g is None or g.dtype != w.dtype or g.shape != w.shape or not g.is_contiguous():
        return None
    hooks = w._post_accumulate_grad_hooks
    if hooks:
        owner = getattr(w, "_prl_grad_buckets", None)  # finetune/grad_sync.py: fires only when armed
        if owner is None or owner.armed or len(hooks) != 1:
            return None
    return g


def _wgrad(dy, x, w):
    """dW for parameter w, or None after adding it into w.grad in the GEMM (see above)."""
    g = _accum_target(w)
    if g is not None:
        gemm.linear_wgrad(dy, x, out=g, accumulate=True)
        return None
    return gemm.linear_wgrad(dy, x)


# Fused gate/up projection: one GEMM over the concatenated [2 I, H] weight instead of two over
# [I, H] (7B at 8 192 tokens through prl_gemm: forward 1.82 -> 1.53 ms, dgrad 1.93 -> 1.65 ms,
# wgrad 1.66 -> 1.58 ms per layer, tools/fused_proj_bench.py [round 1-3 tool, in git history], profiles/r02_fused_proj_bench.jsonl).  The weights stay separate Parameters; the
# concatenation is cached and rebuilt only when a member's version counter moves (once per
# optimizer step).  Off under FSDP (shard_model) and with PRL_FUSED_GATE_UP=0 (A/B).
_FUSED_GATE_UP = os.environ.get("PRL_FUSED_GATE_UP", "1") != "0"
# Used up to this many tokens per micro-batch: the fused [2 I, H] shape runs the library heuristic
# (no swept solution), which wins at C3's <= 12 000-token micro-batches (7B step 1539 -> 1527 ms,
# profiles/r02_fused_gate_up_ab.jsonl) and loses at 65 536 (1.5B C2 step 1211 -> 1225 ms)
_FUSED_GATE_UP_MAX_ROWS = int(os.environ.get("PRL_FUSED_GATE_UP_MAX_ROWS", "12288"))


def disable_fused_projections() -> None:
    global _FUSED_GATE_UP, _FUSED_QKV
    _FUSED_GATE_UP = _FUSED_QKV = False


# Bumped by the build's writers that change weights through raw pointers (PrlAdamW.step and
# HipFlatPacker.unflatten; both also move the version counters): a second key of the fused-weight
# caches beside the version counters, which a write through ``p.data`` or a raw pointer does not
# move.  In-place torch writes (load_state_dict, torch's optimizers, ``copy_`` under no_grad) move
# the version counters and need no call; any new raw-pointer or ``.data`` writer must call
# weights_written().
_WEIGHT_EPOCH = [0]


def weights_written() -> None:
    """Invalidate every fused-weight cache (call after writing parameters outside autograd)."""
    _WEIGHT_EPOCH[0] += 1


def _adjacent_view(ws) -> torch.Tensor | None:
    """``ws`` as ONE tensor, without a copy, when they lie back to back in one storage with matching
    trailing shapes — the case for gate_proj / up_proj once the parameters are re-homed into the
    weight broadcast's flat layout (weight_update.py, snapshot="zero_copy": consecutive
    named_parameters, 16-B aligned, and I x H is a multiple of 8) — else None."""
    w0 = ws[0]
    try:
        base = w0.untyped_storage().data_ptr()
    except Exception:  # noqa: BLE001
        return None
    off = w0.storage_offset()
    for w in ws:
        if (not w.is_contiguous() or w.dtype != w0.dtype or w.device != w0.device or w.shape[1:] != w0.shape[1:]
                or w.untyped_storage().data_ptr() != base or w.storage_offset() != off):
            return None
        off += w.numel()
    rows = sum(int(w.shape[0]) for w in ws)
    return w0.detach().as_strided((rows,) + tuple(w0.shape[1:]), w0.stride(), w0.storage_offset())


def _fused_weight(holder, ws, slot: str = "_prl_fused_w") -> torch.Tensor:
    """cat(ws): a view when the members are adjacent in memory (nothing cached: it always reads the
    current weights), else a copy cached on the module ``holder`` (so it lives and dies with the
    model), rebuilt when a member's version counter or storage changes, or when weights_written()
    was called."""
    view = _adjacent_view(ws)
    if view is not None:
        holder.__dict__.pop(slot, None)  # a copy made before the parameters were re-homed
        return view
    ver = (_WEIGHT_EPOCH[0],) + tuple(w._version for w in ws) + tuple(w.data_ptr() for w in ws)
    hit = holder.__dict__.get(slot)
    if hit is not None and hit[0] == ver:
        return hit[1]
    with torch.no_grad():
        wf = torch.cat([w.detach() for w in ws])
    holder.__dict__[slot] = (ver, wf)
    return wf


def _adjacent_grads(gs) -> torch.Tensor | None:
    """The [sum N, K] view over gradient tensors that sit back to back in one storage, else None."""
    if any(g is None for g in gs):
        return None
    K = gs[0].shape[1]
    for a, b in zip(gs, gs[1:]):
        if (b.untyped_storage().data_ptr() != a.untyped_storage().data_ptr() or b.shape[1] != K
                or b.storage_offset() != a.storage_offset() + a.numel()):
            return None
    return torch.as_strided(gs[0], (sum(g.shape[0] for g in gs), K), (K, 1))


def _wgrad_group(dy, x, params):
    """Weight gradients of layers fused along N (dW = dY^T X, one GEMM): added in the GEMM into
    their .grad when those sit back to back (and no hook is due), else returned as row blocks of
    one [sum N, K] tensor for autograd to accumulate."""
    targets = [_accum_target(p) for p in params]
    if all(t is not None for t in targets):
        G = _adjacent_grads(targets)
        if G is not None and G.data_ptr() % 16 == 0:
            gemm.linear_wgrad(dy, x, out=G, accumulate=True)
            return [None] * len(params)
    dW = gemm.linear_wgrad(dy, x)
    if (_FUSE_GRAD_ACCUM and all(isinstance(p, torch.nn.Parameter) and p.requires_grad and p.grad is None
                                 and not p._post_accumulate_grad_hooks for p in params)):
        # the step's first micro-batch: the gradients become row blocks of dW, so the next
        # micro-batches find them back to back (what AccumulateGrad would store: dW itself)
        a = 0
        for p in params:
            p.grad = dW[a:a + p.shape[0]]
            a += p.shape[0]
        return [None] * len(params)
    out, a = [], 0
    for p in params:  # a frozen member gets no gradient (its block is dropped)
        out.append(dW[a:a + p.shape[0]] if p.requires_grad else None)
        a += p.shape[0]
    return out


class GateUpSwiGLUFn(torch.autograd.Function):
    """h = bf16(silu(x Wg^T)) * (x Wu^T) with gate and up as one GEMM over cat(Wg, Wu) (bias-free
    layers, Qwen2MLP): the GEMM output [T, 2 I] feeds the row-strided SwiGLU kernel; the backward
    writes dgate / dup into one [T, 2 I] buffer for one dgrad and one wgrad GEMM.  Saves x and
    the GEMM output (what the separate form saves: x, gate, up)."""

    @staticmethod
    def forward(ctx, x, wg, wu, holder):
        I, H = wg.shape
        wf = _fused_weight(holder, (wg, wu))
        x2 = x.reshape(-1, H)
        rows = x2.shape[0]
        gu = gemm.linear_fwd(x2, wf, solution=_fused_solution("fwd", rows, 2 * I, H))
        h = torch.empty((rows, I), dtype=x.dtype, device=x.device)
        _native.check(_native.load().prl_swiglu_forward_rows(gu.data_ptr(), gu.data_ptr() + 2 * I, h.data_ptr(), rows,
                                                             I, 2 * I, 2 * I, I, _stream(x)),
                      "prl_swiglu_forward_rows")
        ctx.save_for_backward(x2, gu, wf)
        ctx.params = (wg, wu)
        ctx.shape = x.shape
        return h.view(*x.shape[:-1], I)

    @staticmethod
    def backward(ctx, dh):
        x2, gu, wf = ctx.saved_tensors
        wg, wu = ctx.params
        I = wg.shape[0]
        rows = x2.shape[0]
        dh = dh.reshape(rows, I)
        dh = dh if dh.is_contiguous() else dh.contiguous()
        dgu = torch.empty_like(gu)
        _native.check(_native.load().prl_swiglu_backward_rows(dh.data_ptr(), gu.data_ptr(), gu.data_ptr() + 2 * I,
                                                              dgu.data_ptr(), dgu.data_ptr() + 2 * I, rows, I, I,
                                                              2 * I, 2 * I, 2 * I, 2 * I, _stream(dh)),
                      "prl_swiglu_backward_rows")
        dx = gemm.linear_dgrad(dgu, wf) if ctx.needs_input_grad[0] else None
        dwg = dwu = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dwg, dwu = _wgrad_group(dgu, x2, (wg, wu))
        return (dx.view(ctx.shape) if dx is not None else None), dwg, dwu, None


# Fused q/k/v projection: one GEMM over cat(Wq, Wk, Wv) (+ the concatenated bias in the epilogue)
# instead of three (7B 8 k tokens 0.97 -> 0.75 ms per layer fwd + dgrad + wgrad alone,
# profiles/r02_fused_proj_bench.jsonl).  q / k / v leave as column ranges of the [T, Nq + 2 Nkv]
# output (RoPE reads them strided); the backward concatenates their gradients for one dgrad and one
# wgrad GEMM.  OFF by default (PRL_FUSED_QKV=1 turns it on): in the C3 7B step it cut kernel time
# 1.1 % but the step's wall time rose 3.3 % (GPU idle between kernels, not yet explained;
# profiles/r02_fused_qkv_ab.jsonl, profiles/r02_c3_qkv_kernel_stats_*.csv); +0.4 % at C2.
_FUSED_QKV = os.environ.get("PRL_FUSED_QKV", "0") == "1"


class QKVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, holder, *wb):
        ws, bs = wb[0::2], wb[1::2]
        H = ws[0].shape[1]
        ns = [w.shape[0] for w in ws]
        wf = _fused_weight(holder, ws)
        has_bias = all(b is not None for b in bs)
        bf = _fused_weight(holder, bs, "_prl_fused_b") if has_bias else None
        x2 = x.reshape(-1, H)
        rows = x2.shape[0]
        y = gemm.linear_fwd(x2, wf, bf, solution=_fused_solution("fwd", rows, sum(ns), H))
        ctx.save_for_backward(x2, wf)
        ctx.params, ctx.ns, ctx.has_bias, ctx.shape = ws, ns, tuple(b is not None for b in bs), x.shape
        ctx.set_materialize_grads(False)
        outs, a = [], 0
        for n in ns:
            outs.append(y[:, a:a + n].view(*x.shape[:-1], n))
            a += n
        return tuple(outs)

    @staticmethod
    def backward(ctx, *dys):
        x2, wf = ctx.saved_tensors
        rows = x2.shape[0]
        parts = [d.reshape(rows, n) if d is not None else torch.zeros((rows, n), dtype=x2.dtype, device=x2.device)
                 for d, n in zip(dys, ctx.ns)]
        dy = torch.cat(parts, dim=1)
        dx = gemm.linear_dgrad(dy, wf).view(ctx.shape) if ctx.needs_input_grad[0] else None
        dws = _wgrad_group(dy, x2, ctx.params) if any(ctx.needs_input_grad[2::2]) else [None] * len(ctx.ns)
        dbs = [None] * len(ctx.ns)
        if any(ctx.has_bias) and any(ctx.needs_input_grad[3::2]):
            db = dy.sum(0, dtype=torch.float32).to(dy.dtype)
            a = 0
            for i, n in enumerate(ctx.ns):
                dbs[i] = db[a:a + n] if ctx.has_bias[i] else None
                a += n
        grads = [dx, None]
        for dw, db in zip(dws, dbs):
            grads += [dw, db]
        return tuple(grads)


def _fused_solution(pas: str, T: int, N: int, K: int) -> int:
    sol = gemm.solution_for(pas, T, N, K)
    return -1 if sol is None else sol  # -1: the ROCm 7.2 library heuristic (measured, fused_proj_bench)


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
        ctx.param = w  # the Parameter itself (its .grad: the fused accumulation)
        ctx.has_bias = b is not None
        return _fwd_gemm(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy if dy.is_contiguous() else dy.contiguous()
        dx = gemm.linear_dgrad(dy, w) if ctx.needs_input_grad[0] else None
        dw = _wgrad(dy, x, ctx.param) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0, dtype=torch.float32).to(dy.dtype)
        return dx, dw, db


class SharedInputLinearFn(torch.autograd.Function):
    """Several linear layers on ONE input (q/k/v, gate/up): each forward as PrlLinearFn's; in the
    backward the input gradients are summed in the dgrad GEMMs' epilogue (dX = dY0 W0, then
    dX += dYi Wi with beta = 1) instead of by autograd's separate bf16 add kernels (one
    [T, K] read-read-write per extra layer).  Arguments: x, w0, b0, w1, b1, ..."""

    @staticmethod
    def forward(ctx, x, *wb):
        ws, bs = wb[0::2], wb[1::2]
        ctx.set_materialize_grads(False)  # an unused output's gradient stays None: no GEMMs for it
        ctx.save_for_backward(x, *ws)
        ctx.params = ws
        ctx.has_bias = tuple(b is not None for b in bs)
        return tuple(_fwd_gemm(x, w, b) for w, b in zip(ws, bs))

    @staticmethod
    def backward(ctx, *dys):
        x, *ws = ctx.saved_tensors
        grads = [None]
        dx = None
        for i, (dy, w) in enumerate(zip(dys, ws)):
            if dy is None:
                grads += [None, None]
                continue
            dy = dy if dy.is_contiguous() else dy.contiguous()
            if ctx.needs_input_grad[0]:
                dx = gemm.linear_dgrad(dy, w) if dx is None else gemm.linear_dgrad(dy, w, out=dx, accumulate=True)
            dw = _wgrad(dy, x, ctx.params[i]) if ctx.needs_input_grad[1 + 2 * i] else None
            db = None
            if ctx.has_bias[i] and ctx.needs_input_grad[2 + 2 * i]:
                db = dy.reshape(-1, dy.shape[-1]).sum(0, dtype=torch.float32).to(dy.dtype)
            grads += [dw, db]
        grads[0] = dx
        return tuple(grads)


def _fwd_gemm(x, w, b):
    T = x.numel() // x.shape[-1]
    sol = gemm.solution_for("fwd", T, w.shape[0], w.shape[1])
    if sol is not None and (b is None or (b.dtype == torch.bfloat16 and b.is_contiguous())):
        return gemm.linear_fwd(x, w, b, solution=sol)
    return torch.nn.functional.linear(x, w, b)


class _Group:
    """Linear layers that read the same input (an attention's q/k/v): the first call with an
    input computes all of them in one SharedInputLinearFn and hands the others their outputs
    when they are called with that same tensor."""

    def __init__(self, mods):
        self.mods = list(mods)
        self.x = None
        self.out: dict[int, torch.Tensor] = {}

    def __call__(self, lin, x):
        if self.x is x and id(lin) in self.out:
            y = self.out.pop(id(lin))
            if not self.out:
                self.x = None
            return y
        if not all(_linear_ok(x, m.weight) for m in self.mods):
            return None
        wb = [t for m in self.mods for t in (m.weight, m.bias)]
        biases = [m.bias for m in self.mods]
        if (_FUSED_QKV and x.data_ptr() % 16 == 0 and
                (all(b is None for b in biases) or all(b is not None and b.dtype == torch.bfloat16 for b in biases))):
            ys = QKVFn.apply(x, self, *wb)
        else:
            ys = SharedInputLinearFn.apply(x, *wb)
        self.x = x
        self.out = {id(m): y for m, y in zip(self.mods, ys) if m is not lin}
        return ys[self.mods.index(lin)]


def _linear_ok(x, w) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
            and x.dim() >= 2 and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0)


def _prl_linear_forward(self, x):
    grp = self.__dict__.get("_prl_group")
    if grp is not None:
        y = grp(self, x)
        if y is not None:
            return y
    if _linear_ok(x, self.weight):
        return PrlLinearFn.apply(x, self.weight, self.bias)
    return torch.nn.functional.linear(x, self.weight, self.bias)


# ------------------------------------------------------------------------------------------
# patching

def _rmsnorm_forward(self, hidden_states):
    pend = self.__dict__.get("_prl_pending")
    if pend is not None:  # the previous decoder layer already normalised this tensor (fused add)
        self.__dict__["_prl_pending"] = None
        if pend[0] is hidden_states:
            return pend[1]
    w = self.weight
    H = hidden_states.shape[-1]
    if _ok(hidden_states, w) and H % 8 == 0 and H <= 5120:
        return RMSNormFn.apply(hidden_states, w, self.variance_epsilon)
    return self._prl_orig_forward(hidden_states)


def _mlp_forward(self, x):
    gp, up = self.gate_proj, self.up_proj
    if (_FUSED_GATE_UP and x.numel() // max(1, x.shape[-1]) <= _FUSED_GATE_UP_MAX_ROWS
            and getattr(gp, "_prl_linear", False) and getattr(up, "_prl_linear", False)
            and gp.bias is None and up.bias is None and gp.weight.shape == up.weight.shape
            and gp.weight.shape[0] % 8 == 0 and _linear_ok(x, gp.weight) and _linear_ok(x, up.weight)
            and x.data_ptr() % 16 == 0):
        return self.down_proj(GateUpSwiGLUFn.apply(x, gp.weight, up.weight, self))
    if getattr(gp, "_prl_linear", False) and getattr(up, "_prl_linear", False) and _linear_ok(x, gp.weight) \
            and _linear_ok(x, up.weight):
        g, u = SharedInputLinearFn.apply(x, gp.weight, gp.bias, up.weight, up.bias)
    else:
        g, u = gp(x), up(x)
    if _ok(g, u) and g.numel() % 8 == 0:
        return self.down_proj(SwiGLUFn.apply(g, u))
    return self.down_proj(self.act_fn(g) * u)


def _add_norm_ok(norm, residual, x) -> bool:
    w = getattr(norm, "weight", None)
    H = x.shape[-1]
    return (getattr(norm, "_prl_orig_forward", None) is not None and w is not None
            and not hasattr(w, "_local_tensor") and _ok(residual, x, w) and residual.shape == x.shape
            and H % 8 == 0 and H <= 5120)


def _add_norm(norm, residual, x):
    """(residual + x, norm(residual + x)) through AddRMSNormFn, or the eager pair."""
    if _add_norm_ok(norm, residual, x):
        return AddRMSNormFn.apply(residual, x, norm.weight, norm.variance_epsilon)
    h = residual + x
    return h, norm(h)


def _layer_call_args(layer, hidden_states, args, kwargs) -> tuple[dict, bool]:
    """Map a decoder-layer call onto keyword arguments for its self_attn, under either
    transformers layer contract: 5.x ``forward(hidden_states, attention_mask, position_ids,
    past_key_values, use_cache, position_embeddings, **kw) -> Tensor`` or 4.x (the reference pins
    4.51.1, pyproject.toml:20) ``forward(hidden_states, attention_mask, position_ids,
    past_key_value, output_attentions, use_cache, cache_position, position_embeddings, **kw) ->
    tuple`` (Qwen2Model takes ``layer_outputs[0]``; gradient checkpointing passes them
    positionally).  Returns (self_attn kwargs, whether the layer returns a tuple)."""
    sig = layer.__dict__.get("_prl_sig")
    if sig is None:
        sig = inspect.signature(layer.__dict__["_prl_orig_forward"])
        layer.__dict__["_prl_sig"] = sig
    bound = sig.bind(hidden_states, *args, **kwargs).arguments
    attn_kw: dict = {}
    for name, v in bound.items():
        if name == "hidden_states":
            continue
        if sig.parameters[name].kind is inspect.Parameter.VAR_KEYWORD:
            attn_kw.update(v)
        else:
            attn_kw[name] = v
    return attn_kw, "output_attentions" in sig.parameters


def _decoder_forward(self, hidden_states, *args, **kwargs):
    """transformers Qwen2DecoderLayer.forward with both residual adds fused into the norms that
    read their results: `residual + attn` into post_attention_layernorm, and `residual + mlp`
    into the NEXT layer's input_layernorm (or the final norm), whose output is handed over via
    that norm module (`_prl_pending`, consumed by the next call with this very tensor).  The
    cross-layer hand-over is skipped under gradient checkpointing and for sharded (FSDP) norm
    weights, which the next layer only gathers in its own forward.  Returns what the installed
    transformers' layer returns (a tensor on 5.x, a tuple on 4.x)."""
    attn_kw, tuple_out = _layer_call_args(self, hidden_states, args, kwargs)
    n1 = self.input_layernorm(hidden_states)
    a, attn_w = self.self_attn(hidden_states=n1, **attn_kw)
    h1, n2 = _add_norm(self.post_attention_layernorm, hidden_states, a)
    m = self.mlp(n2)
    nxt = self.__dict__.get("_prl_next_norm")
    if nxt is not None and not (self.training and getattr(self, "gradient_checkpointing", False)) \
            and _add_norm_ok(nxt, h1, m):
        h2, n_next = AddRMSNormFn.apply(h1, m, nxt.weight, nxt.variance_epsilon)
        nxt.__dict__["_prl_pending"] = (h2, n_next)
    else:
        h2 = h1 + m
    if not tuple_out:
        return h2
    return (h2, attn_w) if attn_kw.get("output_attentions") else (h2,)


def _token_major(t) -> bool:
    """t [B, T, H, D]: contiguous, or rows of a wider token-major buffer (a fused-qkv column range:
    stride(1) = the buffer's row, H and D dense)."""
    B, T, H, D = t.shape
    return (t.is_cuda and t.dtype == torch.bfloat16 and t.stride(3) == 1 and t.stride(2) == D
            and t.stride(1) >= H * D and t.stride(1) % 4 == 0 and (B == 1 or t.stride(0) == T * t.stride(1))
            and t.data_ptr() % 8 == 0)


def _rope_ok(q, k, cos, sin) -> bool:
    if q.dim() != 4 or k.dim() != 4 or cos.dim() != 3:
        return False
    qt, kt = q.transpose(1, 2), k.transpose(1, 2)
    B, hq, T, D = q.shape
    return (_token_major(qt) and _token_major(kt) and _ok(cos, sin) and D % 8 == 0 and cos.shape == (B, T, D)
            and sin.shape == (B, T, D) and k.shape[0] == B and k.shape[2] == T and k.shape[3] == D)


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
            # gate and up gradients side by side in gradient buckets (finetune/grad_sync.py), in
            # the fused GEMM's row order, so GateUpSwiGLUFn can add into both in one wgrad GEMM
            m.up_proj.weight._prl_follows = m.gate_proj.weight
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
    # q/k/v of each attention share their input: one SharedInputLinearFn (dgrads summed in the
    # GEMM epilogue).  PRL_QKV_GROUP=0 keeps them separate (A/B measurements)
    n_group = 0
    if n_linear and os.environ.get("PRL_QKV_GROUP", "1") != "0":
        for m in model.modules():
            lins = [getattr(m, a, None) for a in ("q_proj", "k_proj", "v_proj")]
            if type(m).__name__.endswith("Attention") and all(getattr(l, "_prl_linear", False) for l in lins):
                if "_prl_group" not in lins[0].__dict__:
                    g = _Group(lins)
                    for l in lins:
                        l.__dict__["_prl_group"] = g
                    # q, k, v gradients back to back in gradient buckets: rows of the fused GEMM
                    lins[1].weight._prl_follows = lins[0].weight
                    lins[2].weight._prl_follows = lins[1].weight
                n_group += 1
    # decoder layers (input_layernorm / self_attn / post_attention_layernorm / mlp, Qwen2 / Llama
    # style): residual adds fused into the norms
    n_addnorm = 0
    inner = getattr(model, "model", model)
    layers = list(getattr(inner, "layers", []))
    final = getattr(inner, "norm", None)
    if layers and all(type(l).__name__.endswith("DecoderLayer") and all(
            hasattr(l, a) for a in ("input_layernorm", "self_attn", "post_attention_layernorm", "mlp"))
            and hasattr(l.post_attention_layernorm, "_prl_orig_forward") for l in layers):
        for i, l in enumerate(layers):
            nxt = layers[i + 1].input_layernorm if i + 1 < len(layers) else final
            l.__dict__["_prl_next_norm"] = nxt if hasattr(nxt, "_prl_orig_forward") else None
            if "_prl_orig_forward" not in l.__dict__:
                l.__dict__["_prl_orig_forward"] = l.forward
                l.forward = types.MethodType(_decoder_forward, l)
            n_addnorm += 1
    n_rope = 0
    for modname in mods:
        mod = sys.modules.get(modname)
        f = getattr(mod, "apply_rotary_pos_emb", None)
        if f is not None and not getattr(f, "_prl_fused", False):
            mod.apply_rotary_pos_emb = _make_rope(f)
        if f is not None:
            n_rope += 1
    counts = {"rmsnorm": n_norm, "swiglu_mlp": n_mlp, "rope_modules": n_rope, "prl_linear": n_linear,
              "qkv_groups": n_group, "add_norm_layers": n_addnorm}
    logger.info(f"fused model ops patched: {counts}")
    return counts
