"""Label-row lm_head + GRPO loss head, chunked.

The reference materialises logits for every packed position (``model(...)`` then
``logits[:, :-1]``, rl/__init__.py:197-208) and back-propagates a full [T, V] dlogits
through ``lm_head``.  Prompt rows (``labels[:, 1:] == -100``, :152-153) never carry a gradient
and only enter the statistics through finiteness checks.  This function instead takes the
final hidden states and the ``lm_head`` weight and, for the label rows only, in chunks of
``chunk_rows``:

  logits_c  = h_c @ W^T                      (hipBLASLt GEMM, [c, V])
  prl_grpo_forward_rows(logits_c)            (HIP loss kernel; dlogits written in place)
  dh_c      = dlogits_c @ W                  (GEMM, prl_gemm for bf16)
  dW       += dlogits_c^T @ h_c              (GEMM, fp32 accumulator, prl_gemm for bf16)

then one ``prl_grpo_stats`` pass over all rows.  Peak extra memory is one [c, V] chunk (plus an
fp32 [V, H] accumulator when there are several) instead of two [T, V] tensors, and the three lm_head GEMMs and the
loss kernel skip the prompt rows.  The backward scales the saved dh / dW by the upstream
gradient on device (relative to ``params.grad_scale``, the loss scale the forward formed them at).

Semantics vs the reference: identical loss, statistics and gradients when the prompt rows'
logits are finite.  Non-finite logits on a prompt row are not seen (the reference's finiteness
assertion at :209 covers every row); rl_step checks the prompt rows' hidden states for
finiteness instead.  ``RLConfig.fused_lm_head`` (default on).
"""

from __future__ import annotations

import ctypes

import torch

from ... import _native, gemm
from ..._native import NSTAT, PRL_BF16, PRL_F32
from .fused import GrpoParams, _ptr, _relative, _workspace

_ADDMM_F32: dict[str, bool] = {}
# Parity-test tap (tests/test_configs_gpu.py): when set, called as tap(stage, q_rows, chunk, rows)
# with stage "logits" just before the loss kernel runs on a chunk and "dlogits" just after (the
# chunk then holds the gradient, written in place), so a test can read the label-row path's own
# logits, per-row outputs and dlogits.  Enqueues nothing when None (the product default).
ROW_TAP = None


def _accumulate_dw(dw: torch.Tensor, dlg: torch.Tensor, hc: torch.Tensor) -> None:
    """dw (fp32) += dlg^T @ hc with the bf16 GEMM accumulating into fp32 (addmm out_dtype)."""
    key = str(dw.device)
    if _ADDMM_F32.get(key, True) and dlg.dtype != torch.float32:
        try:
            torch.addmm(dw, dlg.t(), hc, torch.float32, out=dw)
            _ADDMM_F32[key] = True
            return
        except (RuntimeError, NotImplementedError):
            _ADDMM_F32[key] = False  # this build's BLAS has no bf16 -> fp32 path
    dw.add_(torch.mm(dlg.t(), hc).float())


def _c_batch(ptr: int, dtype: torch.dtype, B: int, L: int, V: int, ld: int, f: dict,
             values: torch.Tensor | None = None) -> _native.PrlGrpoBatch:
    return _native.PrlGrpoBatch(
        ptr, PRL_BF16 if dtype == torch.bfloat16 else PRL_F32, 0, B, L, V, ld,
        f["input_ids"].data_ptr(), f["labels"].data_ptr(), f["rewards"].data_ptr(), f["advantages"].data_ptr(),
        f["ref_logprobs"].data_ptr(), f["old_logprobs"].data_ptr(), f["group_tokens"].data_ptr(),
        f["num_labels"].data_ptr(), f["overflow"].data_ptr(), _ptr(values))


def _weight_grad(dw: torch.Tensor, g: torch.Tensor, param, w_dtype):
    """The lm_head weight gradient bf16(dw * g) (g: the upstream scale, fp32 on the device, not
    rounded to bf16).  bf16 weights: one prl_grad_scale_bf16 pass — added into param.grad when
    it already holds a gradient (the result autograd's AccumulateGrad would store, without the
    extra tensors; returns None then), else scaled in place (nothing written when g == 1)."""
    if w_dtype != torch.bfloat16 or not dw.is_contiguous() or dw.data_ptr() % 16:
        return (dw.float() * g).to(w_dtype)
    from ..model_ops import _accum_target

    lib = _native.load()
    stream = torch.cuda.current_stream(dw.device).cuda_stream
    src_dt = _native.PRL_F32 if dw.dtype == torch.float32 else _native.PRL_BF16
    g = g.reshape(1).contiguous()
    target = _accum_target(param)
    if target is not None and target.data_ptr() % 16 == 0:
        _native.check(lib.prl_grad_scale_bf16(dw.data_ptr(), src_dt, g.data_ptr(), target.data_ptr(), dw.numel(), 1,
                                              stream), "prl_grad_scale_bf16")
        return None
    out = dw if src_dt == _native.PRL_BF16 else torch.empty(dw.shape, dtype=torch.bfloat16, device=dw.device)
    _native.check(lib.prl_grad_scale_bf16(dw.data_ptr(), src_dt, g.data_ptr(), out.data_ptr(), dw.numel(), 0, stream),
                  "prl_grad_scale_bf16")
    return out


class LinearGrpoLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, weight, fields, params: GrpoParams, chunk_rows: int, label_rows=None, values=None):
        if hidden.device.type != "cuda":
            raise RuntimeError("the fused lm_head + GRPO loss runs on a HIP device only (no CPU fallback)")
        if hidden.dim() != 3 or weight.dim() != 2 or hidden.shape[-1] != weight.shape[1]:
            raise ValueError(f"hidden [B, L, H] / weight [V, H] expected, got {tuple(hidden.shape)} / "
                             f"{tuple(weight.shape)}")
        lib = _native.load()
        B, L, Hd = hidden.shape
        V = weight.shape[0]
        dev = hidden.device
        Q = B * (L - 1)
        w = weight.detach()
        h2 = hidden.detach().reshape(B * L, Hd)
        if w.dtype != h2.dtype:
            h2 = h2.to(w.dtype)
        write_grad = bool(hidden.requires_grad or weight.requires_grad)
        # lp, H, lse, tok_loss, g_lp, g_h, row max, row log2-sum; unscored rows stay 0
        rows = torch.zeros((8, max(Q, 1)), dtype=torch.float32, device=dev)
        stats = torch.empty(NSTAT, dtype=torch.float64, device=dev)
        dh = torch.zeros((B * L, Hd), dtype=h2.dtype, device=dev) if write_grad else None
        dw = None
        stream = torch.cuda.current_stream(dev).cuda_stream
        cp = params.to_c(write_grad)
        # a value head (values [B, L], every row): the rows read them for the advantage
        # (reward - value); the value loss, its statistics and dvalues come from the statistics
        # pass (rl/__init__.py:239-248, :294-310)
        vals = dvalues = None
        if values is not None:
            if tuple(values.shape) != (B, L):
                raise ValueError(f"values must be [B, L] = {(B, L)}, got {tuple(values.shape)}")
            vals = values.detach().to(torch.float32).contiguous()
            dvalues = torch.empty((B, L), dtype=torch.float32, device=dev)
        if Q > 0:
            if label_rows is not None and label_rows.device == dev:  # counted on the host by the loader
                qsel = label_rows
            else:
                mask = (fields["labels"][:, 1:] != -100).reshape(-1)
                qsel = torch.nonzero(mask).reshape(-1)  # one host sync: the GEMM shapes need the count
            hrow = qsel + torch.div(qsel, L - 1, rounding_mode="floor")  # q = b*(L-1)+t -> b*L+t
            R = int(qsel.numel())
            step = max(1, int(chunk_rows))
            use_prl = w.dtype == torch.bfloat16 and w.is_contiguous() and Hd % 8 == 0 and V % 8 == 0
            # one chunk: dW straight from one bf16-output GEMM over all label rows (the
            # reference's own rounding; 1.3x faster than the fp32-accumulating form at 1.5B
            # shapes).  Several chunks: an fp32 accumulator across them.
            single = R <= step and use_prl
            if write_grad and not single:
                dw = torch.zeros((V, Hd), dtype=torch.float32, device=dev)
            for a in range(0, R, step):
                idx = hrow[a:a + step]
                qc = qsel[a:a + step].contiguous()
                hc = h2.index_select(0, idx)
                # [c, V] contiguous
                lg = gemm.linear_fwd(hc, w) if use_prl and gemm.solution_for("fwd", hc.shape[0], V, Hd) is not None \
                    else torch.mm(hc, w.t())
                cb = _c_batch(lg.data_ptr(), lg.dtype, B, L, V, V, fields, vals)
                co = _native.PrlGrpoOutputs(*[rows[i].data_ptr() for i in range(8)], _ptr(dvalues),
                                            lg.data_ptr() if write_grad else None, None)
                if ROW_TAP is not None:
                    ROW_TAP("logits", qc, lg, rows)
                ws = _workspace(dev)
                _native.check(lib.prl_grpo_forward_rows(ctypes.byref(cb), ctypes.byref(cp), qc.data_ptr(),
                                                        qc.numel(), ctypes.byref(co), ws.data_ptr(), ws.numel(),
                                                        stream), "prl_grpo_forward_rows")
                if ROW_TAP is not None:
                    ROW_TAP("dlogits", qc, lg, rows)
                if write_grad and use_prl:  # ROCm hipBLASLt (include/prl_gemm.h)
                    dh.index_copy_(0, idx, gemm.linear_dgrad(lg, w))
                    if single:
                        dw = gemm.linear_wgrad(lg, hc)
                    else:
                        gemm.linear_wgrad(lg, hc, out=dw, accumulate=True)
                elif write_grad:
                    dh.index_copy_(0, idx, torch.mm(lg, w))
                    _accumulate_dw(dw, lg, hc)
                del lg, hc
        cb = _c_batch(0, w.dtype, B, L, V, V, fields, vals)
        co = _native.PrlGrpoOutputs(*[rows[i].data_ptr() for i in range(8)], _ptr(dvalues), None, stats.data_ptr())
        ws = _workspace(dev)
        _native.check(lib.prl_grpo_stats(ctypes.byref(cb), ctypes.byref(cp), ctypes.byref(co), ws.data_ptr(),
                                         ws.numel(), stream), "prl_grpo_stats")
        loss = (-stats[0] + params.value_loss_coef * stats[1]).to(torch.float32) if values is not None \
            else (-stats[0]).to(torch.float32)
        ctx.mark_non_differentiable(stats, rows)
        if write_grad and dw is None:  # no label rows: zero weight gradient
            dw = torch.zeros((V, Hd), dtype=torch.float32, device=dev)
        ctx.dh, ctx.dw, ctx.dvalues = dh, dw, dvalues
        ctx.param = weight  # the Parameter (its .grad: fused accumulation, _weight_grad)
        ctx.shape = (B, L, Hd)
        ctx.h_dtype, ctx.w_dtype = hidden.dtype, weight.dtype
        ctx.grad_scale = float(params.grad_scale)
        return loss, stats, rows

    @staticmethod
    def backward(ctx, g_loss, g_stats, g_rows):
        d_hidden = d_weight = d_values = None
        if g_loss is not None:
            g = _relative(g_loss.detach().to(torch.float32), ctx.grad_scale)  # dh / dW formed at grad_scale
            if ctx.dh is not None and ctx.needs_input_grad[0]:
                d_hidden = (ctx.dh.view(ctx.shape) * g.to(ctx.dh.dtype)).to(ctx.h_dtype)
            if ctx.dh is not None and ctx.needs_input_grad[1]:
                d_weight = _weight_grad(ctx.dw, g, ctx.param, ctx.w_dtype)
            if ctx.dvalues is not None and ctx.needs_input_grad[6]:
                d_values = ctx.dvalues * g
        ctx.dh = ctx.dw = ctx.dvalues = None
        return d_hidden, d_weight, None, None, None, None, d_values


def linear_grpo_loss(hidden: torch.Tensor, weight: torch.Tensor, fields: dict, params: GrpoParams,
                     chunk_rows: int = 65536, label_rows: torch.Tensor | None = None,
                     values: torch.Tensor | None = None):
    """(loss, stats [NSTAT] f64 device, rows [8, B*(L-1)]) of lm_head(hidden) -> GRPO loss head,
    scoring only the label rows.  ``weight``: the lm_head weight [V, H] (no bias).
    ``label_rows``: the rows q = b*(L-1)+t with a label (int64, on the device), if the caller
    counted them on the host (the trainer's loader does); else they are found on the device and
    their count read back.  ``values``: a value head's output [B, L] (every row; the loss then adds
    ``value_loss_coef`` x the value loss and d loss / d values flows back into the head)."""
    return LinearGrpoLossFn.apply(hidden, weight, fields, params, chunk_rows, label_rows, values)
