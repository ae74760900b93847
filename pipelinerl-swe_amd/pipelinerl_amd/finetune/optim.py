"""Optimizer with decay / no-decay parameter groups (contract of pipelinerl/finetune/optim.py:8-45).

adamw_torch on the GPU is ``PrlAdamW``: torch.optim.AdamW(fused=True) (same param_groups, state
keys and checkpoints) whose step runs the HIP kernel of csrc/adamw.hip, with the gradient-clipping
multiply folded in (``clip_grad_norm``); elsewhere torch's AdamW.  adafactor comes from
transformers.  DeepSpeed's cpuadam and Lion are out of scope.
"""

from __future__ import annotations

import os

import numpy as np
import torch
from torch.autograd.graph import increment_version

NO_DECAY = ("bias", "LayerNorm.weight")


def get_grouped_params(model, weight_decay: float, no_decay=NO_DECAY):
    with_wd, without_wd = [], []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (without_wd if any(nd in n for nd in no_decay) else with_wd).append(p)
    return [{"params": with_wd, "weight_decay": weight_decay}, {"params": without_wd, "weight_decay": 0.0}]


_DTYPES = {torch.bfloat16: 1, torch.float32: 0}  # PRL_BF16 / PRL_F32 (include/prl_hip.h)


class PrlAdamW(torch.optim.AdamW):
    """torch.optim.AdamW(fused=True) with the step on csrc/adamw.hip (prl_adamw_step): one pass
    per tensor that reads p, g, m, v and writes p, m, v, bit-identical to torch's fused kernel
    (ATen fused_adam_utils.cuh) — which it replaces because torch launches it 320 blocks at a time,
    ~360 launches for a 7B model at ~3.3 TB/s.  ``defer_grad_scale(coef)``: the next step
    multiplies every gradient by the device scalar ``coef`` first, as clip_grad_norm_'s
    foreach_mul_ would have (the gradients themselves are left unscaled).  Groups the kernel does
    not cover (amsgrad, maximize, capturable, differentiable, tensor lr, mixed dtypes, non-CUDA or
    DTensor parameters) take torch's own step, with the deferred scale applied first."""

    def __init__(self, params, lr: float = 1e-3, weight_decay: float = 1e-2, **kw):
        kw["fused"] = True
        super().__init__(params, lr=lr, weight_decay=weight_decay, **kw)
        self._grad_scale: torch.Tensor | None = None

    def defer_grad_scale(self, coef: torch.Tensor) -> None:
        self._grad_scale = coef

    @staticmethod
    def _native_ok(group, params) -> bool:
        if group["amsgrad"] or group["maximize"] or group["capturable"] or group["differentiable"]:
            return False
        if torch.is_tensor(group["lr"]) or any(torch.is_tensor(b) for b in group["betas"]):
            return False
        if not params:
            return True
        dt = params[0].dtype
        return dt in _DTYPES and all(
            type(p) is torch.nn.Parameter and p.is_cuda and p.dtype == dt and p.grad.dtype == dt
            and not p.grad.is_sparse and p.is_contiguous() and p.grad.is_contiguous() for p in params)

    @torch.no_grad()
    def step(self, closure=None):
        from .model_ops import weights_written

        weights_written()  # parameters change below (either path): drop the fused-weight caches
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        scale, self._grad_scale = self._grad_scale, None
        plan = []
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            plan.append((group, params))
        dts = {ps[0].dtype for _, ps in plan if ps}
        if len(dts) > 1 or not all(self._native_ok(g, ps) for g, ps in plan):
            if scale is not None:
                grads = [p.grad for _, ps in plan for p in ps]
                if grads:
                    torch._foreach_mul_(grads, scale)
            return super().step()
        from .. import _native

        lib = _native.load()
        for group, params in plan:
            if not params:
                continue
            steps, ms, vs = [], [], []
            for p in params:
                st = self.state[p]
                if len(st) == 0:  # torch's fused-AdamW state (Adam._init_group), so checkpoints interchange
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                steps.append(st["step"])
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
            torch._foreach_add_(steps, 1)
            dt = params[0].dtype
            sc = None
            if scale is not None:
                sc = scale.to(device=params[0].device, dtype=dt).reshape(1).contiguous()
            ptr = lambda ts: np.fromiter((t.data_ptr() for t in ts), dtype=np.uint64, count=len(ts))  # noqa: E731
            arrs = [ptr(params), ptr([p.grad for p in params]), ptr(ms), ptr(vs), ptr(steps),
                    np.fromiter((p.numel() for p in params), dtype=np.int64, count=len(params))]
            beta1, beta2 = group["betas"]
            _native.check(lib.prl_adamw_step(len(params), *(a.ctypes.data for a in arrs), _DTYPES[dt],
                                             float(group["lr"]), float(beta1), float(beta2),
                                             float(group["weight_decay"]), float(group["eps"]),
                                             sc.data_ptr() if sc is not None else None,
                                             torch.cuda.current_stream(params[0].device).cuda_stream),
                          "prl_adamw_step")
            # the kernel wrote p, m, v through raw pointers: move their version counters as torch's
            # in-place step would, so caches keyed on them (model_ops._fused_weight: the fused
            # gate/up and q/k/v weights) see the update
            increment_version(params)
            increment_version(ms)
            increment_version(vs)
        return loss


def clip_grad_norm(parameters, max_norm: float, optimizer=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_(parameters, max_norm) — same total norm, same coefficient
    (max_norm / (norm + 1e-6) clamped to 1) — except that with a PrlAdamW ``optimizer`` the
    multiply is handed to its next step (one fewer read + write of every gradient) instead of
    done here.  Call optimizer.step() next, as the loop does.  Returns the total norm."""
    if not isinstance(optimizer, PrlAdamW):
        return torch.nn.utils.clip_grad_norm_(parameters, max_norm)
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    total = torch.nn.utils.get_total_norm(grads, 2.0, False, None)
    optimizer.defer_grad_scale(torch.clamp(float(max_norm) / (total + 1e-6), max=1.0))
    return total


def get_optimizer(name: str, model, learning_rate: float, weight_decay: float):
    groups = get_grouped_params(model, weight_decay)
    if name == "adamw_torch":
        on_gpu = all(p.is_cuda for g in groups for p in g["params"])
        plain = all(type(p) is torch.nn.Parameter for g in groups for p in g["params"])  # not FSDP DTensors
        if on_gpu and plain and os.environ.get("PRL_NATIVE_ADAMW", "1") != "0":  # 0: torch's fused AdamW (A/B)
            return PrlAdamW(groups, lr=learning_rate, weight_decay=weight_decay)
        return torch.optim.AdamW(groups, lr=learning_rate, fused=on_gpu or None)
    if name == "adafactor":
        from transformers import Adafactor

        return Adafactor(groups, lr=learning_rate, relative_step=False, scale_parameter=False)
    raise ValueError(f"Unknown optimizer: {name}")
