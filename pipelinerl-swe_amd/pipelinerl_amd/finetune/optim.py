"""Optimizer with decay / no-decay parameter groups (contract of pipelinerl/finetune/optim.py:8-45).

adamw_torch on the GPU is ``PrlAdamW``: torch.optim.AdamW(fused=True) (same param_groups, state
keys and checkpoints) whose step runs the HIP kernel of csrc/adamw.hip, with the gradient-clipping
multiply folded in (``clip_grad_norm``); elsewhere torch's AdamW.  adafactor comes from
transformers.  DeepSpeed's cpuadam and Lion are out of scope.
"""

from __future__ import annotations

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


MASTER_KEYS = ("master", "exp_avg", "exp_avg_sq")  # fp32 state of a master-weight parameter


class PrlAdamW(torch.optim.AdamW):
    """torch.optim.AdamW(fused=True) with the step on csrc/adamw.hip (prl_adamw_step): one pass
    per tensor that reads p, g, m, v and writes p, m, v, bit-identical to torch's fused kernel
    (ATen fused_adam_utils.cuh) — which it replaces because torch launches it 320 blocks at a time,
    ~360 launches for a 7B model at ~3.3 TB/s.  ``defer_grad_scale(coef)``: the next step
    multiplies every gradient by the device scalar ``coef`` first, as clip_grad_norm_'s
    foreach_mul_ would have (the gradients themselves are left unscaled).  Groups the kernel does
    not cover (amsgrad, maximize, capturable, differentiable, tensor lr, mixed dtypes, non-CUDA or
    DTensor parameters) take torch's own step, with the deferred scale applied first.

    ``master_weights=True`` (the default the trainer picks, ``finetune.master_weights``): every bf16
    parameter gets an fp32 master copy and fp32 moments (state keys ``master``, ``exp_avg``,
    ``exp_avg_sq``), as the reference's default DeepSpeed bf16 ZeRO optimizer and its FSDP mixed
    precision keep them; the step is prl_adamw_master_step — the fp32 gradient (the bf16 gradient
    times the clip coefficient in fp32) updates the fp32 state with torch's fused-AdamW fp32
    arithmetic, and the bf16 parameter becomes the new master's round-to-nearest-even, written in
    place.  Bit-identical to clip_grad_norm_ + torch.optim.AdamW(fused=True) on fp32 copies of the
    parameters and gradients followed by ``p.copy_(master)``.  fp32 parameters are their own
    masters (plain AdamW)."""

    def __init__(self, params, lr: float = 1e-3, weight_decay: float = 1e-2, master_weights: bool = False, **kw):
        kw["fused"] = True
        super().__init__(params, lr=lr, weight_decay=weight_decay, **kw)
        self._grad_scale: torch.Tensor | None = None
        self.master_weights = bool(master_weights)

    def defer_grad_scale(self, coef: torch.Tensor) -> None:
        self._grad_scale = coef

    def _uses_master(self, p) -> bool:
        return self.master_weights and p.dtype == torch.bfloat16 and type(p) is torch.nn.Parameter

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

    def _master_state(self, p) -> dict:
        st = self.state[p]
        if "master" not in st:  # first step (or a checkpoint written without master weights)
            st.setdefault("step", torch.zeros((), dtype=torch.float32, device=p.device))
            st["master"] = p.detach().float().contiguous()
            for k in ("exp_avg", "exp_avg_sq"):
                st[k] = st[k].float().contiguous() if k in st else torch.zeros_like(st["master"])
        return st

    def load_state_dict(self, state_dict):
        """torch's load, except that the fp32 master state stays fp32 (torch casts every floating
        state tensor to its parameter's dtype, which would round the masters and moments to bf16).
        A checkpoint written without master weights resumes with masters = the loaded bf16
        parameters and its moments widened; with ``master_weights=False`` saved masters are dropped."""
        saved = {pid: {k: v for k, v in st.items() if k in MASTER_KEYS and torch.is_tensor(v)}
                 for pid, st in state_dict["state"].items()}
        super().load_state_dict(state_dict)
        ids = [pid for g in state_dict["param_groups"] for pid in g["params"]]
        params = [p for g in self.param_groups for p in g["params"]]
        for pid, p in zip(ids, params):
            st = self.state.get(p)
            if not st:
                continue
            if not self._uses_master(p):
                st.pop("master", None)
                continue
            for k, v in saved.get(pid, {}).items():
                st[k] = v.to(device=p.device, dtype=torch.float32).contiguous()
            self._master_state(p)

    def _master_step(self, group, params, scale) -> None:
        """The master-weight update of ``params`` (bf16, plain Parameters) of ``group``."""
        states = [self._master_state(p) for p in params]
        steps = [st["step"] for st in states]
        torch._foreach_add_(steps, 1)
        beta1, beta2 = group["betas"]
        hyper = (float(group["lr"]), float(beta1), float(beta2), float(group["weight_decay"]), float(group["eps"]))
        if all(p.is_cuda and p.is_contiguous() and p.grad.is_contiguous() and not p.grad.is_sparse
               and p.grad.dtype in _DTYPES for p in params) and len({p.grad.dtype for p in params}) == 1:
            from .. import _native

            lib = _native.load()
            dev = params[0].device
            sc = None
            if scale is not None:
                sc = scale.to(device=dev, dtype=torch.float32).reshape(1).contiguous()
            ptr = lambda ts: np.fromiter((t.data_ptr() for t in ts), dtype=np.uint64, count=len(ts))  # noqa: E731
            arrs = [ptr(params), ptr([p.grad for p in params]), ptr([st["master"] for st in states]),
                    ptr([st["exp_avg"] for st in states]), ptr([st["exp_avg_sq"] for st in states]), ptr(steps),
                    np.fromiter((p.numel() for p in params), dtype=np.int64, count=len(params))]
            _native.check(lib.prl_adamw_master_step(len(params), *(a.ctypes.data for a in arrs),
                                                    _DTYPES[params[0].grad.dtype], *hyper,
                                                    sc.data_ptr() if sc is not None else None,
                                                    torch.cuda.current_stream(dev).cuda_stream),
                          "prl_adamw_master_step")
            increment_version(params)
            increment_version([st[k] for st in states for k in MASTER_KEYS])
            return
        # torch's fused fp32 AdamW on the masters, then the bf16 rounding back (CPU, odd layouts)
        grads = [p.grad.float() for p in params]
        if scale is not None:
            torch._foreach_mul_(grads, scale.to(device=grads[0].device, dtype=torch.float32))
        lr, b1, b2, wd, eps = hyper
        torch._fused_adamw_([st["master"] for st in states], grads, [st["exp_avg"] for st in states],
                            [st["exp_avg_sq"] for st in states], [], steps, lr=lr, beta1=b1, beta2=b2,
                            weight_decay=wd, eps=eps, amsgrad=False, maximize=False)
        for p, st in zip(params, states):
            p.copy_(st["master"])

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
        if self.master_weights and any(self._uses_master(p) for _, ps in plan for p in ps):
            if any(g["amsgrad"] or g["maximize"] or g["capturable"] or g["differentiable"] or torch.is_tensor(g["lr"])
                   for g, _ in plan):
                raise NotImplementedError("master_weights supports plain AdamW groups only (no amsgrad, maximize, "
                                          "capturable, differentiable or tensor lr)")
            rest = []
            for group, params in plan:
                mp = [p for p in params if self._uses_master(p)]
                if mp:
                    self._master_step(group, mp, scale)
                rest.append((group, [p for p in params if not self._uses_master(p)]))
            if any(ps for _, ps in rest):  # fp32 parameters beside bf16 ones: plain AdamW for them
                self._plain_step(rest, scale)
            return loss
        self._plain_step(plan, scale)
        return loss

    def _plain_step(self, plan, scale) -> None:
        dts = {ps[0].dtype for _, ps in plan if ps}
        if len(dts) > 1 or not all(self._native_ok(g, ps) for g, ps in plan):
            if scale is not None:
                grads = [p.grad for _, ps in plan for p in ps]
                if grads:
                    torch._foreach_mul_(grads, scale)
            keep = {id(p) for _, ps in plan for p in ps}
            hidden = [(p, p.grad) for g in self.param_groups for p in g["params"]
                      if p.grad is not None and id(p) not in keep]  # stepped by _master_step
            for p, _ in hidden:
                p.grad = None
            try:
                super().step()
            finally:
                for p, gr in hidden:
                    p.grad = gr
            return
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


def clip_grad_norm(parameters, max_norm: float, optimizer=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_(parameters, max_norm) — same total norm, same coefficient
    (max_norm / (norm + 1e-6) clamped to 1) — except that with a PrlAdamW ``optimizer`` the
    multiply is handed to its next step (one fewer read + write of every gradient) instead of
    done here.  Call optimizer.step() next, as the loop does.  Returns the total norm.  With
    master weights the norm and the coefficient are fp32, as DeepSpeed / FSDP compute them on the
    fp32 gradients (torch.linalg.vector_norm of each bf16 gradient upcast to fp32)."""
    if not isinstance(optimizer, PrlAdamW):
        return torch.nn.utils.clip_grad_norm_(parameters, max_norm)
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    if optimizer.master_weights:
        norms = torch._foreach_norm(grads, 2.0, dtype=torch.float32)
        total = torch.linalg.vector_norm(torch.stack([n.to(grads[0].device) for n in norms]), 2.0)
    else:
        total = torch.nn.utils.get_total_norm(grads, 2.0, False, None)
    optimizer.defer_grad_scale(torch.clamp(float(max_norm) / (total + 1e-6), max=1.0))
    return total


def master_weights_requested(cfg) -> bool:
    """Whether the optimizer keeps fp32 master weights and moments (``finetune.master_weights``:
    true | false | auto, default auto).  ``auto`` follows the reference's backend: its default
    DeepSpeed bf16 ZeRO optimizer (``use_deepspeed: true``, conf/base.yaml:94-95) and its FSDP mixed
    precision (``use_fsdp``: accelerate upcasts the parameters to fp32 in ``prepare``,
    finetune_loop.py:355-396) keep fp32 masters; only its plain-DDP launch (``use_deepspeed: false``
    and ``use_fsdp: false`` given explicitly) trains the bf16 weights themselves.  A config that names
    neither backend gets the reference default's (master weights)."""
    args = cfg.finetune if "finetune" in cfg else cfg
    mode = args.get("master_weights", "auto")
    if isinstance(mode, bool):
        return mode
    if str(mode) != "auto":
        raise ValueError(f"finetune.master_weights must be true, false or 'auto', got {mode!r}")
    if cfg.get("use_fsdp", False):
        return True
    return cfg.get("use_deepspeed", None) is not False


def get_optimizer(name: str, model, learning_rate: float, weight_decay: float, master_weights: bool = False):
    """The reference's optimizers (finetune/optim.py:25-45).  ``master_weights``: bf16 parameters get
    fp32 masters and moments (PrlAdamW); FSDP-sharded parameters are upcast by the sharding itself
    (finetune/sharding.py) and need no separate copy."""
    groups = get_grouped_params(model, weight_decay)
    if name == "adamw_torch":
        on_gpu = all(p.is_cuda for g in groups for p in g["params"])
        plain = all(type(p) is torch.nn.Parameter for g in groups for p in g["params"])  # not FSDP DTensors
        if plain and (on_gpu or master_weights):  # CPU masters: torch's fused fp32 step (gloo rehearsals)
            return PrlAdamW(groups, lr=learning_rate, weight_decay=weight_decay, master_weights=master_weights)
        return torch.optim.AdamW(groups, lr=learning_rate, fused=on_gpu or None)
    if name == "adafactor":
        from transformers import Adafactor

        return Adafactor(groups, lr=learning_rate, relative_step=False, scale_parameter=False)
    raise ValueError(f"Unknown optimizer: {name}")
