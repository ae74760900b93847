"""Fused GRPO loss head as a torch.autograd.Function over the C-ABI HIP library.

Replaces the ATen op chain of rl_step (pipelinerl/finetune/rl/__init__.py:199-366) and its
autograd backward:
  forward  — one HIP pass over the [B, L, V] logits computes log-softmax, target
             log-prob, entropy, the per-token policy/KL/entropy loss, the masked
             statistics, and (when the logits require grad) writes dlogits for an upstream
             gradient of 1;
  backward — reads the upstream gradient on device; if it is 1 the precomputed dlogits are
             returned untouched (no extra pass, no host sync); the forward writes them for
             ``params.grad_scale`` (DeepSpeed's 1/GAS loss scale, passed in by the loop); any
             other upstream (sentinel batches multiply the loss by 0) recomputes dlogits from
             the logits with that scale.
The statistics stay on device; the caller reads them back once.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from ... import _native
from ..._native import PRL_BF16, PRL_F32, PRL_PPO, PRL_REINFORCE, NSTAT

def _workspace(device: torch.device) -> torch.Tensor:
    """The loss head's workspace (statistics partials + row-kernel scratch, include/prl_hip.h) for the
    current stream of ``device``: zero-filled once, one per (device, stream)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    lib = _native.load()
    nbytes = ctypes.c_size_t(0)
    _native.check(lib.prl_grpo_workspace_bytes(idx, ctypes.byref(nbytes)), "prl_grpo_workspace_bytes")
    return _native.stream_scratch("grpo", nbytes.value, device, torch.cuda.current_stream(device).cuda_stream)


@dataclass
class GrpoParams:
    """Scalar parameters of the loss head (RLConfig fields + decayed coefficients)."""
    policy_loss: str = "ppo"
    use_advantages: bool = True
    relu_log_p_weights: bool = False
    group_normalization: bool = False
    overlong_filtering: bool = False
    epsilon: float = 0.2
    kl_coef: float = 0.0
    entropy_coef: float = 0.0
    clamp_log_ratio: float = 10.0
    temperature: float = 1.0
    batch_size: float = 0.0
    value_loss_coef: float = 0.0
    # the upstream gradient the forward writes dlogits / dvalues for (the caller's loss scale)
    grad_scale: float = 1.0
    # fp32 logits: the pair kernel's partner wait (0 default, < 0 none) and the part-resident kernel
    # instead of the pair kernel (f32_rows 1) — measurement and test controls (include/prl_hip.h)
    pair_spin_ticks: int = 0
    f32_rows: int = 0

    def to_c(self, write_grad: bool) -> _native.PrlGrpoParams:
        if self.policy_loss == "ppo":
            kind = PRL_PPO
        elif self.policy_loss == "reinforce":
            kind = PRL_REINFORCE
        else:
            raise ValueError(f"Unknown algorithm {self.policy_loss}")
        return _native.PrlGrpoParams(
            kind, int(self.use_advantages), int(self.relu_log_p_weights), int(self.group_normalization),
            int(self.overlong_filtering), int(write_grad), self.epsilon, self.kl_coef, self.entropy_coef,
            self.clamp_log_ratio, self.temperature, float(self.batch_size), self.value_loss_coef,
            float(self.grad_scale), int(self.pair_spin_ticks), int(self.f32_rows))


FIELDS = ("input_ids", "labels", "rewards", "advantages", "ref_logprobs", "old_logprobs", "group_tokens",
          "num_labels", "overflow")


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def prepare_fields(batch, device: torch.device) -> dict[str, torch.Tensor]:
    """Device-resident, contiguous copies (no-ops when already so) of the token fields."""
    out = {}
    for k in FIELDS:
        t = getattr(batch, k) if not isinstance(batch, dict) else batch[k]
        dt = torch.long if k in ("input_ids", "labels") else torch.float32
        out[k] = t.to(device=device, dtype=dt).contiguous()
    return out


def _c_batch(logits: torch.Tensor, f: dict, values: torch.Tensor | None) -> _native.PrlGrpoBatch:
    B, L, V = logits.shape
    dt = PRL_BF16 if logits.dtype == torch.bfloat16 else PRL_F32
    return _native.PrlGrpoBatch(
        logits.data_ptr(), dt, 0, B, L, V, logits.stride(1),
        f["input_ids"].data_ptr(), f["labels"].data_ptr(), f["rewards"].data_ptr(), f["advantages"].data_ptr(),
        f["ref_logprobs"].data_ptr(), f["old_logprobs"].data_ptr(), f["group_tokens"].data_ptr(),
        f["num_labels"].data_ptr(), f["overflow"].data_ptr(), _ptr(values))


def _normalise_logits(logits: torch.Tensor) -> torch.Tensor:
    if logits.device.type != "cuda":
        raise RuntimeError("the fused GRPO loss head runs on a HIP device only (no CPU fallback)")
    if logits.dim() != 3:
        raise ValueError(f"logits must be [B, L, V], got {tuple(logits.shape)}")
    if logits.dtype not in (torch.bfloat16, torch.float32):
        logits = logits.float()
    B, L, V = logits.shape
    if logits.stride(2) != 1 or logits.stride(0) != L * logits.stride(1):
        logits = logits.contiguous()
    return logits


class GrpoLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, values, fields, params: GrpoParams):
        lib = _native.load()
        x = _normalise_logits(logits)
        B, L, V = x.shape
        dev = x.device
        R = max(B * (L - 1), 1)
        # lp, H, lse, tok_loss, g_lp, g_h, row max, row log2-sum
        rows = torch.empty((8, R), dtype=torch.float32, device=dev)
        stats = torch.empty(NSTAT, dtype=torch.float64, device=dev)
        write_grad = bool(logits.requires_grad)
        # same strides as the logits (a view with a wider row stride keeps its layout)
        dlogits = torch.empty_strided(x.shape, x.stride(), dtype=x.dtype, device=dev) if write_grad else None
        vals = None
        dvalues = None
        if values is not None:
            vals = values.detach().to(torch.float32).contiguous()
            dvalues = torch.empty((B, L), dtype=torch.float32, device=dev)
        cb = _c_batch(x, fields, vals)
        cp = params.to_c(write_grad)
        co = _native.PrlGrpoOutputs(*[rows[i].data_ptr() for i in range(8)], _ptr(dvalues), _ptr(dlogits),
                                    stats.data_ptr())
        ws = _workspace(dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        _native.check(lib.prl_grpo_forward(ctypes.byref(cb), ctypes.byref(cp), ctypes.byref(co), ws.data_ptr(),
                                           ws.numel(), stream), "prl_grpo_forward")
        loss = (-stats[0] + params.value_loss_coef * stats[1]).to(torch.float32) if values is not None \
            else (-stats[0]).to(torch.float32)
        ctx.mark_non_differentiable(stats, rows)
        ctx.x = x
        ctx.fields = fields
        ctx.vals = vals
        ctx.params = params
        ctx.dlogits = dlogits
        ctx.dvalues = dvalues
        ctx.rows = rows
        ctx.logits_dtype = logits.dtype
        return loss, stats, rows

    @staticmethod
    def backward(ctx, g_loss, g_stats, g_rows):
        d_logits = d_values = None
        if g_loss is None:
            return None, None, None, None
        # absolute upstream: the kernel compares it with params.grad_scale (the scale the forward
        # wrote dlogits at) and skips when they are equal
        g = g_loss.detach().to(torch.float32).reshape(1).contiguous()
        if ctx.dlogits is not None and ctx.needs_input_grad[0]:
            lib = _native.load()
            cb = _c_batch(ctx.x, ctx.fields, ctx.vals)
            cp = ctx.params.to_c(True)
            r = ctx.rows
            stream = torch.cuda.current_stream(ctx.x.device).cuda_stream
            _native.check(lib.prl_grpo_backward(ctypes.byref(cb), ctypes.byref(cp), r[6].data_ptr(), r[7].data_ptr(),
                                                r[1].data_ptr(), r[4].data_ptr(), r[5].data_ptr(), g.data_ptr(),
                                                ctx.dlogits.data_ptr(), stream), "prl_grpo_backward")
            d_logits = ctx.dlogits if ctx.logits_dtype == ctx.dlogits.dtype else ctx.dlogits.to(ctx.logits_dtype)
        if ctx.dvalues is not None and ctx.needs_input_grad[1]:
            d_values = ctx.dvalues * _relative(g, ctx.params.grad_scale)
        ctx.dlogits = None
        return d_logits, d_values, None, None


def _relative(g: torch.Tensor, scale: float) -> torch.Tensor:
    """g / scale on device, exactly 1 where g == scale (gradients saved at ``scale``)."""
    if scale == 1.0:
        return g
    return torch.where(g == scale, torch.ones_like(g), g / scale)


def grpo_loss(logits: torch.Tensor, fields: dict, params: GrpoParams, values: torch.Tensor | None = None):
    """Returns (loss [float32 scalar, differentiable], stats [NSTAT] float64 device tensor,
    rows [8, B*(L-1)] float32: new_logprobs, entropy, lse, token_loss, g_lp, g_h, row max,
    row log2-sum)."""
    return GrpoLossFn.apply(logits, values, fields, params)
