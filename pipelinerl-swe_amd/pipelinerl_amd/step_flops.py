"""Model FLOPs of one packed-GRPO optimizer step and its MFMA roofline (the north star's "fraction
of roofline" for the trainer step; reference throughput keys: finetune_loop.py:741-754).

Counted from the shapes actually run, as matrix-multiply FLOPs (2 per multiply-add), forward +
backward, no recompute (the usual model-FLOPs convention; a recomputed forward is not counted):

  * decoder linear layers (q, k, v, o, gate, up, down): 6 x their weight count x tokens
    (forward 2, input gradient 2, weight gradient 2 per weight and token);
  * lm_head: 6 x V x H x label rows — the trainer's label-row lm_head (RLConfig.fused_lm_head)
    forms logits only for rows whose next token is a label (rl/__init__.py:152-153);
  * causal attention: per sequence of length L, head and layer, QK^T and PV forward and the four
    backward products, each over the L(L+1)/2 unmasked score entries: 6 x d x L(L+1) FLOPs
    (d = head dim), over the query heads.

Biases, norms, activations, the embedding lookup, the loss head and the optimizer are vector /
HBM work and not counted.  Peak: MI355X dense bf16 MFMA, 2.5 PFLOP/s
(/opt/skills/guides/MI355X_MICROARCH.md; the 2:1-sparse 5 PF is never the reference).
"""

from __future__ import annotations

from dataclasses import dataclass

MFMA_BF16_DENSE_TFLOPS = 2500.0


@dataclass
class MicroBatchShape:
    tokens: int            # attention_mask sum (the reference's token count, finetune_loop.py:259-263)
    seq_lens: list[int]    # the packed sequences' lengths
    label_rows: int        # rows whose shifted label is not -100 (the label-row lm_head's rows)


def linear_weights_per_layer(cfg) -> int:
    """Weights of one Qwen2 decoder layer's seven projections."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    nh, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
    d = getattr(cfg, "head_dim", None) or H // nh
    q, kv = nh * d, nkv * d
    return H * q + 2 * H * kv + q * H + 3 * H * I


def shape_of(batch) -> MicroBatchShape:
    """The shape a PipelineBatchEncoding micro-batch puts through the step (packed: B = 1)."""
    import torch

    mask = batch.attention_mask
    tokens = int(mask.sum())
    if getattr(batch, "seq_boundaries", None) is not None:
        sb = [int(x) for x in torch.as_tensor(batch.seq_boundaries).reshape(-1).tolist()]
        lens = [b - a for a, b in zip(sb[:-1], sb[1:]) if b > a]
    elif getattr(batch, "position_ids", None) is not None:
        pos = batch.position_ids.reshape(-1).cpu()
        starts = (pos == 0).nonzero().reshape(-1).tolist() + [pos.numel()]
        lens = [b - a for a, b in zip(starts[:-1], starts[1:]) if b > a]
    else:
        lens = [int(x) for x in mask.sum(-1).reshape(-1).tolist()]
    if getattr(batch, "seq_boundaries", None) is not None and int(getattr(batch, "padding", 0) or 0) > 0:
        lens = lens[:-1]  # the trailing padding segment (finetune_loop.py:266-276) is not a sequence
    labels = batch.labels
    label_rows = int((labels[..., 1:] != -100).sum())
    return MicroBatchShape(tokens=tokens, seq_lens=lens, label_rows=label_rows)


def step_flops(cfg, shapes: list[MicroBatchShape], label_row_head: bool = True) -> dict:
    """FLOPs of one optimizer step over ``shapes`` (this rank's micro-batches) for a Qwen2 ``cfg``:
    {"linear", "lm_head", "attention", "total"}."""
    L = cfg.num_hidden_layers
    H, V = cfg.hidden_size, cfg.vocab_size
    nh = cfg.num_attention_heads
    d = getattr(cfg, "head_dim", None) or H // nh
    tokens = sum(s.tokens for s in shapes)
    rows = sum(s.label_rows for s in shapes) if label_row_head else tokens
    linear = 6 * linear_weights_per_layer(cfg) * L * tokens
    lm_head = 6 * V * H * rows
    attention = 6 * d * nh * L * sum(n * (n + 1) for s in shapes for n in s.seq_lens)
    return {"linear": linear, "lm_head": lm_head, "attention": attention, "total": linear + lm_head + attention,
            "tokens": tokens, "label_rows": rows}


def kernel_class(name: str) -> str:
    """gemm (hipBLASLt / Tensile "Cijk_" kernels, rocBLAS / CK gemms), attention (the build's
    attn_* kernels, flash attention), or other."""
    n = name.lower()
    if name.startswith("Cijk_") or "gemm" in n or "cijk" in n:
        return "gemm"
    if "attn" in n or "flash" in n or "fmha" in n:
        return "attention"
    return "other"


def kernel_breakdown(fn, device) -> dict:
    """Run ``fn()`` once under torch.profiler (device activity only) and sum its kernels' device
    time by class: {"gemm_ms", "attention_ms", "other_ms", "kernel_ms", "kernels"}."""
    import torch
    from torch.profiler import ProfilerActivity, profile

    torch.cuda.synchronize(device)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize(device)
    us = {"gemm": 0.0, "attention": 0.0, "other": 0.0}
    n = 0
    for ev in prof.events():
        if getattr(ev, "device_type", None) is None or str(ev.device_type).split(".")[-1] != "CUDA":
            continue
        t = getattr(ev, "device_time", None)
        if t is None:
            t = getattr(ev, "cuda_time", 0.0)
        us[kernel_class(ev.name)] += float(t)
        n += 1
    tot = sum(us.values())
    return {"gemm_ms": round(us["gemm"] / 1e3, 2), "attention_ms": round(us["attention"] / 1e3, 2),
            "other_ms": round(us["other"] / 1e3, 2), "kernel_ms": round(tot / 1e3, 2), "kernels": n}


def mfma_roofline(flops: dict, seconds: float, gemm: dict | None = None) -> dict:
    """The bench line's trainer-step ``roofline`` object: achieved TFLOP/s over the dense bf16 MFMA
    peak; ``gemm`` (optional): the same step's GEMM kernel time from its kernel trace."""
    achieved = flops["total"] / seconds / 1e12
    out = {"bound": "mfma", "achieved": round(achieved, 1), "peak": MFMA_BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
           "frac": round(achieved / MFMA_BF16_DENSE_TFLOPS, 4), "traffic": None,
           "flops_per_step": {k: flops[k] for k in ("linear", "lm_head", "attention", "total")},
           "flops_convention": "model FLOPs (fwd + bwd matrix products, no recompute), step_flops.py"}
    if gemm and gemm.get("gemm_ms"):
        g = flops["linear"] + flops["lm_head"]  # the products that run as library GEMMs
        out.update({"kernel_breakdown": gemm,
                    "gemm_share_of_kernel_time": round(gemm["gemm_ms"] / gemm["kernel_ms"], 4),
                    "gemm_achieved": round(g / (gemm["gemm_ms"] * 1e-3) / 1e12, 1),
                    "gemm_frac": round(g / (gemm["gemm_ms"] * 1e-3) / 1e12 / MFMA_BF16_DENSE_TFLOPS, 4)})
        if gemm.get("attention_ms"):
            out["attention_achieved"] = round(flops["attention"] / (gemm["attention_ms"] * 1e-3) / 1e12, 1)
    return out
