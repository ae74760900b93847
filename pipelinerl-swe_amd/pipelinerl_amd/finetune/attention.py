"""Packed-sequence (varlen) attention for the trainer's model forward.

The reference trains packed micro-batches with flash-attn-2 varlen: one [1, T] row holding many
rollouts, attention confined to each rollout (finetune/checkpoints.py:96-101, position_ids fed
to the model at rl/__init__.py:188-189).  This registers an HF attention implementation
``prl_varlen`` that does the same on ROCm with torch's flash-attention varlen
(``torch.nn.attention.varlen.varlen_attn``), given cumulative sequence offsets computed ONCE
per micro-batch on the host (``cu_seq_lens_q/k``, ``max_length_q/k`` — the FlashAttention
kwargs HF propagates to every layer).  If varlen is unavailable for the inputs it runs causal
SDPA per sequence (same result, no T x T mask either way).  For bf16, head dim 128 the backward is
the build's HIP flash-attention backward (csrc/attn_bwd.hip; 1.41x / 1.15x the library's at
8 x 2048 / 2 x 8192 on MI355X); PRL_ATTN_BWD=torch keeps the library's.
"""

from __future__ import annotations

import heapq
import logging
import os

import torch
import torch.nn.functional as F

logger = logging.getLogger(__name__)

PRL_VARLEN = "prl_varlen"
_registered = False
_varlen_ok: bool | None = None
_ITEMS: dict[tuple, tuple] = {}
BLOCK = 128  # keys / queries per workgroup of the HIP backward (csrc/attn_bwd.hip)


def _to_device(rows: list, width: int, device) -> torch.Tensor:
    """int32 [n, width] device copy of host rows without a host sync: staged in pinned memory, the
    copy queued non-blocking (torch's pinned allocator keeps the staging buffer until it is done)."""
    t = torch.tensor(rows if rows else [(0,) * width], dtype=torch.int32)
    if torch.device(device).type != "cuda":
        return t
    return t.pin_memory().to(device, non_blocking=True)


def _items(bounds: list[int], device) -> tuple:
    """(kv_items, q_items, n) int32 [n, 3] device tensors: (seq_start, seq_end, block_start) per
    128-row block of every sequence, heaviest first: key blocks by the causal query rows after
    them, query blocks by the key rows before them (the workgroups are dispatched in list order,
    so the long ones start first and the short ones fill the tail)."""
    key = (tuple(bounds), str(device))
    hit = _ITEMS.get(key)
    if hit is None:
        rows = [(a, b, x) for a, b in zip(bounds[:-1], bounds[1:]) for x in range(a, b, BLOCK)]
        kv = sorted(rows, key=lambda r: -(r[1] - r[2]))
        qb = sorted(rows, key=lambda r: -(min(r[2] + BLOCK, r[1]) - r[0]))
        hit = (_to_device(kv, 3, device), _to_device(qb, 3, device), len(rows))
        if len(_ITEMS) > 64:
            _ITEMS.clear()
        _ITEMS[key] = hit
    return hit


_SPLITS: dict[tuple, tuple] = {}
SPLIT_MIN_RATIO = 1.2
# part cap as a fraction of the target; None: chosen per packing by _makespan.  PRL_ATTN_SPLIT_CAP=1.0
# is the round-2 rule (A/B), tools/attn_role_split.py [round 1-3 tool, in git history] sweeps it
SPLIT_CAP_FRAC: float | None = float(os.environ["PRL_ATTN_SPLIT_CAP"]) if os.environ.get("PRL_ATTN_SPLIT_CAP") else None
SPLIT_CAPS = (1.0, 0.5, 0.33)
SPLIT_MARGIN = 0.04
# Costs of the list-schedule model (MI355X, 28 / 4 and 12 / 2 heads, profiles/r03_attn_cap_sweep.jsonl):
# one 32-query tile of one query head in a dK/dV workgroup, one 32-key tile in a dQ workgroup, the
# fp32 partial a split part writes, and attn_bwd_dkdv_reduce (launch + reading the partials).
KV_TILE_US, Q_TILE_US, PART_US = 1.2, 0.93, 4.0
REDUCE_US, REDUCE_US_PER_SLOT = 5.0, 0.033


def _plan(rows: list, w_kv: dict, rep: int, kv_heads: int, cap: float | None) -> tuple[list, list, list, int]:
    kv_rows, units, groups, slot = [], [], [], 0
    for r in rows:
        parts = min(rep, -(-w_kv[r] // cap)) if cap is not None and w_kv[r] > SPLIT_MIN_RATIO * cap else 1
        if parts <= 1:
            kv_rows.append(r)
            continue
        cuts = [rep * i // parts for i in range(parts + 1)]
        for g in range(kv_heads):
            groups.append((r[1], r[2], g, slot, parts))
            for p in range(parts):
                units.append((r[0], r[1], r[2], g, g * rep + cuts[p], g * rep + cuts[p + 1], slot))
                slot += 1
    units.sort(key=lambda u: -(u[5] - u[4]) * (u[1] - u[2]))  # heaviest first
    return kv_rows, units, groups, slot


def _makespan(rows: list, kv_rows: list, units: list, slots: int, heads: int, kv_heads: int, cus: int) -> float:
    """Modelled duration (us) of the fused launch + the partial reduce: the workgroups in launch
    order (split parts, key blocks, query blocks, each heaviest first), one per CU, each starting on
    the CU that frees first (one wave per SIMD: a CU runs one workgroup at a time)."""
    rep = heads // kv_heads
    jobs = [(u[5] - u[4]) * -(-(u[1] - u[2]) // 32) * KV_TILE_US + PART_US for u in units]
    for r in sorted(kv_rows, key=lambda r: -(r[1] - r[2])):
        jobs += [rep * -(-(r[1] - r[2]) // 32) * KV_TILE_US] * kv_heads
    for r in sorted(rows, key=lambda r: -(min(r[2] + BLOCK, r[1]) - r[0])):
        jobs += [-(-(min(r[2] + BLOCK, r[1]) - r[0]) // 32) * Q_TILE_US] * heads
    free = [0.0] * max(1, cus)
    end = 0.0
    for j in jobs:
        t = heapq.heappop(free) + j
        heapq.heappush(free, t)
        end = max(end, t)
    return end + (REDUCE_US + REDUCE_US_PER_SLOT * slots if units else 0.0)


def split_plan(bounds: list[int], heads: int, kv_heads: int, cus: int) -> tuple[list, list, list, int]:
    """Which dK/dV key blocks to split over the query heads of their group (host arithmetic only).

    A dK/dV workgroup sweeps all ``rep = heads / kv_heads`` query heads over every query after its
    key block: for the first blocks of a long sequence that is far more than a CU's share of the
    launch (a lone 4 096-token sequence at 28 / 4 heads: its first workgroup alone runs as long as
    two whole sequences, profiles/r02_attn_ragged.jsonl).  Work is counted in MFMAs per wave (one
    wave per SIMD: a workgroup's duration follows it): dK/dV 32 per 32-query tile per query head,
    dQ 24 per 32-key tile; target = max(the per-SIMD average, the largest dQ workgroup).  A plan
    with part cap c cuts the key blocks whose workgroup exceeds 1.2 x (c x target) into
    min(rep, ceil(work / (c x target))) contiguous head ranges.  The caps of SPLIT_CAPS are priced
    by _makespan (a list schedule of the launch with measured per-tile costs); the cheapest is
    taken if it beats the unsplit launch by SPLIT_MARGIN (the parts' fp32 partials and the reduce
    are not free: on 4 x 2048-token packings splitting measured slower, profiles/r03_attn_cap_sweep.jsonl).

    Returns (kv_rows, split_units, split_groups, slots): the unsplit (seq_start, seq_end,
    block_start) rows, the 7-tuples and 5-tuples of prl_attn_bwd_split, and the partial slots."""
    rep = heads // kv_heads
    rows = [(a, b, x) for a, b in zip(bounds[:-1], bounds[1:]) for x in range(a, b, BLOCK)]
    w_kv = {r: rep * 32 * -(-(r[1] - r[2]) // 32) for r in rows}
    w_q = [24 * -(-(min(r[2] + BLOCK, r[1]) - r[0]) // 32) for r in rows]
    total = 4 * (kv_heads * sum(w_kv.values()) + heads * sum(w_q))
    target = max(total / (4 * max(1, cus)), max(w_q, default=0), 1)
    if SPLIT_CAP_FRAC is not None:
        return _plan(rows, w_kv, rep, kv_heads, max(1, int(SPLIT_CAP_FRAC * target)))
    best = _plan(rows, w_kv, rep, kv_heads, None)
    if rep < 2:
        return best
    t_one = _makespan(rows, best[0], best[1], best[3], heads, kv_heads, cus)
    t_best = t_one
    for c in SPLIT_CAPS:
        plan = _plan(rows, w_kv, rep, kv_heads, max(1, int(c * target)))
        if not plan[1]:
            continue
        t = _makespan(rows, plan[0], plan[1], plan[3], heads, kv_heads, cus)
        if t < t_best and t < (1 - SPLIT_MARGIN) * t_one:
            best, t_best = plan, t
    return best


def _split_items(bounds: list[int], heads: int, kv_heads: int, device) -> tuple:
    """Device tensors of split_plan (cached per packing): (kv_items, n_kv, units, n_units, groups,
    n_groups, slots)."""
    key = (tuple(bounds), heads, kv_heads, str(device))
    hit = _SPLITS.get(key)
    if hit is None:
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        kv_rows, units, groups, slots = split_plan(bounds, heads, kv_heads, cus)
        kv_rows = sorted(kv_rows, key=lambda r: -(r[1] - r[2]))
        hit = (_to_device(kv_rows, 3, device), len(kv_rows), _to_device(units, 7, device), len(units),
               _to_device(groups, 5, device), len(groups), slots)
        if len(_SPLITS) > 64:
            _SPLITS.clear()
        _SPLITS[key] = hit
    return hit


class PackedCausalAttention(torch.autograd.Function):
    """HIP flash-attention forward (prl_attn_fwd; PRL_ATTN_FWD=torch: torch's varlen forward, its
    log-sum-exp converted) and HIP backward (prl_attn_bwd; tools/attn_backend_probe.py [round 1-3 tool, in git history],
    profiles/r01_attention_probe.jsonl).
    q: [T, H, 128], k / v: [T, Hkv, 128] bf16 (GQA native: no repeated k / v)."""

    @staticmethod
    def forward(ctx, q, k, v, cu, mx: int, bounds: list[int]):
        from .. import _native

        T, H, D = q.shape
        ctx.bounds = bounds
        ctx.hip_fwd = os.environ.get("PRL_ATTN_FWD", "hip") == "hip"
        ctx.split = os.environ.get("PRL_ATTN_SPLIT", "1") != "0"
        if ctx.split:  # the backward's split plan, built here (cached per packing) so the backward queues only kernels
            _split_items(bounds, H, k.shape[1], q.device)
        if ctx.hip_fwd:  # HIP forward: writes the backward's base-2 log-sum-exp [H, T] directly
            _, q_items, n = _items(bounds, q.device)
            out = torch.empty_like(q)
            lse2 = torch.empty((H, T), dtype=torch.float32, device=q.device)
            _native.check(_native.load().prl_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), q_items.data_ptr(), n,
                                                      out.data_ptr(), lse2.data_ptr(), T, H, k.shape[1], D, D ** -0.5,
                                                      torch.cuda.current_stream(q.device).cuda_stream), "prl_attn_fwd")
            ctx.save_for_backward(q, k, v, out, lse2, cu)
            return out
        out, lse, _, _, _ = torch.ops.aten._flash_attention_forward(q, k, v, cu, cu, mx, mx, 0.0, True, False)
        nseq = len(bounds) - 1
        # torch's varlen log-sum-exp on ROCm: [nseq, H, max_len] (checked: tools/lse_layout_probe.py [round 1-3 tool, in git history])
        if not (lse.dim() == 3 and tuple(lse.shape[:2]) == (nseq, q.shape[1]) and lse.shape[2] >= mx
                and lse.is_contiguous() and lse.dtype == torch.float32 and cu.numel() == nseq + 1):
            raise RuntimeError(f"unexpected flash-attention log-sum-exp layout {tuple(lse.shape)}")
        ctx.save_for_backward(q, k, v, out, lse, cu)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .. import _native

        q, k, v, out, lse, cu = ctx.saved_tensors
        dout = dout.contiguous()
        T, H, D = q.shape
        lib = _native.load()
        st = torch.cuda.current_stream(q.device).cuda_stream
        delta = torch.empty((H, T), dtype=torch.float32, device=q.device)
        if ctx.hip_fwd:
            lse2 = lse
            _native.check(lib.prl_attn_bwd_delta(out.data_ptr(), dout.data_ptr(), delta.data_ptr(), T, H, D, st),
                          "prl_attn_bwd_delta")
        else:
            lse2 = torch.empty((H, T), dtype=torch.float32, device=q.device)
            _native.check(lib.prl_attn_bwd_preprocess(out.data_ptr(), dout.data_ptr(), lse.data_ptr(), cu.data_ptr(),
                                                      lse.shape[0], lse.shape[2], lse2.data_ptr(), delta.data_ptr(),
                                                      T, H, D, st), "prl_attn_bwd_preprocess")
        kv_items, q_items, n = _items(ctx.bounds, q.device)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        if ctx.split:  # heavy key blocks split over query heads
            kv_s, n_kv, units, n_units, groups, n_groups, slots = _split_items(ctx.bounds, H, k.shape[1], q.device)
            parts = torch.empty((max(slots, 1), 2, BLOCK, D), dtype=torch.float32, device=q.device)
            _native.check(lib.prl_attn_bwd_split(
                q.data_ptr(), k.data_ptr(), v.data_ptr(), dout.data_ptr(), lse2.data_ptr(), delta.data_ptr(),
                kv_s.data_ptr(), n_kv, q_items.data_ptr(), n, units.data_ptr(), n_units, groups.data_ptr(), n_groups,
                parts.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), T, H, k.shape[1], D, D ** -0.5, st),
                "prl_attn_bwd_split")
            return dq, dk, dv, None, None, None
        _native.check(lib.prl_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), dout.data_ptr(), lse2.data_ptr(),
                                       delta.data_ptr(), kv_items.data_ptr(), n, q_items.data_ptr(), n, dq.data_ptr(),
                                       dk.data_ptr(), dv.data_ptr(), T, H, k.shape[1], D, D ** -0.5, st),
                      "prl_attn_bwd")
        return dq, dk, dv, None, None, None


def _hip_backward_ok(q, k) -> bool:
    return (q.dtype == torch.bfloat16 and k.dtype == torch.bfloat16 and q.shape[-1] == 128 == k.shape[-1]
            and q.shape[0] == k.shape[0] and q.shape[1] % k.shape[1] == 0
            and os.environ.get("PRL_ATTN_BWD", "hip") == "hip")


def varlen_attention_forward(module, query, key, value, attention_mask, scaling=None, dropout=0.0, **kwargs):
    """HF attention interface: query/key/value [B, H, T, D] -> ([B, T, H, D], None)."""
    cu = kwargs.get("cu_seq_lens_q")
    if cu is None:  # not a packed call: plain causal SDPA semantics
        from transformers.integrations.sdpa_attention import sdpa_attention_forward

        return sdpa_attention_forward(module, query, key, value, attention_mask, scaling=scaling, dropout=dropout,
                                      **kwargs)
    B, Hq, T, D = query.shape
    assert B == 1, "packed batches are [1, T]"
    Hkv = key.shape[1]
    # squeeze, not [0]: select's backward would allocate a zeroed [1, H, T, D] head-major gradient
    # and copy into it; squeeze's is a view, so dq / dk / dv reach RoPE and v_proj token-major
    q = query.squeeze(0).transpose(0, 1)
    k = key.squeeze(0).transpose(0, 1)
    v = value.squeeze(0).transpose(0, 1)
    mx = int(kwargs["max_length_q"])
    bounds = kwargs.get("cu_seq_lens_host")
    hip_bwd = bounds is not None and q.is_cuda and _hip_backward_ok(q, k)
    if Hkv != Hq and not hip_bwd:
        # GQA with the library backward: its native-GQA backward is slower than with repeated k / v
        # (6.32 vs 5.64 ms at 2 x 8192, tools/attn_backend_probe.py [round 1-3 tool, in git history]); the HIP backward takes GQA as is
        k = k.repeat_interleave(Hq // Hkv, dim=1)
        v = v.repeat_interleave(Hq // Hkv, dim=1)
    default_scale = D ** -0.5
    global _varlen_ok
    default_scaling = scaling is None or abs(scaling - default_scale) < 1e-12
    if hip_bwd and default_scaling:  # the build's kernels: errors propagate (no silent fallback)
        out = PackedCausalAttention.apply(q.contiguous(), k.contiguous(), v.contiguous(), cu, mx, list(bounds))
        return out.unsqueeze(0), None
    if default_scaling and q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and _varlen_ok is not False:
        try:
            from torch.nn.attention.varlen import varlen_attn

            out = varlen_attn(q.contiguous(), k.contiguous(), v.contiguous(), cu, cu, mx, mx, is_causal=True)
            _varlen_ok = True
            return out.unsqueeze(0), None
        except (RuntimeError, NotImplementedError) as e:  # the library's varlen kernels only
            if _varlen_ok is None:
                logger.warning(f"varlen flash attention unavailable ({e}); using per-sequence SDPA")
            _varlen_ok = False
    if k.shape[1] != Hq:  # the per-sequence SDPA fallback takes equal head counts
        k = k.repeat_interleave(Hq // Hkv, dim=1)
        v = v.repeat_interleave(Hq // Hkv, dim=1)
    if bounds is None:
        bounds = cu.tolist()
    outs = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        if b <= a:
            continue
        qi, ki, vi = (t[a:b].transpose(0, 1).unsqueeze(0) for t in (q, k, v))
        outs.append(F.scaled_dot_product_attention(qi, ki, vi, is_causal=True, scale=scaling)[0].transpose(0, 1))
    return torch.cat(outs, 0).unsqueeze(0), None


def register() -> str:
    global _registered
    if not _registered:
        from transformers import AttentionInterface
        from transformers.masking_utils import AttentionMaskInterface, flash_attention_mask

        AttentionInterface.register(PRL_VARLEN, varlen_attention_forward)
        AttentionMaskInterface.register(PRL_VARLEN, flash_attention_mask)
        _registered = True
    return PRL_VARLEN


def uses_varlen(model) -> bool:
    cfg = getattr(model, "config", None)
    return getattr(cfg, "_attn_implementation", None) == PRL_VARLEN


def packed_kwargs(batch, device) -> dict:
    """cu_seq_lens / max_length for a packed [1, T] batch, from host-side metadata."""
    sb = batch.seq_boundaries
    if sb is None or sb.numel() < 2:
        pos = batch.position_ids[0].cpu()
        starts = (pos == 0).nonzero().flatten().tolist()
        if not starts or starts[0] != 0:
            starts = [0] + starts
        bounds = starts + [int(pos.numel())]
    else:
        bounds = [int(x) for x in sb.cpu().tolist()]
    lens = [b - a for a, b in zip(bounds[:-1], bounds[1:])]
    cu = _to_device(bounds, 1, device).reshape(-1)
    mx = max(lens) if lens else 0
    return {"cu_seq_lens_q": cu, "cu_seq_lens_k": cu, "max_length_q": mx, "max_length_k": mx,
            "cu_seq_lens_host": bounds}
