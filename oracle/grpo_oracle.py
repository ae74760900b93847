"""CPU oracle for the GRPO loss head (TEST INFRASTRUCTURE — never the product path).

This module is a numpy restatement of the reference's ``rl_step`` loss head, its ~35
statistics and the gradient autograd would produce for it.  It exists only to check the
HIP path: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``pipelinerl_amd``) never imports
anything under ``oracle/`` and fails loudly when its HIP library is missing.

Parity pinning: the restatement is checked against golden vectors produced by running the
reference ``rl_step`` itself in the build container (``tests/golden/make_golden.py``,
fixtures ``tests/golden/f1_*.npz`` and ``f2_*.npz``; test ``tests/test_oracle_golden.py``).

Reference anchors (``/root/reference`` paths):
  * ``pipelinerl/finetune/rl/__init__.py:113-127``  linear_decay_coef
  * ``pipelinerl/finetune/rl/__init__.py:151-181``  masks / packed segments / num_sequences
  * ``pipelinerl/finetune/rl/__init__.py:199-210``  temperature, log_softmax, entropy, gather
  * ``pipelinerl/finetune/rl/__init__.py:212-292``  token weights, ratios, KL, policy loss
  * ``pipelinerl/finetune/rl/__init__.py:294-313``  value loss + final loss
  * ``pipelinerl/finetune/rl/__init__.py:315-377``  statistics
  * ``pipelinerl/finetune/rl/utils.py:25-30,66-87`` mask_sum / sum_sum (nan_to_num semantics)

The backward is the analytic gradient of the same graph, with torch's tie/clamp rules:
``minimum`` splits the gradient in half on ties, ``clamp`` passes the gradient on the
closed interval, ``nan_to_num`` passes it only where its input is finite.
"""

from __future__ import annotations

import math
from concurrent.futures import ThreadPoolExecutor
from typing import Any

import numpy as np

FLT_MAX = float(np.finfo(np.float32).max)

STAT_KEYS = [
    "loss", "max_loss", "min_loss", "reward", "max_reward", "min_reward", "entropy",
    "old_logprobs", "new_logprobs", "ref_logprobs", "advantage", "max_advantage",
    "min_advantage", "kl", "max_kl", "min_kl", "policy_loss", "surr1", "surr2",
    "ratio_new_old", "ratio_new_old_sum", "ratio_new_old_squared_sum", "ratio_ref_new",
    "ratio_ref_old", "clamp_log_ratio_ref_new_indicator",
    "clamp_log_ratio_new_old_indicator", "num_nans", "token_weight", "max_token_weight",
    "min_token_weight", "kl_coef", "entropy_bonus_coef", "num_output_tokens_sum",
    "input_size",
]
VALUE_STAT_KEYS = ["value_mean", "value_max", "value_min", "value_loss", "value_mse"]

RL_DEFAULTS = dict(
    policy_loss="ppo", use_advantages=True, epsilon=0.2, batch_size=0,
    reward_minus_kl_coef=0.0, kl_coef=0.1, final_kl_coef=0.1, entropy_bonus=0.0,
    final_entropy_bonus=0.0, relu_log_p_weights=False, clamp_log_ratio_ref_new_value=10.0,
    divide_advantage_by_std=True, overlong_filtering=False, group_normalization=False,
    temperature=1.0, filter_zero_advantage_groups=False, value_loss_coef=0.0,
)  # rl/__init__.py:38-99


def linear_decay_coef(current_step: int, max_step: int, initial: float, final: float) -> float:
    """rl/__init__.py:113-127."""
    return initial + (final - initial) * current_step / max_step


def _nz(x: np.ndarray) -> np.ndarray:
    """torch.nan_to_num on a float32 tensor: nan->0, +-inf -> +-float32 max (utils.py:28-30)."""
    return np.nan_to_num(x, nan=0.0, posinf=FLT_MAX, neginf=-FLT_MAX)


def _masked_sum(v: np.ndarray, m: np.ndarray) -> float:
    """mask_sum: (values * mask).nan_to_num(0).sum() (utils.py:25-30); the reference reports the
    float32 value of the sum (inf when it exceeds the float32 range)."""
    with np.errstate(invalid="ignore", over="ignore"):
        return float(np.float32(_nz(v * m).sum(dtype=np.float64)))


LN_FLT_MAX = float(np.log(np.finfo(np.float32).max))


def _exp32(x: np.ndarray) -> np.ndarray:
    """exp with float32 overflow semantics (the reference's token-level tensors are float32)."""
    with np.errstate(over="ignore", invalid="ignore"):
        return np.where(x > LN_FLT_MAX, np.inf, np.exp(np.minimum(x, LN_FLT_MAX)))


def num_sequences_of(batch: dict) -> int:
    """rl/__init__.py:158-181: packed -> #(position_ids == 0) with index 0 forced, else rows."""
    if batch.get("is_packed", False):
        pos = np.asarray(batch["position_ids"])[0]
        starts = pos == 0
        starts[0] = True
        return int(starts.sum())
    return int(np.asarray(batch["labels"]).shape[0])


def row_stats(logits: np.ndarray, targets: np.ndarray, inv_temp: float | None,
              temperature: float, dtype=np.float64) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Per-row (lse, entropy, target log-prob) of logits/temperature (rl/__init__.py:200-208).

    ``logits``: [R, V]; ``targets``: [R] int.  Computed in ``dtype`` (float64 by default).
    """
    x = logits.astype(dtype) / dtype(temperature)
    m = x.max(axis=-1, keepdims=True)
    z = x - m
    e = np.exp(z)
    s = e.sum(axis=-1, keepdims=True)
    lse = m + np.log(s)
    lp = x - lse
    p = e / s
    ent = -(p * lp).sum(axis=-1)
    tlp = np.take_along_axis(lp, targets[:, None].astype(np.int64), axis=-1)[:, 0]
    return lse[:, 0], ent, tlp


def row_grad(logits: np.ndarray, targets: np.ndarray, lse: np.ndarray, ent: np.ndarray,
             g_lp: np.ndarray, g_h: np.ndarray, temperature: float, dtype=np.float64) -> np.ndarray:
    """d loss / d logits for rows given per-row upstream grads of (target lp, entropy).

    dx_j = g_lp * (onehot_j - p_j) - g_h * p_j * (lp_j + H);  dlogits = dx / temperature.
    """
    x = logits.astype(dtype) / dtype(temperature)
    lp = x - lse[:, None]
    p = np.exp(lp)
    d = -p * (g_lp[:, None] + g_h[:, None] * (lp + ent[:, None]))
    rows = np.arange(x.shape[0])
    d[rows, targets] += g_lp
    return d / dtype(temperature)


def _rows_parallel(fn, n_rows: int, chunk: int, threads: int):
    spans = [(a, min(a + chunk, n_rows)) for a in range(0, n_rows, chunk)]
    if threads <= 1 or len(spans) == 1:
        return [fn(a, b) for a, b in spans]
    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(lambda ab: fn(*ab), spans))


def rl_step_oracle(logits: np.ndarray, batch: dict, config: dict, current_step: int,
                   max_step: int, values: np.ndarray | None = None, grad_out: float = 1.0,
                   compute_grad: bool = True, dtype=np.float64, threads: int = 1,
                   row_chunk: int = 64, grad_rows: np.ndarray | None = None,
                   rows: dict[str, np.ndarray] | None = None) -> dict[str, Any]:
    """Restatement of rl_step (rl/__init__.py:130-377) on fixed logits.

    ``logits``: [B, L, V] (any float dtype, e.g. float32 or bf16 values held in float32).
    ``batch``: dict of numpy arrays with the PipelineBatchEncoding fields
    (types.py:48-75): input_ids, labels, position_ids (packed), rewards, advantages,
    ref_logprobs, old_logprobs, group_tokens, num_labels, overflow, is_packed.
    ``values``: optional [B, L] value-head output (value_model.py:50-52).
    Returns loss, stats, new_logprobs/entropy [B, L-1], and (optionally) dlogits [B, L, V]
    and dvalues [B, L] for upstream gradient ``grad_out``.  ``grad_rows``: flat loss rows
    q = b*(L-1)+t; when given, only those rows' gradients are formed (``dlogits_rows`` [len, V],
    for full-size checks where [B, L, V] in float64 would not fit).  ``rows``: the per-row
    (lse, entropy, new_logprobs) of an earlier call on the same logits (its returned arrays):
    the pass over [B, L-1, V] is skipped and only the token arithmetic is redone (a full-size
    test reruns it with perturbed parameters to show its tolerance detects the change).
    Raises AssertionError / ValueError exactly where the reference does.
    """
    cfg = dict(RL_DEFAULTS)
    cfg.update(config)
    B, L, V = logits.shape
    input_ids = np.asarray(batch["input_ids"]).astype(np.int64)
    labels = np.asarray(batch["labels"]).astype(np.int64)
    f32 = lambda k: np.asarray(batch[k], dtype=np.float32).astype(dtype)  # noqa: E731
    mask = labels[:, 1:] != -100  # rl/__init__.py:152-153
    mf = mask.astype(dtype)
    num_sequences = num_sequences_of(batch)
    if batch.get("is_packed", False):
        assert num_sequences > 0, "No sequences found in packed batch"

    temperature = float(cfg["temperature"])
    targets = input_ids[:, 1:]
    R = B * (L - 1)
    flat_logits = logits[:, :-1, :].reshape(R, V)
    flat_tgt = targets.reshape(R)

    def _stats(a, b):
        return row_stats(flat_logits[a:b], flat_tgt[a:b], None, temperature, dtype)

    if rows is not None:
        lse, entropy, new_lp = (np.asarray(rows[k]).reshape(B, L - 1) for k in ("lse", "entropy", "new_logprobs"))
    else:
        parts = _rows_parallel(_stats, R, row_chunk, threads)
        lse = np.concatenate([p[0] for p in parts]).reshape(B, L - 1)
        entropy = np.concatenate([p[1] for p in parts]).reshape(B, L - 1)
        new_lp = np.concatenate([p[2] for p in parts]).reshape(B, L - 1)
    if not np.isfinite(new_lp).all():  # :209
        raise AssertionError(f"new_logprobs is not finite: {new_lp}")

    rewards = f32("rewards")[:, 1:]
    ref_lp = f32("ref_logprobs")[:, 1:]
    old_lp = f32("old_logprobs")[:, 1:]
    group_tokens = f32("group_tokens")[:, 1:]
    num_labels = f32("num_labels")[:, 1:]
    overflow = f32("overflow")[:, 1:]

    if cfg["group_normalization"]:  # :220-225
        assert (group_tokens > 0).all(), "group_tokens must be greater than zero for group normalization"
        w = 1.0 / group_tokens
    else:
        w = np.ones_like(group_tokens) / cfg["batch_size"] if cfg["batch_size"] else np.full_like(group_tokens, np.inf)
    if cfg["overlong_filtering"]:  # :227-230
        w = w * (1 - overflow)

    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        log_ratio_new_old = new_lp - old_lp  # :234-236
        ratio = _exp32(log_ratio_new_old)
        log_ratio_ref_new = ref_lp - new_lp
        if not np.isfinite(log_ratio_ref_new).all():  # :237
            raise AssertionError(f"log_ratio_ref_new is not finite: {log_ratio_ref_new}")
        has_value = values is not None
        if has_value:  # :239-248
            vp = np.asarray(values, dtype=np.float32).astype(dtype)[:, :-1]
            advantages = rewards - vp
        else:
            advantages = f32("advantages")[:, 1:]
        lpw = advantages if cfg["use_advantages"] else rewards  # :250
        if cfg["relu_log_p_weights"]:
            lpw = np.where(np.isnan(lpw), lpw, np.maximum(lpw, 0))
        C = float(cfg["clamp_log_ratio_ref_new_value"])
        ind_ref = np.abs(log_ratio_ref_new) > C  # :254
        c = np.clip(log_ratio_ref_new, -C, C)
        approx_kl = np.exp(c) - c - 1  # :262
        if not np.isfinite(approx_kl).all():  # :264
            raise AssertionError(f"approx_kl is not finite: {approx_kl}")
        ent_c = linear_decay_coef(current_step, max_step, cfg["entropy_bonus"], cfg["final_entropy_bonus"])
        kl_c = linear_decay_coef(current_step, max_step, cfg["kl_coef"], cfg["final_kl_coef"])
        eps = float(cfg["epsilon"])
        kind = cfg["policy_loss"]
        if kind == "ppo":  # :270-275
            surr1 = ratio * lpw
            clamped = np.clip(ratio, 1 - eps, 1 + eps)
            ind_no = clamped != ratio
            surr2 = clamped * lpw
            pol = np.minimum(surr1, surr2)
            ratio_used = ratio
        elif kind == "reinforce":  # :276-281
            surr1 = np.zeros_like(ratio)
            surr2 = np.zeros_like(ratio)
            ind_no = ratio > 1 + eps
            ratio_used = np.clip(ratio, 0, 1 + eps)
            pol = new_lp * lpw * ratio_used
        else:
            raise ValueError(f"Unknown algorithm {kind}")
        tok_loss = (pol - kl_c * approx_kl + ent_c * entropy) * w  # :286-290
        policy_loss_total = -_masked_sum(tok_loss, mf)  # :292
        final_loss = policy_loss_total
        if has_value:  # :294-308
            vl = 0.5 * np.square(vp - rewards) * w
            value_loss = _masked_sum(vl, mf)
            final_loss = policy_loss_total + cfg["value_loss_coef"] * value_loss
        final_loss = float(np.float32(final_loss))
        if not math.isfinite(final_loss):  # :313
            raise AssertionError(f"Non-finite loss detected: {final_loss}")

        n_out = int(mask.sum())
        if n_out == 0:  # :315-319
            stats = {"input_size": float(input_ids.size)}
        else:
            S = lambda v: _masked_sum(v, mf)  # noqa: E731
            mx = lambda v: float(v[mask].max())  # noqa: E731
            mn = lambda v: float(v[mask].min())  # noqa: E731
            stats = {
                "loss": final_loss, "max_loss": final_loss, "min_loss": final_loss,
                "reward": S(rewards / num_labels), "max_reward": mx(rewards), "min_reward": mn(rewards),
                "entropy": S(entropy / num_labels),
                "old_logprobs": S(old_lp / num_labels),
                "new_logprobs": S(new_lp / num_labels),
                "ref_logprobs": S(ref_lp / num_labels),
                "advantage": S(advantages / num_labels),
                "max_advantage": mx(advantages), "min_advantage": mn(advantages),
                "kl": S(approx_kl / num_labels), "max_kl": mx(approx_kl), "min_kl": mn(approx_kl),
                "policy_loss": S(pol / num_labels),
                "surr1": S(surr1 / num_labels), "surr2": S(surr2 / num_labels),
                "ratio_new_old": S(ratio_used / num_labels),
                "ratio_new_old_sum": S(ratio_used),
                "ratio_new_old_squared_sum": S(ratio_used * ratio_used),
                "ratio_ref_new": S(_exp32(log_ratio_ref_new) / num_labels),
                "ratio_ref_old": S(_exp32(ref_lp - old_lp) / num_labels),
                "clamp_log_ratio_ref_new_indicator": S(ind_ref / num_labels),
                "clamp_log_ratio_new_old_indicator": S(ind_no / num_labels),
                "num_nans": int(np.isnan(tok_loss).sum()),
                "token_weight": S(w / num_labels),
                "max_token_weight": mx(w), "min_token_weight": mn(w),
                "kl_coef": num_sequences * kl_c,
                "entropy_bonus_coef": num_sequences * ent_c,
                "num_output_tokens_sum": n_out,
                "input_size": int(input_ids.size),
            }
            if has_value:  # :368-375
                stats["value_mean"] = S(vp / num_labels)
                stats["value_max"] = mx(vp)
                stats["value_min"] = mn(vp)
                stats["value_loss"] = float(np.float32(value_loss))
                stats["value_mse"] = S(np.square(vp - rewards) / num_labels)

        out: dict[str, Any] = {"loss": final_loss, "stats": stats, "new_logprobs": new_lp,
                               "entropy": entropy, "lse": lse, "token_loss": tok_loss,
                               "num_sequences": num_sequences}
        if not compute_grad:
            return out

        # ---- analytic backward of the graph above -------------------------------------
        g = float(grad_out)
        fin = np.isfinite(tok_loss * mf)
        g_tok = -g * mf * fin  # d final / d tok_loss (through nan_to_num and mask)
        g_pol = g_tok * w
        g_kl = -g_tok * w * kl_c
        g_h = g_tok * w * ent_c
        if kind == "ppo":
            tie = surr1 == surr2
            g_s1 = g_pol * np.where(tie, 0.5, (surr1 < surr2).astype(dtype))
            g_s2 = g_pol * np.where(tie, 0.5, (surr2 < surr1).astype(dtype))
            inr = ((ratio >= 1 - eps) & (ratio <= 1 + eps)).astype(dtype)
            g_ratio = g_s1 * lpw + g_s2 * lpw * inr
            g_lp = g_ratio * ratio
        else:
            g_lp = g_pol * lpw * ratio_used
        inr_c = ((log_ratio_ref_new >= -C) & (log_ratio_ref_new <= C)).astype(dtype)
        g_lrrn = g_kl * (np.exp(c) - 1) * inr_c
        g_lp = g_lp - g_lrrn
        out["g_lp"] = g_lp
        out["g_h"] = g_h

        flat_glp = g_lp.reshape(R)
        flat_gh = g_h.reshape(R)
        flat_lse = lse.reshape(R)
        flat_ent = entropy.reshape(R)

        def _grad(a, b):
            return row_grad(flat_logits[a:b], flat_tgt[a:b], flat_lse[a:b], flat_ent[a:b],
                            flat_glp[a:b], flat_gh[a:b], temperature, dtype)

        if grad_rows is not None:
            q = np.asarray(grad_rows, dtype=np.int64)
            out["dlogits_rows"] = row_grad(flat_logits[q], flat_tgt[q], flat_lse[q], flat_ent[q], flat_glp[q],
                                           flat_gh[q], temperature, dtype)
            return out
        gparts = _rows_parallel(_grad, R, row_chunk, threads)
        dlogits = np.zeros((B, L, V), dtype=dtype)
        dlogits[:, :-1, :] = np.concatenate(gparts).reshape(B, L - 1, V)
        out["dlogits"] = dlogits
        if has_value:
            fin_v = np.isfinite(vl * mf)
            dv = np.zeros((B, L), dtype=dtype)
            dv[:, :-1] = g * cfg["value_loss_coef"] * mf * fin_v * w * (vp - rewards)
            out["dvalues"] = dv
        return out
