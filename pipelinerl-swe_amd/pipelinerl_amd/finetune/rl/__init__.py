"""GRPO / PPO / REINFORCE objective on MI355X — mirror of pipelinerl/finetune/rl/__init__.py.

Drop-in surface (same names, arguments, return values and errors as the reference):
  RLConfig            rl/__init__.py:38-99   (unknown keys ignored, like pydantic there)
  linear_decay_coef   rl/__init__.py:113-127
  rl_step             rl/__init__.py:130-377 -> (loss tensor, dict[str, float])
  populate_rl_data    rl/__init__.py:380-501
  prepare_rl_fields   rl/__init__.py:504-525

rl_step runs the model forward WITHOUT ``labels`` (the reference passes them, which makes HF
compute and discard a full fp32 cross-entropy over [T, V]; rl/__init__.py:183-197), then the
fused HIP loss head (fused.py), by default over the label rows only with the lm_head fused in
(fused_linear.py).  It reads the ~40 statistics back with ONE device->host copy (the reference
issues ~30 ``.item()`` calls); with ``defer_stats=True`` (the trainer loop) that copy is only
started, and the stats (and the reference's assertions) are materialised by
``RLStats.resolve()`` after the caller has launched the backward, so the GPU queue never drains
between a micro-batch's forward and backward.
"""

from __future__ import annotations

import logging
import math
from typing import Any

import numpy as np
import torch
from pydantic import BaseModel, Field

from ..attention import packed_kwargs, uses_varlen
from ..types import PipelineBatchEncoding
from .fused import GrpoParams, grpo_loss, prepare_fields
from .fused_linear import linear_grpo_loss
from ..._native import S

logger = logging.getLogger(__name__)
_warned: dict[str, bool] = {}

RL_DATA_COLUMNS = ["overflow", "group_tokens", "num_labels", "rewards", "advantages", "old_logprobs",
                   "ref_logprobs"]


class RLConfig(BaseModel):
    policy_loss: str = Field(default="ppo", description="Policy Loss to use for RL")
    use_advantages: bool = Field(default=True)
    epsilon: float = Field(default=0.2)
    batch_size: int = Field(default=0)
    reward_minus_kl_coef: float = Field(default=0.0)
    kl_coef: float = Field(default=0.1)
    final_kl_coef: float = Field(default=0.1)
    entropy_bonus: float = Field(default=0.0)
    final_entropy_bonus: float = Field(default=0.0)
    relu_log_p_weights: bool = Field(default=False)
    clamp_log_ratio_ref_new_value: float = Field(default=10)
    divide_advantage_by_std: bool = Field(default=True)
    overlong_filtering: bool = Field(default=False)
    group_normalization: bool = Field(default=False)
    temperature: float = Field(default=1.0)
    filter_zero_advantage_groups: bool = Field(default=False)
    value_loss_coef: float = Field(default=0.0)
    # build-only keys (absent from the reference; ignored there):
    # lm_head + loss over the label rows only, in row chunks (fused_linear.py); the prompt rows'
    # logits are never formed, their hidden states are checked for finiteness instead
    fused_lm_head: bool = Field(default=True)
    lm_head_chunk_rows: int = Field(default=65536)


def linear_decay_coef(current_step: int, max_step: int, initial_coef: float, final_coef: float) -> float:
    return initial_coef + (final_coef - initial_coef) * current_step / max_step


def _num_sequences_device(batch: PipelineBatchEncoding) -> torch.Tensor | int:
    """rl/__init__.py:158-181 without a host sync (packed: #(position_ids == 0), index 0 forced)."""
    if batch.is_packed:
        pos = batch.position_ids[0]
        return (pos == 0).sum() + (pos[0] != 0).to(torch.long)
    return int(batch.labels.shape[0])


class RLStats:
    """The statistics of one rl_step, still on their way to the host (``defer_stats=True``).
    ``resolve()`` waits for the one D2H copy (not for the backward queued behind it), runs the
    reference's assertions (rl/__init__.py:209, :237, :264, :313) and returns the dict."""

    def __init__(self, dev: torch.Tensor, batch, params, kl_c: float, ent_c: float, nseq, has_value_head: bool,
                 bad_hidden: torch.Tensor | None):
        parts = [dev]
        if isinstance(nseq, torch.Tensor):
            parts.append(nseq.to(dev.device, torch.float64).reshape(1))
        if bad_hidden is not None:
            parts.append(bad_hidden.to(dev.device, torch.float64).reshape(1))
        packed = torch.cat(parts) if len(parts) > 1 else dev
        self._host = torch.empty(packed.shape, dtype=torch.float64, pin_memory=packed.is_cuda)
        self._host.copy_(packed, non_blocking=True)
        self._event = None
        if packed.is_cuda:
            self._event = torch.cuda.Event()
            self._event.record(torch.cuda.current_stream(packed.device))
        self._args = (batch, params, kl_c, ent_c, nseq, has_value_head, bad_hidden is not None)
        self._value: dict[str, float] | None = None

    def resolve(self) -> dict[str, float]:
        if self._value is None:
            if self._event is not None:
                self._event.synchronize()
            h = self._host.numpy()
            batch, params, kl_c, ent_c, nseq, has_value_head, hidden_checked = self._args
            n = len(h) - int(hidden_checked)
            if hidden_checked and h[-1] > 0:  # a prompt row's logits cannot be finite (see below)
                raise AssertionError("new_logprobs is not finite: non-finite hidden states on prompt rows")
            if isinstance(nseq, torch.Tensor):
                num_sequences, n = int(h[n - 1]), n - 1
            else:
                num_sequences = nseq
            self._value = build_stats(h[:n], batch, params, kl_c, ent_c, num_sequences, has_value_head)
            self._args = None
        return self._value


def rl_step(model, batch: PipelineBatchEncoding, current_step: int, max_step: int,
            config: RLConfig, *, grad_scale: float = 1.0,
            defer_stats: bool = False) -> tuple[torch.Tensor, dict[str, float] | RLStats]:
    """One RL micro-batch: model forward + fused loss head.  Returns (loss, stats).

    ``grad_scale``: the factor the caller will multiply the loss by before ``backward()``
    (DeepSpeed's 1/gradient_accumulation_steps, finetune_loop.py:307-312): the fused kernels
    then write their gradients at that scale in the forward pass, so the backward needs no
    second pass over the logits.  Any other upstream gradient is still handled exactly.
    ``defer_stats``: return an RLStats whose ``resolve()`` gives the dict (see module doc)."""
    if config.policy_loss not in ("ppo", "reinforce"):
        raise ValueError(f"Unknown algorithm {config.policy_loss}")
    has_value_head = hasattr(model, "value_head")

    if batch.is_packed:
        # packed [1, T]: attention must stay inside each rollout (flash-attn varlen in the
        # reference).  The prl_varlen attention gets cu_seq_lens computed once on the host.
        model_inputs = {"input_ids": batch.input_ids, "position_ids": batch.position_ids}
        if uses_varlen(model):
            model_inputs.update(packed_kwargs(batch, batch.input_ids.device))
        elif hasattr(model, "config") and not _warned.get("varlen"):
            _warned["varlen"] = True
            logger.warning("packed batch on a model without prl_varlen attention: rollouts may attend "
                           "across sequence boundaries (load the model with attn_implementation="
                           "'flash_attention_2' or 'prl_varlen')")
    else:
        model_inputs = {"input_ids": batch.input_ids, "attention_mask": batch.attention_mask}
    if getattr(batch, "pixel_values", None) is not None:
        model_inputs["pixel_values"] = batch.pixel_values
    if getattr(batch, "image_grid_thw", None) is not None:
        model_inputs["image_grid_thw"] = batch.image_grid_thw
    if getattr(getattr(model, "config", None), "use_cache", None) is not None:
        model_inputs["use_cache"] = False  # training: no KV cache (HF would concatenate k / v per layer)
    fused_head = config.fused_lm_head and _lm_head_of(model) is not None
    bad_hidden = None
    if fused_head:
        from ..sharding import is_sharded

        if has_value_head or is_sharded(model):
            # through the root's own forward (FSDP gathers the root unit — embedding, final norm,
            # lm_head — as it does for the reference's forward; a value head reads the last hidden
            # state on every row), asking for no logits rows: the label-row head forms them below
            hidden, values = _hidden_through_root(model, model_inputs, has_value_head)
        else:
            hidden = _decoder_of(model)(**model_inputs).last_hidden_state
            values = None
        logits = hidden
        # The reference asserts every row's new log-probs finite (rl/__init__.py:209), prompt rows
        # included.  Label rows are checked by the kernel; a prompt row's logits h·Wᵀ are finite
        # when its hidden state is (W is finite, or every label row's log-softmax reports it),
        # barring bf16 overflow of a finite dot product.
        bad_hidden = torch.logical_not(torch.isfinite(hidden[:, :-1]).all())
    else:
        outputs = model(**model_inputs)
        logits = outputs.logits
        values = outputs.value if has_value_head else None

    ent_c = linear_decay_coef(current_step, max_step, config.entropy_bonus, config.final_entropy_bonus)
    kl_c = linear_decay_coef(current_step, max_step, config.kl_coef, config.final_kl_coef)
    params = GrpoParams(
        policy_loss=config.policy_loss, use_advantages=config.use_advantages,
        relu_log_p_weights=config.relu_log_p_weights, group_normalization=config.group_normalization,
        overlong_filtering=config.overlong_filtering, epsilon=config.epsilon, kl_coef=kl_c, entropy_coef=ent_c,
        clamp_log_ratio=float(config.clamp_log_ratio_ref_new_value), temperature=config.temperature,
        batch_size=float(config.batch_size), value_loss_coef=config.value_loss_coef if has_value_head else 0.0,
        grad_scale=float(grad_scale))
    fields = prepare_fields(batch, logits.device)
    if fused_head:
        weight = _lm_head_of(model).weight  # (under FSDP: the root unit's gathered weight)
        from torch.distributed.tensor import DTensor

        if isinstance(weight, DTensor):
            raise RuntimeError("fused_lm_head: the lm_head weight is still sharded after the root forward "
                               "(the FSDP root must keep its unit gathered until the backward: "
                               "finetune/sharding.py shard_model)")
        loss, stats_dev, _ = linear_grpo_loss(hidden, weight, fields, params, config.lm_head_chunk_rows,
                                              getattr(batch, "_label_rows", None), values)
    else:
        loss, stats_dev, _ = grpo_loss(logits, fields, params, values)

    stats = RLStats(stats_dev, batch, params, kl_c, ent_c, _num_sequences_device(batch), has_value_head, bad_hidden)
    return loss, (stats if defer_stats else stats.resolve())


def _decoder_of(model):
    dec = model.get_decoder() if hasattr(model, "get_decoder") else getattr(model, "model", None)
    if dec is None:
        raise ValueError("fused_lm_head needs a causal LM with a decoder (model.get_decoder())")
    return dec


def _lm_head_of(model):
    """The language model's plain bias-free lm_head Linear (under a value-head wrapper: its
    ``pretrained_model``'s), or None (with a one-time warning) when the model does something else
    between the decoder and the logits."""
    lm = getattr(model, "pretrained_model", model)
    head = lm.get_output_embeddings() if hasattr(lm, "get_output_embeddings") else None
    ok = (isinstance(head, torch.nn.Linear) and head.bias is None
          and getattr(getattr(lm, "config", None), "final_logit_softcapping", None) is None)
    if not ok:
        if not _warned.get("fused_lm_head"):
            _warned["fused_lm_head"] = True
            logger.warning("fused_lm_head: model has no plain bias-free lm_head; using the full-logits loss head")
        return None
    return head


def _hidden_through_root(model, model_inputs: dict, has_value_head: bool):
    """(last hidden state [B, L, H], values [B, L] or None) from ``model``'s own forward with no
    logits rows (``logits_to_keep=slice(0, 0)``): the decoder's output is caught by a forward hook.
    Under FSDP the root's pre-forward hook all-gathers the root unit (the embedding, the final norm,
    the lm_head) and keeps it gathered to the backward; a value-head wrapper (value_model.py) computes
    its values from the same hidden state (the reference: value_model.py:99-107)."""
    lm = getattr(model, "pretrained_model", model)
    dec = _decoder_of(lm)
    box: dict[str, torch.Tensor] = {}

    def keep(mod, args, out):
        box["h"] = out.last_hidden_state if hasattr(out, "last_hidden_state") else out[0]

    hook = dec.register_forward_hook(keep)
    try:
        out = model(**model_inputs, logits_to_keep=slice(0, 0))
    finally:
        hook.remove()
    return box["h"], (out.value if has_value_head else None)


def build_stats(h: np.ndarray, batch, params: GrpoParams, kl_c: float, ent_c: float, num_sequences: int,
                has_value_head: bool) -> dict[str, float]:
    """Assertions (in the reference's order) and the stats dict of rl/__init__.py:315-375."""
    if batch.is_packed and num_sequences <= 0:
        raise AssertionError("No sequences found in packed batch")
    if h[S["BAD_ID"]] > 0:
        raise RuntimeError("index out of bounds in gather: a target token id is outside [0, vocab)")
    if h[S["BAD_LP"]] > 0:
        raise AssertionError(f"new_logprobs is not finite: {int(h[S['BAD_LP']])} non-finite values")
    if params.group_normalization and h[S["BAD_GT"]] > 0:
        raise AssertionError("group_tokens must be greater than zero for group normalization")
    if h[S["BAD_LRRN"]] > 0:
        raise AssertionError(f"log_ratio_ref_new is not finite: {int(h[S['BAD_LRRN']])} non-finite values")
    if h[S["BAD_KL"]] > 0:
        raise AssertionError(f"approx_kl is not finite: {int(h[S['BAD_KL']])} non-finite values")
    policy_loss_total = np.float32(-h[S["LOSS_SUM"]])
    final = float(np.float32(policy_loss_total + np.float32(params.value_loss_coef) * np.float32(h[S["VALUE_LOSS"]]))) \
        if has_value_head else float(policy_loss_total)
    if not math.isfinite(final):
        raise AssertionError(f"Non-finite loss detected: {final}")
    input_size = int(batch.input_ids.numel())
    if h[S["NUM_OUT"]] == 0:
        return {"input_size": float(input_size)}
    # the reference reports float32 values (.item() of float32 tensors): round the fp64
    # accumulators, so a sum beyond the float32 range reads inf as it does there
    with np.errstate(over="ignore"):
        h = h.astype(np.float32).astype(np.float64)
    f = lambda k: float(h[S[k]])  # noqa: E731
    stats = {
        "loss": final, "max_loss": final, "min_loss": final,
        "reward": f("REWARD"), "max_reward": f("MAX_REWARD"), "min_reward": f("MIN_REWARD"),
        "entropy": f("ENTROPY"), "old_logprobs": f("OLD_LP"), "new_logprobs": f("NEW_LP"),
        "ref_logprobs": f("REF_LP"), "advantage": f("ADVANTAGE"), "max_advantage": f("MAX_ADV"),
        "min_advantage": f("MIN_ADV"), "kl": f("KL"), "max_kl": f("MAX_KL"), "min_kl": f("MIN_KL"),
        "policy_loss": f("POLICY_LOSS"), "surr1": f("SURR1"), "surr2": f("SURR2"),
        "ratio_new_old": f("RATIO"), "ratio_new_old_sum": f("RATIO_SUM"),
        "ratio_new_old_squared_sum": f("RATIO_SQ_SUM"), "ratio_ref_new": f("RATIO_REF_NEW"),
        "ratio_ref_old": f("RATIO_REF_OLD"), "clamp_log_ratio_ref_new_indicator": f("CLAMP_REF_NEW"),
        "clamp_log_ratio_new_old_indicator": f("CLAMP_NEW_OLD"), "num_nans": int(h[S["NUM_NANS"]]),
        "token_weight": f("TOKEN_WEIGHT"), "max_token_weight": f("MAX_W"), "min_token_weight": f("MIN_W"),
        "kl_coef": num_sequences * kl_c, "entropy_bonus_coef": num_sequences * ent_c,
        "num_output_tokens_sum": int(h[S["NUM_OUT"]]), "input_size": input_size,
    }
    if has_value_head:
        stats["value_mean"] = f("VALUE_MEAN")
        stats["value_max"] = f("MAX_VALUE")
        stats["value_min"] = f("MIN_VALUE")
        stats["value_loss"] = float(np.float32(h[S["VALUE_LOSS"]]))
        stats["value_mse"] = f("VALUE_MSE")
    return stats


# ---------------------------------------------------------------------------------------------
# preprocessing-side RL fields (run in the preprocessor workers, CPU)

def populate_rl_data(dataset: list[dict[str, Any]], eos_token_id: int, config: RLConfig) -> list[dict[str, Any]]:
    """Group advantages, group_tokens, overflow and num_labels (rl/__init__.py:380-501).

    Groups are keyed by (group_id, step_index); mean and sample std (ddof=1, NaN for a single
    rollout) of each rollout's first-token reward, the mean rollout length: pandas' groupby
    aggregations (Kahan mean, Welford std), computed by libprl_data (prl_rl_group_stats).
    advantage = r - mean, or (r - mean) / (nan_to_num(std) + 1e-4) when divide_advantage_by_std.
    """
    from ... import native_data

    keys = [f"{e['group_id']}_{e['step_index']}" for e in dataset]
    first_reward: dict[tuple[str, Any], float] = {}
    for k, e in zip(keys, dataset):
        r0 = e["rewards"][0]
        prev = first_reward.setdefault((k, e["rollout_index"]), r0)
        assert prev == r0, "rewards must be the same for every step of a rollout"
    index: dict[str, int] = {}
    group_of = np.fromiter((index.setdefault(k, len(index)) for k in keys), np.int64, len(keys))
    reward0 = np.fromiter((e["rewards"][0] for e in dataset), np.float64, len(dataset))
    length = np.fromiter((len(e["input_ids"]) for e in dataset), np.int64, len(dataset))
    mean, std, tokens = native_data.rl_group_stats(group_of, len(index), reward0, length)
    zero_var = int(np.count_nonzero(~(std >= 1e-6)))
    if zero_var:
        logger.warning(f"Found {zero_var} groups with zero variance!")
    denom = np.where(np.isnan(std), 0.0, std) + 1e-4
    for g, e in zip(group_of.tolist(), dataset):
        n = len(e["input_ids"])
        r = np.asarray(e["rewards"], dtype=np.float64)
        adv = (r - mean[g]) / denom[g] if config.divide_advantage_by_std else r - mean[g]
        e["advantages"] = adv.tolist()
        e["group_tokens"] = [float(tokens[g])] * n
        e["overflow"] = [0.0 if eos_token_id in e["input_ids"] else 1.0] * len(e["overflow"])
        lab = e["labels"]
        e["num_labels"] = [len(lab) - lab.count(-100) if isinstance(lab, list)
                           else int(np.count_nonzero(np.asarray(lab) != -100))] * n
    return dataset


def prepare_rl_fields(encoding: dict[str, Any], reward: float, old_logprobs: list[float],
                      ref_logprobs: list[float]) -> dict[str, Any]:
    """Per-token reward / log-prob fields for one rollout (rl/__init__.py:504-525)."""
    labels = encoding["labels"]
    n_target = sum(1 for t in labels if t != -100)
    assert n_target == len(old_logprobs), f"Target tokens: {n_target}, old logprobs: {len(old_logprobs)}"
    n = len(labels)
    encoding["rewards"] = [reward] * n
    encoding["advantages"] = [0.0] * n
    encoding["old_logprobs"] = [0] * (n - len(old_logprobs)) + list(old_logprobs)
    encoding["ref_logprobs"] = [0] * (n - len(ref_logprobs)) + list(ref_logprobs)
    encoding["overflow"] = [0] * n
    encoding["group_tokens"] = [0] * n
    encoding["num_labels"] = [1 if t != -100 else 0 for t in labels]
    return encoding
