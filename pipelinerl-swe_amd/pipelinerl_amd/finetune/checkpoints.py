"""Model / tokenizer loading and atomic checkpoints (contract of
pipelinerl/finetune/checkpoints.py:75-296).

Directory layout (unchanged, so actors restart from ``finetune/current``):
  <output_dir>/current/            HF save_pretrained (safetensors) + tokenizer
  <output_dir>/intermediate/<step>/
  <output_dir>/training_state/training_state.pt   optimizer, lr_scheduler, TrainingMetrics
Every directory is written to ``~<name>`` first and renamed into place by rank 0.
"""

from __future__ import annotations

import contextlib
import logging
import os
import shutil
import types
from pathlib import Path
from typing import Any

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)

WEIGHT_FILES = ("pytorch_model.bin", "model.safetensors", "pytorch_model.bin.index.json",
                "model.safetensors.index.json")


def _rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _barrier(group=None) -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=group)


def load_tokenizer(config_name: str, fallback_eos: int | None = None):
    try:
        from transformers import AutoTokenizer

        return AutoTokenizer.from_pretrained(config_name)
    except Exception as e:  # no tokenizer files offline: only eos_token_id is needed on this path
        logger.warning(f"tokenizer for {config_name} unavailable ({e}); using eos_token_id only")
        return types.SimpleNamespace(eos_token_id=fallback_eos if fallback_eos is not None else 2,
                                     save_pretrained=lambda *a, **k: None, padding_side="right")


def has_weights(d: Path) -> bool:
    return any((Path(d) / f).exists() for f in WEIGHT_FILES)


def load_model(args, model_class: str, current_dir: Path, device: torch.device, shard_world=1,
               master_weights: bool | None = None):
    """HF causal LM from ``current_dir`` (resume) or ``args.config_name``; optional value head.
    Gradient checkpointing as the config asks, unless its activations fit the device
    (``gradient_checkpointing_policy``, finetune/recompute.py; ``shard_world``: the FSDP world, or a
    callable deciding it from the built model — finetune/sharding.py decide_sharding;
    ``master_weights``: the optimizer keeps fp32 masters, counted in the memory plan)."""
    from transformers import AutoConfig, AutoModelForCausalLM

    src = str(current_dir) if has_weights(current_dir) else args.config_name
    kw: dict[str, Any] = {}
    if args.get("load_as_bf16", True):
        kw["torch_dtype"] = torch.bfloat16
    attn = args.get("attn_implementation", "sdpa")
    if attn in ("flash_attention_2", "prl_varlen"):  # packed varlen attention (finetune/attention.py)
        from .attention import register

        attn = register()
    kw["attn_implementation"] = attn
    p = Path(src)
    if p.exists() and not has_weights(p):  # a config-only directory: random init of that architecture
        with torch.device(device):  # on the device: a CPU init of billions of parameters takes minutes
            model = AutoModelForCausalLM.from_config(AutoConfig.from_pretrained(src), **kw)
    else:
        model = AutoModelForCausalLM.from_pretrained(src, **kw)
    if device.type == "cuda" and args.get("fused_model_ops", True):  # HIP RMSNorm / SwiGLU / RoPE
        from .model_ops import patch_model

        patch_model(model)
    from .recompute import plan_gradient_checkpointing

    if callable(shard_world):
        shard_world = int(shard_world(model))
    plan = plan_gradient_checkpointing(args, model, device, shard_world, master_weights=master_weights)
    if args.get("gradient_checkpointing", False):
        logger.info(f"gradient checkpointing: {plan.as_dict()}")
    if plan.checkpoint:
        model.gradient_checkpointing_enable(
            gradient_checkpointing_kwargs={"use_reentrant": bool(args.get("reentrant_checkpointing", False))})
        keep_activations(model, plan.keep_layers)
    if model_class == "causal-language-modeling-with-value-head":
        from .value_model import AutoModelForCausalLMWithValueHead

        model = AutoModelForCausalLMWithValueHead(model)
        if src == str(current_dir):  # resume: the saved head too (value_model.py:189-192)
            model.load_value_head(current_dir)
    model.prl_memory_plan = plan  # the FSDP wrap reads gathered_layers (finetune_loop.py, shard_model)
    return model.to(device)


def keep_activations(model, keep: int) -> int:
    """After ``gradient_checkpointing_enable``: the last ``keep`` decoder layers keep their
    activations (their ``gradient_checkpointing`` flag, which transformers' GradientCheckpointingLayer
    reads per call, goes back off); the others recompute.  The kept layers are the last ones, so
    only checkpointed layers precede the boundary: the decoder's cross-layer residual hand-over
    (model_ops._decoder_forward) already stays off out of a checkpointed layer.  Returns how many
    layers keep their activations."""
    if keep <= 0:
        return 0
    from .sharding import decoder_layers

    layers = [m for m in decoder_layers(model) if hasattr(m, "gradient_checkpointing")]
    kept = layers[len(layers) - min(keep, len(layers)):]
    for m in kept:
        m.gradient_checkpointing = False
    return len(kept)


@contextlib.contextmanager
def temporary_folder_and_move(output_dir: Path, group=None):
    output_dir = Path(output_dir).resolve()
    tmp = output_dir.parent / ("~" + output_dir.name)
    if _rank() == 0:
        if tmp.exists():
            shutil.rmtree(tmp)
        tmp.mkdir(parents=True)
    _barrier(group)
    yield tmp
    _barrier(group)
    if _rank() == 0:
        if output_dir.exists():
            shutil.rmtree(output_dir)
        os.rename(tmp, output_dir)


def save_model_and_tokenizer(output_dir: Path, model, tokenizer, *, safe_serialization: bool = False, group=None):
    """checkpoints.py:280-300; ``safe_serialization`` is the config's ``use_safetensors``
    (finetune_loop.py:805-811), ``group`` the CPU control group of the barriers (keyword-only)."""
    from .sharding import full_state_dict, is_sharded

    sd = full_state_dict(model) if is_sharded(model) else None  # collective: every rank
    with temporary_folder_and_move(output_dir, group) as tmp:
        if _rank() == 0:
            m = getattr(model, "module", model)
            if sd is None and getattr(getattr(m, "pretrained_model", m), "_prl_flat_params", False):
                # parameters re-homed into one buffer for in-place weight broadcasts
                # (weight_update.py): save host copies, which share no storage.  Keys in m's own
                # namespace: a value-head wrapper splits them (value_model.save_pretrained)
                sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
            if sd is not None:
                save_dtype = getattr(m, "_prl_save_dtype", None)
                if save_dtype is not None:  # fp32 master shards: save the model's own dtype, as DeepSpeed's
                    # stage3_gather_16bit_weights_on_model_save does (conf/deepspeed/deepspeed_stage3_bf16.json)
                    sd = {k: v.to(save_dtype) if v.is_floating_point() else v for k, v in sd.items()}
                if getattr(getattr(m, "config", None), "tie_word_embeddings", False):
                    # tied copy (finetune_loop.py:228-231), under the wrapper's prefix too
                    lm_prefix = "pretrained_model." if hasattr(m, "pretrained_model") else ""
                    sd.pop(lm_prefix + "lm_head.weight", None)
                m.save_pretrained(tmp, state_dict=sd, safe_serialization=safe_serialization)
            else:
                m.save_pretrained(tmp, safe_serialization=safe_serialization)
            if hasattr(tokenizer, "save_pretrained"):
                tokenizer.save_pretrained(tmp)


def save_training_state(training_state_dir: Path, model, optimizer, lr_scheduler, extra: dict[str, Any], *,
                        group=None):
    """training_state.pt (metrics, lr scheduler, optimizer); with FSDP the sharded optimizer
    state goes to ``optim/`` (torch.distributed.checkpoint, every rank writes its shard)."""
    from .sharding import is_sharded, save_optimizer

    sharded = is_sharded(model)
    with temporary_folder_and_move(training_state_dir, group) as tmp:
        if sharded:
            save_optimizer(tmp / "optim", model, optimizer)
        if _rank() == 0:
            state = dict(extra)
            if not sharded:
                state["optimizer_state"] = optimizer.state_dict()
            state["lr_scheduler_state"] = lr_scheduler.state_dict()
            torch.save(state, tmp / "training_state.pt")


def load_training_state(training_state_dir: Path, model, optimizer, lr_scheduler, metrics):
    """Restores optimizer / scheduler (in place) and returns metrics updated from the file."""
    from .sharding import is_sharded, load_optimizer

    state = torch.load(Path(training_state_dir) / "training_state.pt", map_location="cpu", weights_only=True)
    if is_sharded(model):
        load_optimizer(Path(training_state_dir) / "optim", model, optimizer)
        state.pop("optimizer_state", None)
    else:
        optimizer.load_state_dict(state.pop("optimizer_state"))
    lr_scheduler.load_state_dict(state.pop("lr_scheduler_state"))
    for k, v in state.items():
        if hasattr(metrics, k):
            setattr(metrics, k, v)
    return metrics


def remove_results(*dirs: Path) -> None:
    for d in dirs:
        if Path(d).exists():
            shutil.rmtree(d)
