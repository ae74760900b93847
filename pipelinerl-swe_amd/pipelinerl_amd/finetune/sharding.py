"""Fully sharded data-parallel trainer (the reference's FSDP path for 32B, config C5).

The reference gets FSDP from Accelerate's plugin (``use_fsdp``: conf/accelerate/fsdp_mp.yaml —
FULL_SHARD, transformer-layer wrap, ``fsdp.{param,reduce,buffer}_dtype`` mixed precision,
finetune_loop.py:369-391) and gathers a FULL_STATE_DICT on rank 0 before each weight broadcast
(finetune_loop.py:222-247).  Here: FSDP2 ``fully_shard`` per decoder layer + the root (so the
tied embedding / lm_head and the final norm live in the root group), RCCL reduce-scatter /
all-gather on MI355X; the lockstep / sentinel protocol already guarantees every rank runs the
same number of forward/backward passes, which FSDP's collectives require.

  * gradient accumulation: ``set_requires_gradient_sync`` — the reduce-scatter runs on the
    boundary micro-batch only (the reference's ``no_sync``), unless
    ``fsdp_sync_every_micro_batch`` trades bandwidth for the unsharded gradient memory;
  * ``grad_reduce: sum`` sets the divide factor to 1 (sum instead of mean), as GradBuckets does;
  * weight snapshot for the actors: parameters are gathered FSDP unit by unit (one all-gather of
    each unit's flat shard, every rank takes part), rank 0 packs them into its bf16 staging buffer
    (weight_update.py);
  * checkpoints: full HF weights on rank 0 (``current/``) and the sharded optimizer state with
    torch.distributed.checkpoint (``training_state/optim/``).
"""

from __future__ import annotations

import json
import logging
import re
from pathlib import Path
from typing import Iterator

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}


SHARDING_MODES = ("auto", "fsdp", "none")


def zero_stage(cfg) -> int | None:
    """The ZeRO stage of the reference's DeepSpeed backend, or None when the config does not use it.
    The reference launches DeepSpeed with conf/deepspeed/<deepspeed_config>.json (launch.py:272-277);
    its configs are named for their stage (deepspeed_stage1, _stage1_bf16, _stage2_bf16, _stage3,
    _stage3_bf16, _stage3_bf16_group4).  A config path to an existing JSON file is read instead."""
    if not cfg.get("use_deepspeed", False):
        return None
    name = str(cfg.get("deepspeed_config", "") or "")
    path = Path(name)
    if path.suffix == ".json" and path.is_file():
        try:
            return int(json.loads(path.read_text()).get("zero_optimization", {}).get("stage", 0))
        except (ValueError, OSError, AttributeError):
            pass
    m = re.search(r"stage[_-]?(\d)", name)
    return int(m.group(1)) if m else 0


def fsdp_requested(cfg, args) -> bool:
    """Sharding asked for explicitly: ``use_fsdp`` or ``finetune.sharding: fsdp``."""
    return bool(cfg.get("use_fsdp", False)) or str(args.get("sharding", "auto")) == "fsdp"


def sharding_mode(cfg, args) -> str:
    """How the trainer lays out the model state over the data-parallel ranks: ``fsdp`` (sharded),
    ``none`` (replicas + a bucketed gradient all-reduce) or ``auto`` (decided once the model is
    built: ``decide_sharding``).  ``finetune.sharding`` (build-only key) picks; its default ``auto``
    follows the reference's backend: ``use_fsdp`` shards; DeepSpeed ZeRO (the reference default,
    ``use_deepspeed: true`` with deepspeed_stage3_bf16, conf/base.yaml:94-96) is ``auto``; plain DDP
    replicates."""
    mode = str(args.get("sharding", "auto"))
    if mode not in SHARDING_MODES:
        raise ValueError(f"finetune.sharding must be one of {SHARDING_MODES}, got {mode!r}")
    if mode != "auto":
        return mode
    if cfg.get("use_fsdp", False):
        return "fsdp"
    return "auto" if zero_stage(cfg) else "none"


def decide_sharding(cfg, args, model, device, world: int, master_weights: bool,
                    device_bytes: int | None = None) -> tuple[bool, str]:
    """(shard?, reason) for the built ``model`` over ``world`` data-parallel ranks.

    Under the reference's ZeRO backend (``sharding_mode`` auto) the model state is what ZeRO
    partitions: stage 3 the parameters, gradients and optimizer state, stages 1/2 the optimizer
    state (and gradients).  MI355X has 288 GB per GPU: a 7B model's whole state with fp32 masters
    (122 GB) fits every rank beside its activations, and replicas then trade ZeRO-3's two
    parameter all-gathers per layer and micro-batch (2 x 15 GB per micro-batch at 7B) for one
    bucketed all-reduce per optimizer step.  So ``auto`` keeps replicas while the replicated plan
    fits the device (finetune/recompute.py: model state + activations, recomputing as needed) and
    shards with FSDP2 — the same partitioning as ZeRO-3 — when it does not (a 32B model: 524 GB of
    state).  Numerically the two layouts give the same update (fp32 masters either way); only the
    summation order of the gradient reduction differs."""
    mode = sharding_mode(cfg, args)
    if mode == "fsdp":  # (also on one rank: the FSDP code path itself, as the reference's FSDP launch)
        return True, "sharding requested (use_fsdp / finetune.sharding=fsdp)"
    if world <= 1:
        return False, "one data-parallel rank: nothing to shard"
    if mode == "none":
        return False, ("replicas (finetune.sharding=none)" if str(args.get("sharding", "auto")) == "none"
                       else "replicas: the reference's backend here is plain DDP (no DeepSpeed, no FSDP)")
    from .recompute import ModelStateTooLarge, plan_gradient_checkpointing

    stage = zero_stage(cfg)
    try:
        plan = plan_gradient_checkpointing(args, model, device, 1, device_bytes, master_weights)
    except ModelStateTooLarge as e:
        return True, f"DeepSpeed ZeRO-{stage} config, replicated model state does not fit ({e}): FSDP over {world} ranks"
    if plan.need_bytes and plan.device_bytes and plan.need_bytes > plan.device_bytes:
        return True, (f"DeepSpeed ZeRO-{stage} config, a replica needs {plan.need_bytes / 1e9:.1f} GB of the device's "
                      f"{plan.device_bytes / 1e9:.1f} GB even with recompute: FSDP over {world} ranks")
    return False, (f"DeepSpeed ZeRO-{stage} config, the replicated model state fits the device "
                   f"({plan.need_bytes / 1e9:.1f} of {plan.device_bytes / 1e9:.1f} GB): replicas + bucketed all-reduce"
                   if plan.need_bytes else f"DeepSpeed ZeRO-{stage} config, device not sized: replicas")


def is_sharded(model) -> bool:
    from torch.distributed.fsdp import FSDPModule

    return isinstance(model, FSDPModule)


def decoder_layers(model) -> list[torch.nn.Module]:
    """The transformer blocks (TRANSFORMER_BASED_WRAP): modules named ``*DecoderLayer``."""
    return [m for m in model.modules() if type(m).__name__.endswith("DecoderLayer")]


def shard_model(model, fsdp_cfg=None, grad_reduce: str = "mean", reshard_after_forward: bool = True,
                keep_gathered: int = 0, master_weights: bool = False):
    """Shard ``model`` in place over the default process group; returns it (an FSDPModule).
    ``keep_gathered``: the last that many decoder layers keep their unsharded parameters from their
    forward to their backward (``reshard_after_forward=False``: one all-gather per step instead of
    two; sized by finetune/recompute.py plan_fsdp_gathering).

    ``master_weights``: the sharded parameters are fp32 — the reference's FSDP mixed precision,
    where accelerate upcasts the bf16-loaded parameters to fp32 in ``prepare``
    (finetune_loop.py:355-396), and DeepSpeed ZeRO-3's fp32 partitions: the optimizer then updates
    fp32 shards with fp32 moments.  Each unit is upcast just before it is sharded (peak: the bf16
    model + one fp32 unit).  Compute stays bf16 (``param_dtype`` bf16: each all-gather casts the
    shards, as the reference's bf16 autocast computes its matmuls); the gradients are
    reduce-scattered in ``fsdp.reduce_dtype`` (the reference's default fp32, conf/base.yaml:97-100)
    into fp32 shards."""
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.fsdp import MixedPrecisionPolicy, fully_shard

    from .model_ops import disable_fused_grad_accumulation, disable_fused_projections

    disable_fused_grad_accumulation()  # FSDP2 owns the unsharded gradients: autograd accumulates them
    disable_fused_projections()  # and re-gathers the weights every forward: no concatenation cache
    dev = next(model.parameters()).device
    mesh = init_device_mesh(dev.type, (dist.get_world_size(),))
    fsdp_cfg = fsdp_cfg or {}
    load = next(model.parameters()).dtype
    master = bool(master_weights) and load == torch.bfloat16
    store = torch.float32 if master else load
    pd = _DTYPES.get(str(fsdp_cfg.get("param_dtype", "")), None)
    rd = _DTYPES.get(str(fsdp_cfg.get("reduce_dtype", "")), None)
    if master:
        pd = load  # compute in the loaded dtype; the fp32 copies are the optimizer's
        rd = rd or torch.float32
    param_dtype = pd if pd not in (None, store) else None
    # FSDP2 reduces in param_dtype when reduce_dtype is None: with fp32 master shards computed in bf16
    # an fp32 reduce must be named even though it equals the storage dtype
    reduce_dtype = rd if rd is not None and (rd != store or param_dtype is not None) else None
    mp = MixedPrecisionPolicy(param_dtype=param_dtype, reduce_dtype=reduce_dtype)
    layers = decoder_layers(model)
    first_gathered = len(layers) - max(0, min(int(keep_gathered), len(layers)))
    for i, layer in enumerate(layers):
        if master:
            layer.to(torch.float32)
        fully_shard(layer, mesh=mesh, mp_policy=mp,
                    reshard_after_forward=reshard_after_forward and i < first_gathered)
    if master:  # the root's own parameters (embedding, lm_head, final norm, a value head)
        for mod in model.modules():
            for name, p in list(mod.named_parameters(recurse=False)):
                if p.dtype == load and not _is_dtensor(p):
                    p.data = p.data.to(torch.float32)
    # the root unit (embedding, final norm, lm_head) stays gathered from its forward to its backward:
    # the label-row lm_head + loss (finetune/rl/fused_linear.py) runs after the root forward on the
    # gathered lm_head weight (the backward needs the unit gathered at once anyway)
    fully_shard(model, mesh=mesh, mp_policy=mp, reshard_after_forward=False)
    if master:
        model._prl_save_dtype = load  # checkpoints keep the loaded dtype (finetune/checkpoints.py)
    for m in [*layers, model]:
        if grad_reduce == "sum":
            m.set_gradient_divide_factor(1.0)
        if "nccl" not in str(dist.get_backend()):  # gloo has no PREMUL_SUM / AVG: plain SUM + a scale
            m.set_force_sum_reduction_for_comms(True)
    logger.info(f"FSDP: {len(layers)} decoder layers + root sharded over {dist.get_world_size()} ranks "
                f"({'fp32 master shards, ' if master else ''}param_dtype {mp.param_dtype}, reduce_dtype "
                f"{mp.reduce_dtype}; the last "
                f"{len(layers) - first_gathered} layers stay gathered from forward to backward)")
    return model


def _is_dtensor(t) -> bool:
    from torch.distributed.tensor import DTensor

    return isinstance(t, DTensor)


def set_kept_gathered(model, keep: int) -> int:
    """At run time: the last ``keep`` decoder layers of a sharded model stay gathered from forward to
    backward, the others reshard after their forward (FSDPModule.set_reshard_after_forward).
    Returns how many layers stay gathered."""
    layers = decoder_layers(model)
    first = len(layers) - max(0, min(int(keep), len(layers)))
    for i, layer in enumerate(layers):
        layer.set_reshard_after_forward(i < first, recurse=False)
    return len(layers) - first


def set_gradient_sync(model, enabled: bool) -> None:
    if is_sharded(model):
        model.set_requires_gradient_sync(enabled)


def fsdp_units(model) -> list[tuple[str, torch.nn.Module, list[tuple[str, torch.nn.Parameter]]]]:
    """The FSDP units of a sharded model (each decoder layer, then the root) with the parameters each
    unit owns: [(unit prefix, unit, [(FQN, parameter)])], nested units' parameters excluded."""
    from torch.distributed.fsdp import FSDPModule

    units = [(name, m) for name, m in model.named_modules() if isinstance(m, FSDPModule)]
    unit_ids = {id(m) for _, m in units}
    out = []
    for prefix, unit in units:
        nested = [n + "." for n, sub in unit.named_modules() if sub is not unit and id(sub) in unit_ids]
        own = []
        for n, p in unit.named_parameters():
            if not any(n.startswith(x) for x in nested):
                own.append((f"{prefix}.{n}" if prefix else n, p))
        out.append((prefix, unit, own))
    out.sort(key=lambda u: u[0] == "")  # decoder layers first, the root (embedding, lm_head) last
    return out


def gather_units(model) -> Iterator[list[tuple[str, torch.Tensor]]]:
    """Yield each FSDP unit's parameters unsharded, [(FQN, full tensor)], one unit at a time: ONE
    all-gather per unit (``FSDPModule.unshard``, the same flat collective FSDP's forward issues;
    ~65 for a 64-layer model instead of one per tensor), resharded when the caller asks for the next
    unit.  The caller's reads of the tensors are enqueued on the current stream before the reshard;
    the freed storage is recorded on that stream, so FSDP's next all-gather cannot reuse it early.
    Every rank must iterate it to the end."""
    stream = torch.cuda.current_stream() if torch.cuda.is_available() else None
    for _, unit, own in fsdp_units(model):
        unit.unshard()
        try:
            # after unshard the modules hold the unsharded parameters under the same names
            full = []
            for n, _ in own:
                mod_name, _, attr = n.rpartition(".")
                mod = model.get_submodule(mod_name) if mod_name else model
                full.append((n, getattr(mod, attr)))
            yield [(n, t.detach()) for n, t in full]
            if stream is not None:
                for _, t in full:
                    if t.is_cuda:
                        t.record_stream(stream)
        finally:
            unit.reshard()


def full_state_dict(model) -> dict:
    """Full (unsharded) CPU state dict on rank 0 (empty elsewhere); collective."""
    from torch.distributed.checkpoint.state_dict import StateDictOptions, get_model_state_dict

    return get_model_state_dict(model, options=StateDictOptions(full_state_dict=True, cpu_offload=True))


def save_optimizer(path, model, optimizer) -> None:
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.state_dict import get_optimizer_state_dict

    dcp.save({"optim": get_optimizer_state_dict(model, optimizer)}, checkpoint_id=str(path))


def load_optimizer(path, model, optimizer) -> None:
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.state_dict import get_optimizer_state_dict, set_optimizer_state_dict

    state = {"optim": get_optimizer_state_dict(model, optimizer)}
    dcp.load(state, checkpoint_id=str(path))
    set_optimizer_state_dict(model, optimizer, state["optim"])
