"""Whether to recompute activations (gradient checkpointing), sized for the device's HBM.

The reference's trainer config turns HF gradient checkpointing on unconditionally
(conf/finetune/base.yaml:44-48, "to reduce memory footprint"; applied by
finetune/checkpoints.py when the model is loaded): every decoder layer's forward runs twice,
about a third more compute per micro-batch.  On a 288 GB MI355X the activations of a whole
packed micro-batch usually fit beside the weights, gradients and optimizer state, and
recomputing them only costs time.  The results are the same either way (the recomputed
forward is the same deterministic kernels on the same inputs).

``finetune.gradient_checkpointing_policy`` (build-only key):
  ``auto`` (default)  keep every layer's activations when the estimate below fits the device;
                      else recompute only as many decoder layers as needed: the last K layers keep
                      their activations (K the largest that fits, from the same estimate with a
                      recomputed layer holding only its input hidden state, plus two layers'
                      worth while one is recomputed: its activations and its backward's
                      temporaries), the others recompute — every layer
                      when K = 0.  The results are the same for every K.
  ``always``          the reference's behaviour: checkpoint whenever gradient_checkpointing is set
``finetune.gradient_checkpointing_keep_layers`` (build-only, optional int): K itself (A/B runs).
``finetune.fsdp_keep_gathered_layers`` (build-only, FSDP only): ``auto`` (default) | an int R.
                      FSDP2 frees each decoder layer's unsharded parameters after its forward and
                      all-gathers them again for its backward (two all-gathers and a reduce-scatter
                      per layer and step).  The last R layers instead stay gathered from their forward
                      to their backward (``reshard_after_forward=False``; they reshard after their
                      backward, which comes first): one all-gather fewer per layer, at R unsharded
                      layers more memory at the start of the backward.  ``auto`` spends what the
                      recompute plan leaves of the device on it (R = spare // a layer's unsharded
                      parameters, after the allocator's rounding) — activations first, since a
                      recompute costs a third of a layer's compute and a re-gather only overlappable
                      communication; ``auto`` needs a sized plan (gradient checkpointing on, a HIP
                      device), else R = 0, FSDP's default.  0 turns it off.

The estimate is deliberately conservative (upper bounds, measured against the trainer probes'
peak memory in DESIGN.md): model state = parameters x (weight + gradient + two AdamW moments; with
fp32 master weights, the reference default's optimizer state, 16 B per parameter), divided by the
FSDP world when sharded — a model state that alone exceeds the device raises ModelStateTooLarge; activations = the tensors a patched Qwen2-style decoder
layer keeps for its backward per token (the normed inputs of the q/k/v and gate/up GEMMs, q, k,
v, the attention output, the residual stream, gate, up and the SwiGLU output), times
``seq_length`` tokens, times the layers, times a 1.25 allowance for backward temporaries; one
label-row logits chunk; the build's own long-lived buffers (the fused gate/up weight cache,
2 I x H per layer when finetune/model_ops.py fuses the projection at this micro-batch size and the
model is neither FSDP-sharded nor flat-homed — with flat parameters the fused weight is a view; the lm_head weight gradient's staging, [V, H] bf16 from the single-chunk
GEMM or an fp32 accumulator over several chunks, finetune/rl/fused_linear.py); under FSDP, the
larger of its two unsharded working sets (fsdp_transient_bytes: the start of the backward with the
logits' gradient, the root unit gathered, the lm_head's unsharded gradient and two decoder layers;
the root's reduce-scatter with 3 x the root); each term sized with the device allocator's own
rounding at the micro-batch's largest shapes (devalloc.round_size: the parameters' per-tensor
blocks, the [T, H] / [T, I] / [T, 2I] / [T, kv] activations, the logits chunk); 5 % of the device
plus 4 GiB of headroom.
Checked against the measured steady-state peak of a 32B-shaped FSDP model (tests/test_fsdp_32b_gpu.py:
estimate without the headroom between 1x and 1.3x the measured peak).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass

import torch

logger = logging.getLogger(__name__)

ACT_ALLOWANCE = 1.25
HEADROOM_FRAC = 0.05
HEADROOM_BYTES = 4 << 30


@dataclass
class RecomputePlan:
    checkpoint: bool
    reason: str
    state_bytes: int = 0
    activation_bytes: int = 0
    logits_bytes: int = 0
    buffer_bytes: int = 0
    device_bytes: int = 0
    need_bytes: int = 0  # the terms after the allocator's rounding, plus the headroom
    keep_layers: int = -1  # checkpoint: the last keep_layers decoder layers keep their activations
    gathered_layers: int = 0  # FSDP: the last gathered_layers decoder layers stay unsharded forward -> backward
    gathered_bytes: int = 0  # what they hold beyond FSDP's default (in need_bytes)

    def as_dict(self) -> dict:
        return {"checkpoint": self.checkpoint, "reason": self.reason, "state_gb": round(self.state_bytes / 1e9, 2),
                "activation_gb": round(self.activation_bytes / 1e9, 2), "logits_gb": round(self.logits_bytes / 1e9, 2),
                "buffer_gb": round(self.buffer_bytes / 1e9, 2), "device_gb": round(self.device_bytes / 1e9, 2),
                "need_gb": round(self.need_bytes / 1e9, 2), "keep_layers": self.keep_layers,
                "gathered_layers": self.gathered_layers, "gathered_gb": round(self.gathered_bytes / 1e9, 2)}


def activation_bytes_per_token(config, dtype_bytes: int = 2) -> int:
    """Bytes one token keeps for the backward across every decoder layer (upper bound)."""
    H = int(config.hidden_size)
    inter = int(getattr(config, "intermediate_size", 4 * H))
    heads = int(getattr(config, "num_attention_heads", 1))
    kv_heads = int(getattr(config, "num_key_value_heads", None) or heads)
    head_dim = int(getattr(config, "head_dim", None) or H // heads)
    kv = kv_heads * head_dim
    layers = int(config.num_hidden_layers)
    # residual in, normed (attention), q, attention out, residual mid, normed (MLP): 6 H;
    # k, v: 2 kv; gate, up, SwiGLU out: 3 I; per-row statistics (rstd, lse) are negligible
    per_layer = 6 * H + 2 * kv + 3 * inter
    return per_layer * layers * dtype_bytes


def build_buffer_bytes(config, seq: int, chunk: int, shard_world: int, dtype_bytes: int = 2,
                       flat_params: bool = False) -> int:
    """Long-lived buffers of the build's fused paths at this micro-batch size (upper bound).
    ``flat_params``: the parameters live in one flat buffer (finetune.flat_parameters), so the fused
    gate / up weight is a view of it, not a cached concatenation."""
    from . import model_ops

    H = int(config.hidden_size)
    inter = int(getattr(config, "intermediate_size", 4 * H))
    layers = int(config.num_hidden_layers)
    vocab = int(getattr(config, "vocab_size", 0))
    out = 0
    if shard_world <= 1 and model_ops._FUSED_GATE_UP and seq <= model_ops._FUSED_GATE_UP_MAX_ROWS and not flat_params:
        out += 2 * inter * H * layers * dtype_bytes  # cat(Wg, Wu) per layer (_fused_weight)
    if shard_world <= 1 and getattr(model_ops, "_FUSED_QKV", False):
        heads = int(getattr(config, "num_attention_heads", 1))
        kv = int(getattr(config, "num_key_value_heads", None) or heads) * (H // heads)
        out += (H + 2 * kv) * H * layers * dtype_bytes
    # lm_head dW: bf16 from one GEMM (one chunk) or an fp32 accumulator (several chunks); under
    # FSDP the one-chunk dW becomes the root unit's unsharded lm_head gradient, counted in
    # fsdp_transient_bytes
    if shard_world <= 1:
        out += vocab * H * (dtype_bytes if seq <= chunk else 4)
    return out


def compute_bytes(model, param_bytes: int) -> int:
    """Bytes per element of the tensors the model computes with: the parameters' own size, except
    for a model sharded with fp32 master shards (finetune/sharding.py), whose gathered weights and
    activations are in the loaded dtype (``_prl_save_dtype``, bf16)."""
    dt = getattr(model, "_prl_save_dtype", None)
    return min(param_bytes, torch.empty((), dtype=dt).element_size()) if dt is not None else param_bytes


def fsdp_unit_bytes(model) -> tuple[int, int]:
    """(root unit, largest decoder-layer unit) parameter bytes of an FSDP-wrapped model (or of the
    model that will be wrapped): the root holds the embedding, lm_head and final norm."""
    from .sharding import decoder_layers

    def nbytes(params) -> int:  # unsharded, in the compute dtype (what an all-gather materialises)
        return sum(p.numel() * compute_bytes(model, p.element_size()) for p in params)

    layers = decoder_layers(model)
    layer = max((nbytes(m.parameters()) for m in layers), default=0)
    root = nbytes(model.parameters()) - sum(nbytes(m.parameters()) for m in layers)
    return root, layer


def fsdp_transient_bytes(model, shard_world: int, act: int, logits: int, head_grad: int,
                         reduce_factor: int = 1) -> int:
    """FSDP2's unsharded working set beyond the activations (upper bound), the larger of its two
    peaks in a step: (a) the start of the backward — every activation, the logits' gradient
    (``logits``: the full-logits loss head writes it beside the logits; 0 for the label-row head,
    which writes it in place), the root unit gathered, the lm_head's unsharded gradient and a
    decoder layer in use plus the next prefetched; (b) the root's
    reduce-scatter at the end of the backward — the root gathered, its unsharded gradients and the
    reduce-scatter input FSDP copies them into (3 x the root).  ``reduce_factor``: the reduce dtype's
    bytes over the compute dtype's; with 2 (fp32 master shards computed in bf16, reduced in fp32) the
    input is twice the root and the fp32 output shard exists beside it (the 32B-shaped GPU test's
    peak, 34.4 GB per rank, needs all of them: tests/test_fsdp_32b_gpu.py).  Returned as that peak
    minus ``act`` (the plan adds the activations itself).  0 when not sharded."""
    if shard_world <= 1:
        return 0
    root, layer = fsdp_unit_bytes(model)
    start = act + logits + root + head_grad + 2 * layer
    end = (2 + reduce_factor) * root + (reduce_factor * root // shard_world if reduce_factor > 1 else 0)
    return max(start, end) - act


def gathered_layer_bytes(model) -> int:
    """The largest decoder layer's unsharded parameters as FSDP2 allocates them (one block per
    parameter, reused across gathers) after the device allocator's rounding."""
    from ..devalloc import round_size
    from .sharding import decoder_layers

    return max((sum(round_size(p.numel() * compute_bytes(model, p.element_size())) for p in m.parameters())
                for m in decoder_layers(model)), default=0)


def plan_fsdp_gathering(args, model, plan: RecomputePlan, shard_world: int) -> RecomputePlan:
    """``plan`` with ``gathered_layers`` / ``gathered_bytes`` set (finetune.fsdp_keep_gathered_layers,
    module docstring); ``need_bytes`` grows by the gathered bytes."""
    policy = args.get("fsdp_keep_gathered_layers", "auto")
    if policy != "auto" and (isinstance(policy, bool) or not isinstance(policy, int) or policy < 0):
        raise ValueError(f"fsdp_keep_gathered_layers must be 'auto' or an int >= 0, got {policy!r}")
    if int(shard_world) <= 1:
        return plan
    from .sharding import decoder_layers

    L = len(decoder_layers(model))
    per = gathered_layer_bytes(model)
    if policy == "auto":
        if plan.need_bytes <= 0 or plan.device_bytes <= 0 or per <= 0:
            return plan  # unsized: FSDP's default
        n = min(L, max(0, (plan.device_bytes - plan.need_bytes) // per))
    else:
        n = min(L, int(policy))
    plan.gathered_layers, plan.gathered_bytes = int(n), int(n) * per
    if plan.need_bytes > 0:
        plan.need_bytes += plan.gathered_bytes
    return plan


class ModelStateTooLarge(MemoryError):
    """The model state alone (weights, gradients, optimizer state) does not fit one device: no
    recompute plan can help; the model must be sharded (FSDP)."""


def state_bytes_per_param(param_bytes: int, master_weights: bool) -> int:
    """Model-state bytes per parameter: weight + gradient + the two AdamW moments in the parameter
    dtype (pure bf16: 8 B), or with fp32 master weights (finetune/optim.py; an FSDP-sharded model
    keeps its sharded parameters and gradients in fp32 instead, finetune/sharding.py) a bf16
    weight + gradient and an fp32 master + two fp32 moments: 16 B."""
    if master_weights and param_bytes == 2:
        return 16
    return 4 * param_bytes


def model_state_bytes(model, shard_world: int = 1, master_weights: bool = True) -> int:
    params = list(model.parameters())
    pbytes = params[0].element_size() if params else 2
    return state_bytes_per_param(pbytes, master_weights) * sum(p.numel() for p in params) // max(1, int(shard_world))


def _master_weights_of(args, master_weights: bool | None) -> bool:
    if master_weights is not None:
        return bool(master_weights)
    mode = args.get("master_weights", "auto")
    return mode if isinstance(mode, bool) else True  # auto: the reference default's (masters)


def check_model_state_fits(model, device: torch.device, shard_world: int = 1, master_weights: bool = True,
                           device_bytes: int | None = None) -> None:
    """Raise ModelStateTooLarge when the model state alone exceeds the device (less the plan's
    headroom); silently returns when the device cannot be sized (not a HIP device, no size given)."""
    if device_bytes is None:
        if device.type != "cuda":
            return
        device_bytes = int(torch.cuda.get_device_properties(device).total_memory)
    state = model_state_bytes(model, shard_world, master_weights)
    room = int(device_bytes) - int(HEADROOM_FRAC * int(device_bytes)) - HEADROOM_BYTES
    if state > room:
        n = sum(p.numel() for p in model.parameters())
        raise ModelStateTooLarge(
            f"model state {state / 1e9:.1f} GB ({n / 1e9:.2f} B parameters x "
            f"{state_bytes_per_param(next(model.parameters()).element_size(), master_weights)} B"
            f"{'' if shard_world <= 1 else f' / {shard_world} ranks'}) exceeds the device's "
            f"{room / 1e9:.1f} GB usable: shard the model (use_fsdp=true, finetune.sharding=fsdp, or the "
            "reference's default DeepSpeed ZeRO-3 config with finetune.sharding=auto) over more ranks")


def plan_gradient_checkpointing(args, model, device: torch.device, shard_world: int = 1,
                                device_bytes: int | None = None, master_weights: bool | None = None) -> RecomputePlan:
    """The decision for ``model`` (already built) under the trainer config ``args``;
    ``device_bytes``: the device's memory (default: queried from the HIP device); ``master_weights``:
    the optimizer keeps fp32 masters (default: ``args.master_weights``, ``auto`` counting them).
    Under FSDP (``shard_world`` > 1) also how many decoder layers stay gathered
    (plan_fsdp_gathering).  Raises ModelStateTooLarge when the model state alone cannot fit."""
    master = _master_weights_of(args, master_weights)
    check_model_state_fits(model, device, shard_world, master, device_bytes)
    return plan_fsdp_gathering(args, model, _plan_recompute(args, model, device, shard_world, device_bytes, master),
                               shard_world)


def _plan_recompute(args, model, device: torch.device, shard_world: int, device_bytes: int | None,
                    master: bool = True) -> RecomputePlan:
    if not args.get("gradient_checkpointing", False):
        return RecomputePlan(False, "gradient_checkpointing is off")
    policy = str(args.get("gradient_checkpointing_policy", "auto"))
    if policy not in ("auto", "always"):
        raise ValueError(f"gradient_checkpointing_policy must be 'auto' or 'always', got {policy!r}")
    forced = args.get("gradient_checkpointing_keep_layers", None)
    if policy == "always" and forced is None:
        return RecomputePlan(True, "policy always (the reference's behaviour)", keep_layers=0)
    if device_bytes is None and device.type != "cuda":
        if forced is not None:  # K stated by the config: nothing to size
            L = int(getattr(getattr(model, "config", None), "num_hidden_layers", 0) or 0)
            keep = max(0, min(int(forced), L))
            return RecomputePlan(keep < L, f"keep_layers {keep} of {L} (finetune.gradient_checkpointing_keep_layers)",
                                 keep_layers=keep if keep < L else -1)
        return RecomputePlan(True, "not a HIP device: the reference's behaviour", keep_layers=0)
    seq = args.get("seq_length")
    config = getattr(model, "config", None)
    if not seq or config is None or not hasattr(config, "hidden_size") or not hasattr(config, "num_hidden_layers"):
        return RecomputePlan(True, "no seq_length / decoder shape to size the activations: the reference's behaviour",
                             keep_layers=0)
    total = int(device_bytes) if device_bytes is not None else int(torch.cuda.get_device_properties(device).total_memory)
    params = list(model.parameters())
    n = sum(p.numel() for p in params)
    pbytes = params[0].element_size() if params else 2
    sw = max(1, int(shard_world))
    L = int(config.num_hidden_layers)
    # weight + gradient + exp_avg + exp_avg_sq in the parameter dtype, or with fp32 masters
    # (PrlAdamW master_weights / FSDP's fp32 shards) 16 B per parameter
    state = state_bytes_per_param(pbytes, master) * n // sw
    pbytes = compute_bytes(model, pbytes)  # activations, logits and gathered weights: the compute dtype
    act = int(ACT_ALLOWANCE * int(seq) * activation_bytes_per_token(config, pbytes))
    vocab = int(getattr(config, "vocab_size", 0))
    rl = args.get("rl", None) or {}
    chunk = min(int(seq), int(rl.get("lm_head_chunk_rows", 65536) or 65536))  # RLConfig default
    fused = bool(rl.get("fused_lm_head", True))  # the label-row head writes dlogits in place
    logits = chunk * vocab * pbytes
    head = 0 if getattr(config, "tie_word_embeddings", False) else vocab * int(config.hidden_size) * pbytes
    # the device allocator's size rounding (devalloc.py) at the largest shapes of the micro-batch
    # (rounding is monotonic: shorter micro-batches round to no more)
    from ..devalloc import round_size, rounded_factor

    H = int(config.hidden_size)
    inter = int(getattr(config, "intermediate_size", 4 * H))
    heads = int(getattr(config, "num_attention_heads", 1))
    kvw = int(getattr(config, "num_key_value_heads", None) or heads) * int(getattr(config, "head_dim", None) or H // heads)
    f_act = max(rounded_factor(int(seq) * w * pbytes) for w in (H, inter, 2 * inter, kvw))
    f_logits = rounded_factor(logits) if logits else 1.0
    sizes = [p.numel() * pbytes // sw for p in params]
    f_state = (sum(round_size(b) for b in sizes if b) / max(1, sum(sizes))) if sizes else 1.0
    act_layer = act // max(1, L)
    # the loop re-homes a non-FSDP bf16 model into one flat buffer (finetune_loop.py, flat_parameters)
    flat = sw <= 1 and pbytes == 2 and bool(args.get("flat_parameters", True))
    saved_input = round_size(int(seq) * H * pbytes)  # what a recomputed layer keeps: its input

    def need_for(keep: int) -> tuple[int, int, int]:
        """(bytes compared with the device, activation bytes, buffer bytes) when the last ``keep``
        layers keep their activations and the others recompute."""
        # + the layer being recomputed and its backward's own temporaries (measured on an 8-layer
        # 7B model at K = 4: one layer's worth was 5 % short, tests/test_recompute_gpu.py)
        a = act if keep >= L else keep * act_layer + 2 * act_layer
        a_bytes = int(a * f_act) + (0 if keep >= L else (L - keep) * saved_input)
        buffers = build_buffer_bytes(config, int(seq), chunk, int(shard_world), pbytes, flat) + \
            fsdp_transient_bytes(model, int(shard_world), a, 0 if fused else logits, head,
                                 reduce_factor=2 if master and pbytes == 2 else 1)
        need = int(state * f_state) + a_bytes + int(logits * f_logits) + \
            int(buffers * max(f_state, f_act, f_logits)) + int(HEADROOM_FRAC * total) + HEADROOM_BYTES
        return need, a_bytes, buffers

    if forced is not None:
        keep = max(0, min(int(forced), L))
        need, _, buffers = need_for(keep)
        return RecomputePlan(keep < L, f"keep_layers {keep} of {L} (finetune.gradient_checkpointing_keep_layers)",
                             state, act, logits, buffers, total, need, keep if keep < L else -1)
    need, _, buffers = need_for(L)
    if need <= total:
        return RecomputePlan(False, "activations fit: no recompute", state, act, logits, buffers, total, need)
    keep = L - 1
    while keep > 0 and need_for(keep)[0] > total:
        keep -= 1
    need_k, _, buffers_k = need_for(keep)
    if keep == 0 and need_k > total:
        raise ModelStateTooLarge(
            f"the model does not fit the device even with every layer recomputed: {need_k / 1e9:.1f} GB needed "
            f"(model state {state / 1e9:.1f} GB{'' if sw <= 1 else f' per rank over {sw}'}) of {total / 1e9:.1f} GB: "
            "shard the model (use_fsdp=true, finetune.sharding=fsdp) over more ranks, or shorten seq_length")
    reason = (f"activations of the last {keep} of {L} layers fit: {L - keep} recompute" if keep > 0
              else "activations do not fit: recompute")
    return RecomputePlan(True, reason, state, act, logits, buffers_k, total, need_k, keep)
