"""Device caching-allocator settings for the trainer loop.

Packed micro-batches differ in length from one to the next (the packer fills up to
``seq_length``, finetune/packing.py), so every large per-micro-batch tensor (the saved
activations, the label-row logits chunk [R, V], the attention workspaces) is requested at a new
size each time.  PyTorch's caching allocator serves a request only from a cached block at least as
large, so each new high-water length allocates a fresh block and the previous one stays cached:
the cache fills the device with near-duplicate blocks, and once a request no longer fits, the
allocator synchronises the device, frees every cached block and allocates them again.  On the
1.5B loop at 64 k-token packing that one retry costs ≈5 s (a 6.3 s step instead of 1.3 s):
306.8 GB reserved for 163.5 GB allocated (profiles/r04_loop_alloc_ab.jsonl).  Rounding request
sizes up to 4 subdivisions per power of two lets a cached block serve every nearby length: no
retry, 216.5 GB reserved, 106 k tokens/s steady over the same six steps instead of 59 k
(4 divisions everywhere; the default below measured the same way in that file).
(``expandable_segments``, the usual remedy, is not supported by the ROCm allocator of this
torch build: it warns and ignores it.)

Rounding costs memory: a block is up to 1/d larger than its request (d divisions).  The default
rounds requests under 512 MB (parameters, their gradients and AdamW moments, most activations) to
16 divisions and larger ones (the logits chunk, long activations, the flat parameter buffer) to 4,
and the gradient-checkpointing plan multiplies its estimate by ``rounding_allowance()``
(finetune/recompute.py).

``finetune.allocator_settings`` (build-only key; default ``DEFAULT_SETTINGS``; empty or null keeps
torch's defaults).  Settings the user exports in ``PYTORCH_HIP_ALLOC_CONF`` /
``PYTORCH_CUDA_ALLOC_CONF`` win: nothing is changed then.
"""

from __future__ import annotations

import logging
import os
import re

import torch

logger = logging.getLogger(__name__)

DEFAULT_SETTINGS = "roundup_power2_divisions:[512:16,>:4]"
ENV_KEYS = ("PYTORCH_HIP_ALLOC_CONF", "PYTORCH_CUDA_ALLOC_CONF")
_applied: str | None = None  # what configure_device_allocator set in this process


def divisions(settings: str | None) -> list[int]:
    """The division counts a ``roundup_power2_divisions`` setting names: ``N`` or the per-interval
    list ``[<MB>:N, ..., >:N]`` ([] when the setting is absent)."""
    m = re.search(r"roundup_power2_divisions:(\[[^\]]*\]|\d+)", settings or "")
    if not m:
        return []
    v = m.group(1)
    if v.startswith("["):
        return [int(x.rsplit(":", 1)[1]) for x in v[1:-1].split(",") if ":" in x]
    return [int(v)]


def rounding_allowance() -> float:
    """Upper bound of a block's size over its request under the settings in force (ours, else the
    user's environment): 1 + 1/d for the smallest division count d > 1 (1.0: no rounding; a count
    of 1 or 0 leaves sizes unrounded)."""
    src = _applied or next((os.environ[k] for k in ENV_KEYS if os.environ.get(k)), None)
    ds = [d for d in divisions(src) if d > 1]
    return 1.0 + 1.0 / min(ds) if ds else 1.0


def _set_allocator_settings(settings: str) -> None:
    fn = getattr(torch._C, "_accelerator_setAllocatorSettings", None)  # torch >= 2.9's name
    (fn or torch.cuda.memory._set_allocator_settings)(settings)


def configure_device_allocator(settings: str | None = DEFAULT_SETTINGS) -> str | None:
    """Apply ``settings`` to the device caching allocator (future allocations only; safe after
    device initialisation).  Returns what was applied, or None when nothing was (no settings, no
    HIP device, or the user's own allocator environment)."""
    if not settings or not torch.cuda.is_available():
        return None
    user = [k for k in ENV_KEYS if os.environ.get(k)]
    if user:
        logger.info("device allocator: keeping %s=%s", user[0], os.environ[user[0]])
        return None
    global _applied
    _set_allocator_settings(str(settings))
    _applied = str(settings)
    logger.info("device allocator: %s", settings)
    return str(settings)
