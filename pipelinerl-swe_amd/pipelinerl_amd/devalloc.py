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
16 divisions and larger ones (the logits chunk, long activations, the flat parameter buffer) to 4.
The gradient-checkpointing plan (finetune/recompute.py) sizes each of its terms with the
allocator's own rounding (``round_size``) at the micro-batch's largest shapes — rounding is
monotonic, so shorter micro-batches never round above them; a flat 1 + 1/d allowance
(``rounding_allowance``) flipped the 32B FSDP plan at 8 ranks to recomputing every layer.

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


_MB = 1 << 20
_INTERVALS = 16  # PyTorch's per-power-of-two division table: [< 2 MiB, < 4 MiB, ..., >= 32 GiB]


def division_table(settings: str | None) -> list[int]:
    """The caching allocator's divisions per power-of-two size interval under ``settings`` (index i:
    sizes in [2^(20+i), 2^(21+i)), index 0 also below, the last also above), following PyTorch's
    parser: ``N`` fills every interval; ``[<MB>:N, ..., >:N]`` fills up to log2(MB) with each
    count and the rest with the ``>`` count.  All zeros: no rounding."""
    table = [0] * _INTERVALS
    m = re.search(r"roundup_power2_divisions:(\[[^\]]*\]|\d+)", settings or "")
    if not m:
        return table
    v = m.group(1)
    if not v.startswith("["):
        return [int(v)] * _INTERVALS
    last = 0
    for item in v[1:-1].split(","):
        if ":" not in item:
            continue
        key, n = item.rsplit(":", 1)
        n = int(n)
        if key.strip() == ">":
            table[last:] = [n] * (_INTERVALS - last)
        else:
            idx = min(max(int(key).bit_length() - 1, 0), _INTERVALS - 1)
            table[last:idx] = [n] * (idx - last)
            last = idx
    return table


def _in_force() -> str | None:
    return _applied or next((os.environ[k] for k in ENV_KEYS if os.environ.get(k)), None)


def round_size(nbytes: int, settings: str | None = None) -> int:
    """The block the caching allocator serves an ``nbytes`` request with (PyTorch's round_size:
    512-B granules, or the next of ``d`` equal steps between two powers of two when the request's
    interval has d > 1 divisions and exceeds 512·d bytes).  ``settings``: the settings in force by default."""
    n = int(nbytes)
    if n < 512:
        return 512
    table = division_table(settings if settings is not None else _in_force())
    d = table[min(max(n.bit_length() - 1 - 20, 0), _INTERVALS - 1)]
    if d > 1 and n > 512 * d:
        if n & (n - 1) == 0:
            return n
        floor = 1 << (n.bit_length() - 1)
        step = floor >> (d.bit_length() - 1)
        if step == 0:
            return floor << 1
        base = n & ~(step - 1)
        return n if base == n else base + step
    return -(-n // 512) * 512


def rounded_factor(nbytes: int, settings: str | None = None) -> float:
    """round_size(nbytes) / nbytes (1.0 for an empty request)."""
    return round_size(nbytes, settings) / nbytes if nbytes > 0 else 1.0


def rounding_allowance() -> float:
    """Upper bound of a block's size over its request under the settings in force (ours, else the
    user's environment): 1 + 1/d for the smallest division count d > 1 (1.0: no rounding; a count
    of 1 or 0 leaves sizes unrounded)."""
    ds = [d for d in divisions(_in_force()) if d > 1]
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
