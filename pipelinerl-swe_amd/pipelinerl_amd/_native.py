"""ctypes binding of libprl_hip.so (C ABI in include/prl_hip.h).

There is no CPU fallback: if the HIP library cannot be loaded, every entry point raises.
Device scratch the kernels need (the loss head's workspace, the SwiGLU chunk counter) is allocated
here, per (device, stream), as torch tensors the library is handed: the library holds none.
"""

from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["PRL_LIB"]) if os.environ.get("PRL_LIB") else _PKG / "libprl_hip.so"
HEADER_PATH = _PKG.parents[1] / "include" / "prl_hip.h"

ABI_VERSION = 3
PRL_F32, PRL_BF16 = 0, 1
PRL_PPO, PRL_REINFORCE = 0, 1

# statistic indices, in enum PrlStat order (checked against the header and the library)
STATS = [
    "LOSS_SUM", "VALUE_LOSS", "REWARD", "ENTROPY", "OLD_LP", "NEW_LP", "REF_LP", "ADVANTAGE", "KL",
    "POLICY_LOSS", "SURR1", "SURR2", "RATIO", "RATIO_SUM", "RATIO_SQ_SUM", "RATIO_REF_NEW",
    "RATIO_REF_OLD", "CLAMP_REF_NEW", "CLAMP_NEW_OLD", "TOKEN_WEIGHT", "VALUE_MEAN", "VALUE_MSE",
    "NUM_NANS", "NUM_OUT", "BAD_LP", "BAD_LRRN", "BAD_KL", "BAD_GT", "BAD_ID", "MAX_REWARD",
    "MIN_REWARD", "MAX_ADV", "MIN_ADV", "MAX_KL", "MIN_KL", "MAX_W", "MIN_W", "MAX_VALUE",
    "MIN_VALUE",
]
S = {name: i for i, name in enumerate(STATS)}
NSTAT = len(STATS)


class PrlGrpoBatch(ctypes.Structure):
    _fields_ = [
        ("logits", c_void_p), ("logits_dtype", c_int32), ("_pad0", c_int32),
        ("B", c_int64), ("L", c_int64), ("V", c_int64), ("ld", c_int64),
        ("input_ids", c_void_p), ("labels", c_void_p), ("rewards", c_void_p),
        ("advantages", c_void_p), ("ref_logprobs", c_void_p), ("old_logprobs", c_void_p),
        ("group_tokens", c_void_p), ("num_labels", c_void_p), ("overflow", c_void_p),
        ("values", c_void_p),
    ]


class PrlGrpoParams(ctypes.Structure):
    _fields_ = [
        ("policy_loss", c_int32), ("use_advantages", c_int32), ("relu_log_p_weights", c_int32),
        ("group_normalization", c_int32), ("overlong_filtering", c_int32), ("write_grad", c_int32),
        ("epsilon", c_float), ("kl_coef", c_float), ("entropy_coef", c_float),
        ("clamp_log_ratio", c_float), ("temperature", c_float), ("batch_size", c_float),
        ("value_loss_coef", c_float), ("grad_scale", c_float), ("pair_spin_ticks", c_int32), ("f32_rows", c_int32),
    ]


class PrlGrpoOutputs(ctypes.Structure):
    _fields_ = [
        ("new_logprobs", c_void_p), ("entropy", c_void_p), ("lse", c_void_p),
        ("token_loss", c_void_p), ("g_lp", c_void_p), ("g_h", c_void_p), ("row_max", c_void_p),
        ("row_log2sum", c_void_p), ("dvalues", c_void_p),
        ("dlogits", c_void_p), ("stats", c_void_p),
    ]


_SIGNATURES = {
    "prl_abi_version": (c_int, []),
    "prl_error_string": (c_char_p, [c_int]),
    "prl_grpo_workspace_bytes": (c_int, [c_int, POINTER(c_size_t)]),
    "prl_grpo_forward": (c_int, [POINTER(PrlGrpoBatch), POINTER(PrlGrpoParams), POINTER(PrlGrpoOutputs),
                                 c_void_p, c_size_t, c_void_p]),
    "prl_grpo_backward": (c_int, [POINTER(PrlGrpoBatch), POINTER(PrlGrpoParams), c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "prl_grpo_forward_rows": (c_int, [POINTER(PrlGrpoBatch), POINTER(PrlGrpoParams), c_void_p, c_int64,
                                      POINTER(PrlGrpoOutputs), c_void_p, c_size_t, c_void_p]),
    "prl_grpo_stats": (c_int, [POINTER(PrlGrpoBatch), POINTER(PrlGrpoParams), POINTER(PrlGrpoOutputs),
                               c_void_p, c_size_t, c_void_p]),
    "prl_grpo_nstat": (c_int, []),
    "prl_flatten_bf16": (c_int, [POINTER(c_void_p), POINTER(c_int32), POINTER(c_int64), POINTER(c_int64),
                                 c_int32, c_void_p, c_void_p]),
    "prl_unflatten_bf16": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_int32), POINTER(c_int64),
                                   POINTER(c_int64), c_int32, c_void_p]),
    "prl_grad_scale_bf16": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p]),
    "prl_paced_read": (c_int, [c_void_p, c_int64, c_double, c_int32, c_void_p, c_void_p]),
    "prl_grpo_pair_fallbacks": (c_int, [c_void_p, c_size_t, c_void_p, POINTER(ctypes.c_uint64)]),
    "prl_adamw_step": (c_int, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                               c_double, c_double, c_double, c_double, c_double, c_void_p, c_void_p]),
    "prl_adamw_master_step": (c_int, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_int32, c_double, c_double, c_double, c_double, c_double, c_void_p,
                                      c_void_p]),
    "prl_grad_sqnorm": (c_int, [POINTER(c_void_p), POINTER(c_int32), POINTER(c_int64), c_int32,
                                POINTER(c_double), c_void_p, c_size_t, c_void_p]),
    "prl_rmsnorm_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_float, c_void_p]),
    "prl_rmsnorm_workspace_bytes": (c_int, [c_int64, POINTER(c_size_t)]),
    "prl_rmsnorm_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                     c_int64, c_int64, c_void_p]),
    "prl_add_rmsnorm_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                        c_float, c_void_p]),
    "prl_add_rmsnorm_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_size_t, c_int64, c_int64, c_void_p]),
    "prl_swiglu_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "prl_swiglu_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "prl_swiglu_forward_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                                        c_void_p]),
    "prl_swiglu_backward_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                                         c_int64, c_int64, c_int64, c_int64, c_void_p]),
    "prl_rope_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                 c_int32, c_int32, c_void_p]),
    "prl_rope_forward_strided": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                         c_int32, c_int32, c_int64, c_int64, c_void_p]),
    "prl_rope_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                  c_int32, c_int32, c_void_p]),
    "prl_attn_bwd_preprocess": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_void_p,
                                        c_int64, c_int32, c_int32, c_void_p]),
    "prl_attn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_int32,
                             c_int32, c_int32, c_float, c_void_p]),
    "prl_attn_bwd_delta": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p]),
    "prl_attn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                             c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_float,
                             c_void_p]),
    "prl_attn_bwd_split": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                   c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_float, c_void_p]),
}

_lib = None
_SCRATCH: dict[tuple, object] = {}


def stream_scratch(kind: str, nbytes: int, device, stream: int):
    """A zero-filled uint8 device tensor of ``nbytes`` for ``kind`` on (device, stream): the caller-owned
    scratch of include/prl_hip.h (one stream at a time per workspace).  Cached: torch draws its
    streams from fixed pools, so the keys stay few."""
    import torch

    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (kind, idx, int(stream or 0))
    t = _SCRATCH.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.zeros(max(1, nbytes), dtype=torch.uint8, device=torch.device("cuda", idx))
        _SCRATCH[key] = t
    return t


class PrlError(RuntimeError):
    pass


def header_symbols() -> list[str]:
    """Function names declared in include/prl_hip.h."""
    text = HEADER_PATH.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(prl_\w+)\s*\(", text, flags=re.M)))


def load():
    """Load the HIP library (building it first if a compiler is present and it is stale)."""
    global _lib
    if _lib is not None:
        return _lib
    if (not LIB_PATH.exists() or os.environ.get("PRL_REBUILD")) and not os.environ.get("PRL_LIB"):
        try:
            from . import _build
            _build.build()
        except Exception as e:  # no hipcc on this machine and no prebuilt library
            raise PrlError(f"libprl_hip.so is missing and could not be built: {e}") from e
    try:
        lib = ctypes.CDLL(str(LIB_PATH))
    except OSError as e:
        raise PrlError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.prl_abi_version() != ABI_VERSION:
        raise PrlError(f"libprl_hip.so has ABI {lib.prl_abi_version()}, binding expects {ABI_VERSION}: rebuild it")
    if lib.prl_grpo_nstat() != NSTAT:
        raise PrlError(f"libprl_hip.so has {lib.prl_grpo_nstat()} statistics, binding expects {NSTAT}")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().prl_error_string(rc).decode()
        raise PrlError(f"{what} failed: {msg} (code {rc})")
