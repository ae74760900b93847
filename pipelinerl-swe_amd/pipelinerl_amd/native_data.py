"""ctypes binding of libprl_data.so (C ABI in include/prl_data.h): the trainer's input path in
native code.

* ``decode_document`` / ``decode_batch``: one training_data stream line (a JSON micro-batch,
  pipelinerl/streams.py:238-277) into tensors, the numeric arrays decoded by C++ straight into
  (optionally pinned) tensor storage with the GIL released, in parallel over fields.  Same
  values, dtypes and shapes as ``json.loads`` + the PipelineBatchEncoding validators
  (pipelinerl/finetune/types.py:48-117: numpy.asarray then torch.as_tensor); an array the
  native path cannot take (ragged, strings, bools, ints beyond int64) is handed to ``json`` so
  the Python path's behaviour and errors apply.
* ``encode_document``: the writer side, byte-identical to ``streams.dumps`` (Python's float
  repr, NaN / Infinity as json writes them).
* ``rl_group_stats`` / ``collate_arrays``: populate_rl_data's group statistics
  (rl/__init__.py:408-416, pandas' Kahan mean and Welford std) and collate_packed's token
  layout (data.py:215-279) over flat arrays.

There is no silent fallback to a Python implementation of these functions: if the library is
missing and cannot be built, ``load()`` raises.
"""

from __future__ import annotations

import ctypes
import json
import math
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p
from pathlib import Path
from typing import Any

import numpy as np
import torch

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libprl_data.so"
HEADER_PATH = _PKG.parents[1] / "include" / "prl_data.h"
ABI = 1
MAX_DIMS = 8
DT_I64, DT_I32, DT_F32, DT_F64 = 0, 1, 2, 3
_TORCH_DT = {DT_I64: torch.int64, DT_I32: torch.int32, DT_F32: torch.float32, DT_F64: torch.float64}
_NP_TO_DT = {np.dtype(np.int64): DT_I64, np.dtype(np.int32): DT_I32, np.dtype(np.float32): DT_F32,
             np.dtype(np.float64): DT_F64}
E_ECAP = 5005


class PrlJsonMember(ctypes.Structure):
    _fields_ = [("key_off", c_int64), ("key_len", c_int64), ("val_off", c_int64), ("val_len", c_int64)]


class PrlJsonArray(ctypes.Structure):
    _fields_ = [("text", c_void_p), ("len", c_int64), ("dtype", c_int32), ("ndim", c_int32),
                ("shape", c_int64 * MAX_DIMS), ("has_float", c_int32), ("status", c_int32), ("out", c_void_p)]


_SIGNATURES = {
    "prl_data_abi_version": (c_int, []),
    "prl_data_error_string": (c_char_p, [c_int]),
    "prl_json_members": (c_int, [c_void_p, c_int64, POINTER(PrlJsonMember), c_int32, POINTER(c_int32)]),
    "prl_json_array_shape": (c_int, [POINTER(PrlJsonArray)]),
    "prl_json_array_fill": (c_int, [POINTER(PrlJsonArray), c_int32, c_int32]),
    "prl_json_format_bound": (c_int64, [c_int64, c_int32, POINTER(c_int64)]),
    "prl_json_array_format": (c_int, [c_void_p, c_int32, c_int32, POINTER(c_int64), c_void_p, c_int64,
                                      POINTER(c_int64)]),
    "prl_rl_group_stats": (c_int, [c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "prl_collate_packed": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
}

_lib = None
_pylib = None


class PrlDataError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists() or os.environ.get("PRL_REBUILD"):
        try:
            from . import _build
            _build.build_data()
        except Exception as e:
            raise PrlDataError(f"libprl_data.so is missing and could not be built: {e}") from e
    try:
        lib = ctypes.CDLL(str(LIB_PATH))  # CDLL: every call releases the GIL
    except OSError as e:
        raise PrlDataError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.prl_data_abi_version() != ABI:
        raise PrlDataError(f"libprl_data.so has ABI {lib.prl_data_abi_version()}, binding expects {ABI}: rebuild it")
    _lib = lib
    return lib


def pylib():
    """The same library through ctypes.PyDLL (GIL held) for the Python-object helpers
    (csrc/pyconv.cpp), or None when it was built without them."""
    global _pylib
    if _pylib is None:
        load()
        lib = ctypes.PyDLL(str(LIB_PATH))
        if hasattr(lib, "prl_py_concat"):
            lib.prl_py_concat.restype = c_int
            lib.prl_py_concat.argtypes = [ctypes.py_object, c_int, c_void_p, c_int64]
            _pylib = lib
        else:
            _pylib = False
    return _pylib or None


def concat_lists(seqs: list, dtype: int, total: int) -> np.ndarray | None:
    """The lists in `seqs` concatenated into one int64 / float64 array (numpy's values), or None
    when an element is not a plain Python int / float (the caller converts in Python)."""
    lib = pylib()
    if lib is None:
        return None
    out = np.empty(total, np.int64 if dtype == DT_I64 else np.float64)
    rc = lib.prl_py_concat(seqs, dtype, out.ctypes.data, total)
    return out if rc == 0 else None


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise PrlDataError(f"{what} failed: {load().prl_data_error_string(rc).decode()} (code {rc})")


def _ptr(t) -> int:
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return t.ctypes.data


# ---------------------------------------------------------------------------------------------
# stream documents

def batch_field_dtypes() -> dict[str, int]:
    """PipelineBatchEncoding's numeric fields and the dtype its validators give them."""
    from .finetune.types import FLOAT_FIELDS, LONG_FIELDS
    d = {k: DT_I64 for k in LONG_FIELDS}
    d.update({k: DT_F32 for k in FLOAT_FIELDS})
    d["seq_boundaries"] = DT_I32
    return d


def members(doc: bytes) -> list[tuple[str, int, int]]:
    """(key, value offset, value length) of a JSON object's members."""
    lib = load()
    base = ctypes.cast(ctypes.c_char_p(doc), c_void_p).value
    cap = 32
    while True:
        out = (PrlJsonMember * cap)()
        n = c_int32(0)
        rc = lib.prl_json_members(base, len(doc), out, cap, ctypes.byref(n))
        if rc == E_ECAP:
            cap = n.value
            continue
        _check(rc, "prl_json_members")
        return [(doc[m.key_off:m.key_off + m.key_len].decode(), m.val_off, m.val_len) for m in out[:n.value]]


def decode_document(doc: bytes, numeric: dict[str, int], pin: bool = False, threads: int = 4) -> dict[str, Any]:
    """Decode one JSON object: the members named in `numeric` (whose value is a list) into torch
    tensors of that dtype (pinned if `pin`), everything else with json.  Member order kept."""
    lib = load()
    if isinstance(doc, str):
        doc = doc.encode()
    base = ctypes.cast(ctypes.c_char_p(doc), c_void_p).value
    out: dict[str, Any] = {}
    jobs: list[tuple[str, PrlJsonArray, torch.Tensor, int, int]] = []
    for key, off, ln in members(doc):
        dt = numeric.get(key)
        if dt is not None and doc[off:off + 1] == b"[":
            a = PrlJsonArray(text=base + off, len=ln, dtype=dt)
            if lib.prl_json_array_shape(ctypes.byref(a)) == 0:
                t = torch.empty(tuple(a.shape[:a.ndim]), dtype=_TORCH_DT[dt], pin_memory=pin)
                a.out = t.data_ptr()
                jobs.append((key, a, t, off, ln))
                out[key] = t
                continue
        out[key] = json.loads(doc[off:off + ln])
    if jobs:
        arr = (PrlJsonArray * len(jobs))(*[j[1] for j in jobs])
        lib.prl_json_array_fill(arr, len(jobs), max(1, min(threads, len(jobs))))
        for (key, _, _, off, ln), a in zip(jobs, arr):
            if a.status != 0:  # e.g. a float64 -> int overflow: let the Python path decide
                out[key] = json.loads(doc[off:off + ln])
    return out


def decode_batch(doc: bytes, pin: bool = False, threads: int = 4):
    """A training_data line -> PipelineBatchEncoding (the loader's decode, types.py:48-117)."""
    from .finetune.types import PipelineBatchEncoding
    return PipelineBatchEncoding(**decode_document(doc, batch_field_dtypes(), pin=pin, threads=threads))


def format_array(a) -> str:
    """A dense numeric array as nested JSON lists (json.dumps(a.tolist()) with , separators)."""
    lib = load()
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().contiguous().numpy()
    a = np.ascontiguousarray(a)
    dt = _NP_TO_DT.get(a.dtype)
    if dt is None or a.ndim < 1 or a.ndim > MAX_DIMS:
        raise PrlDataError(f"format_array: unsupported array {a.dtype} with {a.ndim} dims")
    shape = (c_int64 * a.ndim)(*a.shape)
    cap = lib.prl_json_format_bound(a.size, a.ndim, shape)
    buf = ctypes.create_string_buffer(cap)
    n = c_int64(0)
    _check(lib.prl_json_array_format(a.ctypes.data if a.size else None, dt, a.ndim, shape, buf, cap,
                                     ctypes.byref(n)), "prl_json_array_format")
    return buf.raw[:n.value].decode()


def _native_array(v):
    if isinstance(v, torch.Tensor) and v.dtype in (torch.int64, torch.int32, torch.float32, torch.float64) \
            and v.dim() >= 1:
        return v
    if isinstance(v, np.ndarray) and v.dtype in _NP_TO_DT and v.ndim >= 1:
        return v
    return None


def encode_document(data: dict[str, Any]) -> str:
    """streams.dumps(data) with the numeric tensors / arrays formatted natively."""
    from .streams import _jsonable
    parts = []
    for k, v in data.items():
        arr = _native_array(v)
        text = format_array(arr) if arr is not None else json.dumps(_jsonable(v), separators=(",", ":"))
        parts.append(json.dumps(k) + ":" + text)
    return "{" + ",".join(parts) + "}"


# ---------------------------------------------------------------------------------------------
# preprocessing arithmetic

def rl_group_stats(group_of: np.ndarray, n_groups: int, reward0: np.ndarray, length: np.ndarray):
    """Per-group (mean reward, sample std, mean length), rl/__init__.py:408-416."""
    lib = load()
    g = np.ascontiguousarray(group_of, dtype=np.int64)
    r = np.ascontiguousarray(reward0, dtype=np.float64)
    ln = np.ascontiguousarray(length, dtype=np.int64)
    mean, std, tok = (np.empty(n_groups, np.float64) for _ in range(3))
    _check(lib.prl_rl_group_stats(len(g), _ptr(g), n_groups, _ptr(r), _ptr(ln), _ptr(mean), _ptr(std), _ptr(tok)),
           "prl_rl_group_stats")
    return mean, std, tok


def collate_arrays(lengths: np.ndarray, ids: np.ndarray, labels: np.ndarray, label_pad: int = -100):
    """collate_packed's token layout: (ids, labels, position_ids, seq_boundaries)."""
    lib = load()
    lengths = np.ascontiguousarray(lengths, dtype=np.int64)
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    labels = np.ascontiguousarray(labels, dtype=np.int64)
    total = int(lengths.sum())
    if ids.size != total or labels.size != total:
        raise PrlDataError(f"collate_arrays: {ids.size} ids / {labels.size} labels for {total} tokens")
    o_ids, o_lab, o_pos = (np.empty(total, np.int64) for _ in range(3))
    bounds = np.empty(len(lengths) + 1, np.int32)
    _check(lib.prl_collate_packed(len(lengths), _ptr(lengths), _ptr(ids), _ptr(labels), label_pad, _ptr(o_ids),
                                  _ptr(o_lab), _ptr(o_pos), _ptr(bounds)), "prl_collate_packed")
    return o_ids, o_lab, o_pos, bounds


def nan_to_num(x: float) -> float:
    return 0.0 if math.isnan(x) else x
