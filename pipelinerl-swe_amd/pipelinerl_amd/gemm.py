"""ctypes binding of libprl_gemm.so (C ABI in include/prl_gemm.h): the trainer's linear-layer GEMMs
through hipBLASLt with a per-problem solution choice.

Row-major torch terms (X [T, K] activations, W [N, K] weight, dY [T, N] upstream gradient):
  linear_fwd    Y  = X W^T       -> column-major D[N, T] = op_T(W) op_N(X)
  linear_dgrad  dX = dY W        -> column-major D[K, T] = op_N(W) op_N(dY)
  linear_wgrad  dW = dY^T X      -> column-major D[K, N] = op_N(X) op_T(dY)
The hipBLASLt is the ROCm installation's (include/prl_gemm.h), not torch's bundled copy.
Solutions come from ``gemm_solutions.json`` (found by ``tools/hipblaslt_probe.cpp`` on MI355X for
the trainer's shapes; nearest tuned token count), else the library heuristic.  No fallback: if the
library cannot be loaded, the entry points raise.
"""

from __future__ import annotations

import ctypes
import json
import math
import os
from pathlib import Path

import torch  # loaded first: libprl_gemm.so then binds torch's own hipBLASLt (same soname)

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["PRL_GEMM_LIB"]) if os.environ.get("PRL_GEMM_LIB") else _PKG / "libprl_gemm.so"
HEADER_PATH = _PKG.parents[1] / "include" / "prl_gemm.h"
SOLUTIONS_PATH = _PKG / "gemm_solutions.json"
ABI_VERSION = 4
N_, T_ = 0, 1
F32, BF16 = 0, 1
PRL_GEMM_E_REFUSED = 4003

_lib = None
_solutions: dict | None = None


class GemmError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        try:
            from ._build import build_gemm

            build_gemm()
        except Exception as e:  # noqa: BLE001
            raise GemmError(f"libprl_gemm.so is missing and could not be built: {e}") from e
    lib = ctypes.CDLL(str(LIB_PATH))
    c = ctypes
    sig = {
        "prl_gemm_abi_version": (c.c_int, []),
        "prl_gemm_error_string": (c.c_char_p, [c.c_int]),
        "prl_gemm_bf16": (c.c_int, [c.c_int, c.c_int, c.c_int64, c.c_int64, c.c_int64, c.c_void_p, c.c_int64,
                                    c.c_void_p, c.c_int64, c.c_void_p, c.c_float, c.c_void_p, c.c_int64, c.c_int,
                                    c.c_int, c.c_void_p]),
        "prl_gemm_heuristic_index": (c.c_int, [c.c_int, c.c_int, c.c_int64, c.c_int64, c.c_int64, c.c_int64,
                                               c.c_int64, c.c_int64, c.c_int, c.c_float]),
        "prl_gemm_library": (c.c_int, [c.c_char_p, c.c_int]),
        "prl_gemm_allow_solutions": (c.c_int, [c.POINTER(c.c_int32), c.c_int]),
        "prl_gemm_handle_count": (c.c_int, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    if lib.prl_gemm_abi_version() != ABI_VERSION:
        raise GemmError("libprl_gemm.so ABI mismatch")
    _lib = lib
    allow(sorted({int(e["index"]) for es in solutions().values() for e in es if int(e["index"]) >= 0}))
    return lib


def allow(indices: list[int]) -> None:
    """Register the solution indices prl_gemm may run (the shipped table's, swept clean on
    MI355X); any other explicit index is refused by the library (PRL_GEMM_E_REFUSED)."""
    arr = (ctypes.c_int32 * max(1, len(indices)))(*indices)
    _check(load().prl_gemm_allow_solutions(arr, len(indices)), "prl_gemm_allow_solutions")


def _check(rc: int, what: str):
    if rc != 0:
        raise GemmError(f"{what} failed: {load().prl_gemm_error_string(rc).decode()} (code {rc})")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def solutions() -> dict:
    global _solutions
    if _solutions is None:  # PRL_GEMM_SOLUTIONS=off: library heuristic only; =<file>: another table (A/B)
        env = os.environ.get("PRL_GEMM_SOLUTIONS", "")
        path = Path(env) if env not in ("", "off") else SOLUTIONS_PATH
        _solutions = json.loads(path.read_text()) if env != "off" and path.exists() else {}
    return _solutions


def solution_for(pas: str, T: int, N: int, K: int, d_dtype: int = BF16, accumulate: bool = False) -> int | None:
    """Routing entry for the nearest tuned token count (log scale) within 2x of T: a solution
    index (>= 0), -1 = the library heuristic (entries measured faster than torch's matmul with
    it, forward only), or None when no entry covers T (forward: torch's F.linear; backward: the
    heuristic).  A solution tuned for 65 536 rows is not trusted at 4 096."""
    entries = solutions().get(f"{pas}:{N}:{K}:{'f32' if d_dtype == F32 else 'bf16'}:{int(accumulate)}")
    if not entries or T <= 0:
        return None
    best = min(entries, key=lambda e: abs(math.log(T) - math.log(e["T"])))
    return int(best["index"]) if abs(math.log(T) - math.log(best["T"])) <= math.log(2.0) + 1e-9 else None


def gemm(op_a: int, op_b: int, m: int, n: int, k: int, a: torch.Tensor, lda: int, b: torch.Tensor, ldb: int,
         d: torch.Tensor, ldd: int, beta: float = 0.0, solution: int = -1,
         bias: torch.Tensor | None = None) -> torch.Tensor:
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or d.dtype not in (torch.bfloat16, torch.float32):
        raise GemmError("prl_gemm: bf16 operands, bf16 / fp32 output")
    if bias is not None and (bias.dtype != torch.bfloat16 or bias.numel() != m or not bias.is_contiguous()):
        raise GemmError("prl_gemm: bias must be a contiguous bf16 vector of m elements")
    dd = F32 if d.dtype == torch.float32 else BF16
    _check(load().prl_gemm_bf16(op_a, op_b, m, n, k, a.data_ptr(), lda, b.data_ptr(), ldb,
                                bias.data_ptr() if bias is not None else None, beta, d.data_ptr(), ldd, dd, solution,
                                _stream(d)), "prl_gemm_bf16")
    return d


def _rows(t: torch.Tensor) -> torch.Tensor:
    t2 = t.reshape(-1, t.shape[-1])
    return t2 if t2.is_contiguous() else t2.contiguous()


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
               solution: int | None = None) -> torch.Tensor:
    """Y = X W^T (+ bias), X [..., K] bf16, W [N, K] bf16 contiguous, bias [N] bf16."""
    x2 = _rows(x)
    T, K = x2.shape
    N = w.shape[0]
    y = torch.empty((T, N), dtype=x.dtype, device=x.device)
    sol = solution_for("fwd", T, N, K) if solution is None else solution
    gemm(T_, N_, N, T, K, w, K, x2, K, y, N, solution=-1 if sol is None else sol, bias=bias)
    return y.view(*x.shape[:-1], N)


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
                 accumulate: bool = False) -> torch.Tensor:
    """dX = dY W, dY [..., N], W [N, K]; with ``out`` (bf16, [..., K] contiguous) and
    accumulate=True the GEMM adds into it (beta = 1): the input gradient of layers sharing one
    input (q/k/v, gate/up) summed in the epilogue instead of by separate add kernels."""
    d2 = _rows(dy)
    T, N = d2.shape
    K = w.shape[1]
    if out is None:
        if accumulate:
            raise GemmError("linear_dgrad: accumulate needs out")
        out = torch.empty((T, K), dtype=dy.dtype, device=dy.device)
    if out.numel() != T * K or out.dtype != dy.dtype or not out.is_contiguous():
        raise GemmError("linear_dgrad: out must be a contiguous bf16 tensor of T x K elements")
    sol = solution_for("dgrad", T, N, K, BF16, accumulate)
    if sol is None and accumulate:  # a swept beta = 0 solution; prl_gemm checks it supports beta = 1
        sol = solution_for("dgrad", T, N, K)
    gemm(N_, N_, K, T, N, w, K, d2, N, out, K, beta=1.0 if accumulate else 0.0, solution=-1 if sol is None else sol)
    return out.view(*dy.shape[:-1], K)


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
                 accumulate: bool = False) -> torch.Tensor:
    """dW = dY^T X ([N, K]); with ``out`` ([N, K] contiguous, fp32 or bf16) and accumulate=True the
    GEMM adds into it (beta = 1): the chunked lm_head's fp32 sum, a weight's gradient accumulated
    over micro-batches (finetune/model_ops.py _wgrad)."""
    d2, x2 = _rows(dy), _rows(x)
    T, N = d2.shape
    K = x2.shape[1]
    if out is None:
        out = torch.empty((N, K), dtype=dy.dtype, device=dy.device)
    if out.shape != (N, K) or not out.is_contiguous():
        raise GemmError("linear_wgrad: out must be a contiguous [N, K] tensor")
    dd = F32 if out.dtype == torch.float32 else BF16
    sol = solution_for("wgrad", T, N, K, dd, accumulate)
    if sol is None and accumulate:  # a swept beta = 0 solution; prl_gemm checks it supports beta = 1
        sol = solution_for("wgrad", T, N, K, dd)
    gemm(N_, T_, K, N, T, x2, K, d2, N, out, K, beta=1.0 if accumulate else 0.0, solution=-1 if sol is None else sol)
    return out


def library() -> str:
    """Path and version of the hipBLASLt prl_gemm runs on (needs a device)."""
    buf = ctypes.create_string_buffer(512)
    rc = load().prl_gemm_library(buf, 512)
    _check(rc, "prl_gemm_library")
    return buf.value.decode()
