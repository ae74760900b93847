"""The C-ABI library loads without a GPU and exports every symbol include/prl_hip.h declares;
the Python binding's statistic table matches the header's enum."""

import ctypes

import pytest
import re

from conftest import ROOT


def test_library_exports_header_symbols():
    from pipelinerl_amd import _native

    lib = _native.load()
    declared = _native.header_symbols()
    assert len(declared) >= 9
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.prl_abi_version() == _native.ABI_VERSION == 3
    assert lib.prl_grpo_nstat() == _native.NSTAT
    assert lib.prl_error_string(1001).decode() == "invalid argument"
    nbytes = ctypes.c_size_t(0)
    assert lib.prl_grpo_workspace_bytes(0, ctypes.byref(nbytes)) == 0 and nbytes.value > 0


def test_stat_enum_matches_header():
    from pipelinerl_amd import _native

    text = (ROOT / "include" / "prl_hip.h").read_text()
    body = text[text.index("enum PrlStat {"):text.index("PRL_NSTAT\n")]
    names = re.findall(r"PRL_S_(\w+)", body)
    assert names == _native.STATS


def test_struct_layouts():
    from pipelinerl_amd import _native

    assert ctypes.sizeof(_native.PrlGrpoBatch) == 8 + 4 + 4 + 4 * 8 + 10 * 8
    assert ctypes.sizeof(_native.PrlGrpoParams) == 6 * 4 + 8 * 4 + 2 * 4  # + pair_spin_ticks, f32_rows (ABI 3)
    assert ctypes.sizeof(_native.PrlGrpoOutputs) == 11 * 8


def test_invalid_arguments_rejected_without_gpu():
    from pipelinerl_amd import _native

    lib = _native.load()
    b = _native.PrlGrpoBatch()
    p = _native.PrlGrpoParams()
    o = _native.PrlGrpoOutputs()
    # null pointers / zero shapes are rejected before any device call
    assert lib.prl_grpo_forward(ctypes.byref(b), ctypes.byref(p), ctypes.byref(o), None, 0, None) == 1001
    assert lib.prl_flatten_bf16(None, None, None, None, -1, None, None) == 1001
    assert lib.prl_grpo_pair_fallbacks(None, 0, None, None) == 1001
    n = ctypes.c_uint64(7)
    assert lib.prl_grpo_pair_fallbacks(None, 0, None, ctypes.byref(n)) == 1003 and n.value == 0  # no workspace
    assert lib.prl_paced_read(None, 1 << 20, 153.0, 16, None, None) == 1001
    assert lib.prl_paced_read(16, 1 << 20, 0.0, 16, 16, None) == 1001  # a rate must be given
    assert lib.prl_paced_read(16, 1 << 20, 153.0, 0, 16, None) == 1001
    assert lib.prl_paced_read(8, 1 << 20, 153.0, 16, 16, None) == 1001  # 16-B aligned source


def test_comm_library_exports_header_symbols():
    """libprl_comm.so (RCCL C ABI, include/prl_comm.h) loads without a GPU and exports every
    declared function."""
    from pipelinerl_amd import comm

    lib = comm.load()
    text = comm.HEADER_PATH.read_text()
    declared = sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(prl_comm_\w+)\s*\(", text, flags=re.M)))
    assert len(declared) >= 10
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.prl_comm_abi_version() == 1
    assert lib.prl_comm_error_string(3001).decode() == "invalid argument"
    h = ctypes.c_void_p()
    assert lib.prl_comm_init(None, 0, 1, 0, ctypes.byref(h)) == 3001  # argument checks before any HIP call


def test_gemm_library_exports_header_symbols():
    """libprl_gemm.so (hipBLASLt C ABI, include/prl_gemm.h) loads without a GPU, exports every
    declared function, and rejects bad arguments before opening hipBLASLt or touching a device."""
    from pipelinerl_amd import gemm

    lib = gemm.load()
    text = gemm.HEADER_PATH.read_text()
    declared = sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(prl_gemm_\w+)\s*\(", text, flags=re.M)))
    assert len(declared) >= 5
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.prl_gemm_abi_version() == gemm.ABI_VERSION == 4
    assert lib.prl_gemm_error_string(4001).decode() == "invalid argument"
    # m = 0, a bad op, null pointers, lda < m: all PRL_GEMM_E_INVALID
    assert lib.prl_gemm_bf16(0, 0, 0, 4, 4, 1, 4, 1, 4, None, 0.0, 1, 4, 1, -1, None) == 4001
    assert lib.prl_gemm_bf16(2, 0, 4, 4, 4, 1, 4, 1, 4, None, 0.0, 1, 4, 1, -1, None) == 4001
    assert lib.prl_gemm_bf16(0, 0, 4, 4, 4, None, 4, 1, 4, None, 0.0, 1, 4, 1, -1, None) == 4001
    assert lib.prl_gemm_bf16(0, 0, 8, 4, 4, 1, 4, 1, 4, None, 0.0, 1, 8, 1, -1, None) == 4001
    assert lib.prl_gemm_bf16(0, 0, 4, 4, 4, 1, 4, 1, 4, None, 0.5, 1, 4, 1, -1, None) == 4001  # beta in {0, 1}
    assert lib.prl_gemm_bf16(0, 0, 4, 4, 4, 1, 4, 1, 4, 1, 0.0, 1, 4, 0, -1, None) == 4001  # bias needs bf16 D
    assert lib.prl_gemm_heuristic_index(0, 0, 0, 1, 1, 1, 1, 1, 1, 0.0) == -1


def test_gemm_refuses_unswept_solution_indices():
    """prl_gemm runs an explicit hipBLASLt solution index only if it is in the registered
    (swept-clean) set: the binding registers gemm_solutions.json's indices at load, and any other
    index is refused with PRL_GEMM_E_REFUSED before a device is touched (a catalog
    solution outside the swept set faulted the GPU in a sweep).  The pointers below are never
    dereferenced: the refusal comes first."""
    import json

    from pipelinerl_amd import gemm

    lib = gemm.load()
    shipped = sorted({int(e["index"]) for es in json.loads(gemm.SOLUTIONS_PATH.read_text()).values() for e in es
                      if int(e["index"]) >= 0})
    assert shipped
    unswept = max(shipped) + 1
    args = (0, 0, 4, 4, 4, 16, 4, 16, 4, None, 0.0, 16, 4, 1)
    assert lib.prl_gemm_bf16(*args, unswept, None) == gemm.PRL_GEMM_E_REFUSED == 4003
    assert b"allowed" in lib.prl_gemm_error_string(4003)
    with pytest.raises(gemm.GemmError, match="allowed"):
        gemm._check(lib.prl_gemm_bf16(*args, unswept, None), "prl_gemm_bf16")
    # re-registering a smaller set refuses what was allowed before; an empty set allows none
    try:
        gemm.allow(shipped[1:])
        assert lib.prl_gemm_bf16(*args, shipped[0], None) == 4003
        gemm.allow([])
        assert all(lib.prl_gemm_bf16(*args, i, None) == 4003 for i in shipped[:3])
        assert lib.prl_gemm_allow_solutions(None, 2) == 4001
    finally:
        gemm.allow(shipped)


def test_gemm_solution_window(monkeypatch):
    """A swept solution is used only within 2x of the token count it was tuned at."""
    from pipelinerl_amd import gemm

    monkeypatch.setattr(gemm, "_solutions", {"wgrad:8:16:bf16:0": [{"T": 1000, "index": 7}, {"T": 8000, "index": 9}]})
    assert gemm.solution_for("wgrad", 1000, 8, 16) == 7
    assert gemm.solution_for("wgrad", 1900, 8, 16) == 7
    assert gemm.solution_for("wgrad", 3000, 8, 16) is None  # 3x from 1000, 2.7x from 8000
    assert gemm.solution_for("wgrad", 16000, 8, 16) == 9
    assert gemm.solution_for("wgrad", 17000, 8, 16) is None
    assert gemm.solution_for("fwd", 1000, 8, 16) is None and gemm.solution_for("wgrad", 0, 8, 16) is None
    assert gemm.solution_for("wgrad", 1000, 8, 16, gemm.F32, True) is None
