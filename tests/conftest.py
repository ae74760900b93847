import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "pipelinerl-swe_amd"
GOLDEN = ROOT / "tests" / "golden"
for p in (str(ROOT), str(PKG_DIR)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run on the GPU box")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_f1():
    """F1 golden fixtures: (batches, outputs, cases)."""
    inp = np.load(GOLDEN / "f1_inputs.npz")
    batches = {}
    for key in inp.files:
        name, field = key.split("__", 1)
        batches.setdefault(name, {})[field] = inp[key]
    for b in batches.values():
        b["is_packed"] = bool(b["is_packed"])
    out = np.load(GOLDEN / "f1_outputs.npz")
    cases = json.loads((GOLDEN / "f1_cases.json").read_text())
    return batches, out, cases


@pytest.fixture(scope="session")
def f1():
    return load_f1()


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # GPU tests on a machine without a GPU are a hard error only if explicitly requested.
    if gpu_available() or os.environ.get("PRL_REQUIRE_GPU"):
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
