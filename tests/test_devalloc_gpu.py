"""The allocator settings take effect on the device (devalloc.py): with the default, a 1.1 GiB
request is served by a 1.25 GiB block (4 divisions per power of two above 512 MB) and a 300 MB one
by 288 MiB (16 divisions below); 512 B granularity without.
Run in a child process: the settings are process-global."""

import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from pipelinerl_amd.devalloc import configure_device_allocator
if sys.argv[2] == "on":
    assert configure_device_allocator() is not None
torch.cuda.init()
out = []
for n in (int(1.1 * 2**30), 300 * 10**6):
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    out.append(torch.cuda.memory_allocated())
    del x
print(*out)
"""


def _blocks(mode: str) -> list[int]:
    env = {k: v for k, v in os.environ.items() if k not in ("PYTORCH_HIP_ALLOC_CONF", "PYTORCH_CUDA_ALLOC_CONF")}
    out = subprocess.run([sys.executable, "-c", CHILD, str(ROOT / "pipelinerl-swe_amd"), mode], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return [int(v) for v in out.stdout.strip().splitlines()[-1].split()]


@pytest.mark.gpu
def test_request_sizes_round_per_interval():
    sizes = (int(1.1 * 2**30), 300 * 10**6)
    assert _blocks("off") == [-(-n // 512) * 512 for n in sizes]
    assert _blocks("on") == [int(1.25 * 2**30), 288 << 20]
