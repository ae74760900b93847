"""The allocator settings take effect on the device (devalloc.py): with the default, a 1.1 GiB
request is served by a 1.25 GiB block (4 divisions per power of two above 512 MB) and a 300 MB one
by 288 MiB (16 divisions below); 512 B granularity without; and devalloc.round_size (the
checkpointing plan's restatement of the rule) agrees with the device for every size tried.
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
for n in map(int, sys.argv[3].split(",")):
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    out.append(torch.cuda.memory_allocated())
    del x
print(*out)
"""


# 1.1 GiB, 300 MB, and the C3 / 1.5B micro-batch tensors the checkpointing plan rounds: [T, H],
# [T, I], [T, 2 I] at 12 000 tokens of 7B, [T, I] and the logits chunk at 65 536 tokens of 1.5B
SIZES = (int(1.1 * 2**30), 300 * 10**6, 12000 * 3584 * 2, 12000 * 18944 * 2, 12000 * 37888 * 2,
         65536 * 8960 * 2, 65536 * 151936 * 2, 4 * 10**6, 1000)


def _blocks(mode: str) -> list[int]:
    env = {k: v for k, v in os.environ.items() if k not in ("PYTORCH_HIP_ALLOC_CONF", "PYTORCH_CUDA_ALLOC_CONF")}
    out = subprocess.run([sys.executable, "-c", CHILD, str(ROOT / "pipelinerl-swe_amd"), mode,
                          ",".join(str(n) for n in SIZES)], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return [int(v) for v in out.stdout.strip().splitlines()[-1].split()]


@pytest.mark.gpu
def test_request_sizes_round_per_interval():
    from pipelinerl_amd import devalloc

    assert _blocks("off") == [-(-n // 512) * 512 for n in SIZES]
    on = _blocks("on")
    assert on[:2] == [int(1.25 * 2**30), 288 << 20]
    # the plan's restatement of the rule (devalloc.round_size) is what the device allocator does
    assert on == [devalloc.round_size(n, devalloc.DEFAULT_SETTINGS) for n in SIZES]
