"""Time the HIP flash-attention backward kernels alone (tools; rocprofv3 gives the split):
Qwen2.5-1.5B attention shapes, 12 q heads / 2 kv heads (GQA native), D 128, T = 16384 as 8 x 2048."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd.finetune.attention import PackedCausalAttention  # noqa: E402

T, seq, H, HKV, D = int(sys.argv[1]) if len(sys.argv) > 1 else 16384, int(sys.argv[2]) if len(sys.argv) > 2 else 2048, 12, 2, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((T, h, D), generator=g, device="cuda").to(torch.bfloat16).requires_grad_() for h in (H, HKV, HKV))
do = torch.randn((T, H, D), generator=g, device="cuda").to(torch.bfloat16)
bounds = list(range(0, T + 1, seq))
cu = torch.tensor(bounds, dtype=torch.int32, device="cuda")
for _ in range(2):
    PackedCausalAttention.apply(q, k, v, cu, seq, bounds).backward(do)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    PackedCausalAttention.apply(q, k, v, cu, seq, bounds).backward(do)
torch.cuda.synchronize()
print(f"fwd+bwd {1e3 * (time.perf_counter() - t0) / 10:.3f} ms")
