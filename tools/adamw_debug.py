"""Where PrlAdamW and torch's fused AdamW differ (debug tool): steps on random tensors, then per
state the mismatch count and, for the first mismatches, which evaluation of
m' = beta1 m + (1 - beta1) g (and v' likewise) each side matches, computed exactly on the host:
  A fma(beta1, m, (1-beta1) g)   B fma(1-beta1, g, beta1 m)   C no fma."""
import sys
from fractions import Fraction as F
from pathlib import Path

import numpy as np
import torch

sys.path[:0] = [str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd")]
from pipelinerl_amd.finetune.optim import PrlAdamW  # noqa: E402


def rd(x):  # exact rational -> nearest double
    return F(float(x))


def forms(b, m, g, sq=False):
    b, m, g = F(b), F(m), F(g)
    ob = rd(1 - b)
    t2 = rd(ob * g) * g if sq else ob * g  # v: ((1-b) g) g, the inner product rounded
    t2r = rd(t2)
    bm = rd(b * m)
    return {"A": float(np.float32(float(rd(b * m + t2r)))), "B": float(np.float32(float(rd(t2 + bm)))),
            "C": float(np.float32(float(rd(bm + t2r))))}


dtype = getattr(torch, sys.argv[1]) if len(sys.argv) > 1 else torch.float32
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = torch.Generator(device="cuda").manual_seed(0)
p0 = (torch.randn(4096, generator=g, device="cuda") * 0.1).to(dtype)
pa, pb = torch.nn.Parameter(p0.clone()), torch.nn.Parameter(p0.clone())
ref = torch.optim.AdamW([pa], lr=3e-4, weight_decay=0.01, fused=True)
opt = PrlAdamW([pb], lr=3e-4, weight_decay=0.01)
for s in range(steps):
    gr = torch.randn(4096, generator=g, device="cuda").to(dtype)
    prev = {k: ref.state[pa][k].clone() for k in ("exp_avg", "exp_avg_sq")} if pa in ref.state else None
    pa.grad, pb.grad = gr.clone(), gr.clone()
    ref.step()
    opt.step()
    if prev is None:
        continue
    for k, b in (("exp_avg", 0.9), ("exp_avg_sq", 0.999)):
        a, c = ref.state[pa][k], opt.state[pb][k]
        d = (a != c).nonzero().flatten()
        print("step", s, k, "mismatches", d.numel(), flush=True)
        for i in d[:6].tolist():
            f = forms(b, float(prev[k][i]), float(gr[i]), sq=k == "exp_avg_sq")
            ta, tb = float(a[i]), float(c[i])
            print(f"   torch={[n for n, v in f.items() if v == ta]} prl={[n for n, v in f.items() if v == tb]}")
    with torch.no_grad():  # continue from torch's state on both sides
        pb.copy_(pa)
        for k in ("exp_avg", "exp_avg_sq"):
            opt.state[pb][k].copy_(ref.state[pa][k])
