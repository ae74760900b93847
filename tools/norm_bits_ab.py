"""Bit-identity of two libprl_hip builds' RMSNorm backward (measurement tool): loads the product
library and the one named by argv[1] side by side (ctypes, RTLD_LOCAL) and compares dx / dw of
prl_rmsnorm_backward and prl_add_rmsnorm_backward bit for bit at the trainer's shapes.

    python tools/norm_bits_ab.py pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_norm_regacc.so
"""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402

from pipelinerl_amd import _native  # noqa: E402


def run(lib, rows, H, add, seed=0, time_iters=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.randn((rows, H), generator=g, device="cuda") * 2).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, generator=g, device="cuda")).to(torch.bfloat16)
    dy = torch.randn((rows, H), generator=g, device="cuda").to(torch.bfloat16)
    dh = torch.randn((rows, H), generator=g, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    rstd = torch.empty(rows, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    c = ctypes
    lib.prl_rmsnorm_forward.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int64, c.c_int64, c.c_float,
                                        c.c_void_p]
    assert lib.prl_rmsnorm_forward(x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), rows, H, 1e-6, st) == 0
    nb = c.c_size_t(0)
    lib.prl_rmsnorm_workspace_bytes.argtypes = [c.c_int64, c.POINTER(c.c_size_t)]
    assert lib.prl_rmsnorm_workspace_bytes(H, c.byref(nb)) == 0
    ws = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    if add:
        f = lib.prl_add_rmsnorm_backward
        f.argtypes = [c.c_void_p] * 7 + [c.c_size_t, c.c_int64, c.c_int64, c.c_void_p]
        rc = f(dy.data_ptr(), dh.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(),
               ws.data_ptr(), nb.value, rows, H, st)
    else:
        f = lib.prl_rmsnorm_backward
        f.argtypes = [c.c_void_p] * 7 + [c.c_size_t, c.c_int64, c.c_int64, c.c_void_p]
        rc = f(dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(), ws.data_ptr(),
               nb.value, rows, H, st)
    assert rc == 0, rc
    torch.cuda.synchronize()
    if time_iters:  # the C-ABI call alone (backward kernel + the two dw folds), HIP events
        args = ((dy.data_ptr(), dh.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(),
                 ws.data_ptr(), nb.value, rows, H, st) if add else
                (dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(), ws.data_ptr(),
                 nb.value, rows, H, st))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(time_iters):
            f(*args)
        e1.record()
        e1.synchronize()
        return dx, dw, e0.elapsed_time(e1) / time_iters
    return dx, dw


def main():
    a = _native.load()
    b = ctypes.CDLL(sys.argv[1])
    out = []
    for rows, H in ((8704, 3584), (4093, 3584), (2048, 2560), (1000, 4096)):
        for add in (False, True):
            dxa, dwa = run(a, rows, H, add)
            dxb, dwb = run(b, rows, H, add)
            out.append({"rows": rows, "H": H, "add": add, "dx_equal": bool(torch.equal(dxa.view(torch.int16), dxb.view(torch.int16))),
                        "dw_equal": bool(torch.equal(dwa.view(torch.int16), dwb.view(torch.int16)))})
    # timing, alternated: the C ABI call at the 7B add-norm shape (C3 micro-batch rows)
    tim = {"product": [], "other": []}
    for _ in range(4):
        for name, lib in (("product", a), ("other", b)):
            tim[name].append(round(run(lib, 8704, 3584, True, time_iters=200)[2] * 1e3, 2))
    nbytes = 4 * 8704 * 3584 * 2
    out.append({"add_rmsnorm_backward_8704x3584_us": tim, "algorithmic_bytes": nbytes,
                "TBps": {k: round(nbytes / (min(v) * 1e-6) / 1e12, 3) for k, v in tim.items()}})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
