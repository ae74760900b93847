"""Bit-identity and timing of two libprl_hip builds' RMSNorm backward (measurement tool).  Each
build runs in its own process (PRL_LIB selects it: two builds' kernels cannot share one process);
dx / dw of prl_rmsnorm_backward and prl_add_rmsnorm_backward are compared bit for bit, and the
C-ABI call (backward kernel + the two dw folds) is timed with HIP events, alternated.

    python tools/norm_bits_ab.py pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_norm_regacc.so
"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SHAPES = ((8704, 3584), (4093, 3584), (2048, 2560), (1000, 4096))


def child(out_path: str, time_iters: int):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    import torch

    from pipelinerl_amd import _native

    lib = _native.load()
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for rows, H in SHAPES:
        for add in (False, True):
            g = torch.Generator(device="cuda").manual_seed(rows + H)
            x = (torch.randn((rows, H), generator=g, device="cuda") * 2).to(torch.bfloat16)
            w = (1 + 0.1 * torch.randn(H, generator=g, device="cuda")).to(torch.bfloat16)
            dy = torch.randn((rows, H), generator=g, device="cuda").to(torch.bfloat16)
            dh = torch.randn((rows, H), generator=g, device="cuda").to(torch.bfloat16)
            y = torch.empty_like(x)
            rstd = torch.empty(rows, dtype=torch.float32, device="cuda")
            _native.check(lib.prl_rmsnorm_forward(x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), rows, H,
                                                  1e-6, st), "fwd")
            nb = ctypes.c_size_t(0)
            _native.check(lib.prl_rmsnorm_workspace_bytes(H, ctypes.byref(nb)), "ws")
            ws = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
            dx, dw = torch.empty_like(x), torch.empty_like(w)
            if add:
                f = lib.prl_add_rmsnorm_backward
                args = (dy.data_ptr(), dh.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                        dw.data_ptr(), ws.data_ptr(), nb.value, rows, H, st)
            else:
                f = lib.prl_rmsnorm_backward
                args = (dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(),
                        ws.data_ptr(), nb.value, rows, H, st)
            _native.check(f(*args), "bwd")
            torch.cuda.synchronize()
            ms = None
            if time_iters and rows == 8704 and add:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(time_iters):
                    f(*args)
                e1.record()
                e1.synchronize()
                ms = e0.elapsed_time(e1) / time_iters
            res[f"{rows}x{H}{'_add' if add else ''}"] = (dx.cpu(), dw.cpu(), ms)
    torch.save(res, out_path)


def run(lib: str | None, out: str, iters: int):
    env = dict(os.environ)
    if lib:
        env["PRL_LIB"] = lib
    else:
        env.pop("PRL_LIB", None)
    subprocess.run([sys.executable, __file__, "--child", out, str(iters)], env=env, check=True)


def main():
    import torch

    other = sys.argv[1]
    tmp = tempfile.mkdtemp()
    times = {"product": [], "other": []}
    outs = {}
    for rep in range(3):
        for name, lib in (("product", None), ("other", other)):
            p = os.path.join(tmp, f"{name}{rep}.pt")
            run(lib, p, 200)
            outs[name] = torch.load(p)
            times[name].append(round(outs[name]["8704x3584_add"][2] * 1e3, 2))
    rows = []
    for k in outs["product"]:
        a, b = outs["product"][k], outs["other"][k]
        rows.append({"case": k, "dx_equal": bool(torch.equal(a[0].view(torch.int16), b[0].view(torch.int16))),
                     "dw_equal": bool(torch.equal(a[1].view(torch.int16), b[1].view(torch.int16)))})
    nbytes = 4 * 8704 * 3584 * 2
    print(json.dumps({"other": other, "bits": rows, "add_rmsnorm_backward_8704x3584_us": times,
                      "algorithmic_bytes": nbytes,
                      "TBps_best": {k: round(nbytes / (min(v) * 1e-6) / 1e12, 3) for k, v in times.items()}}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
    else:
        main()
