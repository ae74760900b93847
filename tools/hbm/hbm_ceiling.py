"""Measure the box's read+write streaming ceiling for the loss head's byte mix (20 GB in,
20 GB out) with torch copy_ and a 16-B/lane grid-stride HIP copy (tools/hbm/stream_copy.hip)."""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
so = HERE / "libstream_copy.so"
if not so.exists():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                           str(HERE / "stream_copy.hip"), "-o", str(so)])
lib = ctypes.CDLL(str(so))
lib.probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
if __name__ == "__main__" and torch.cuda.is_available():
    nbytes = 65536 * 151936 * 2
    a = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda").normal_()
    b = torch.empty_like(a)
    res = {}

    def timeit(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        return round(2 * nbytes / (ms * 1e-3) / 1e9, 1), round(ms, 4)

    res["torch_copy_"] = timeit(lambda: b.copy_(a))
    st = torch.cuda.current_stream().cuda_stream
    for variant, name in [(0, "u4_plain"), (1, "u4_nt"), (2, "u8_nt")]:
        for grid in (1024, 2048, 4096, 8192):
            res[f"hip_{name}_g{grid}"] = timeit(lambda: lib.probe_copy(a.data_ptr(), b.data_ptr(), nbytes, grid, variant, st))
    print(json.dumps({"bytes_read": nbytes, "bytes_written": nbytes, "GBps_ms": res}), flush=True)
    if "--sweep" in sys.argv:
        # size sweep (bytes per direction) of the best copy forms, plus one-direction streams.
        # GB/s counts read + write bytes for copies, one direction for read-only / write-only.
        sweep = {}
        for sz in (512 << 20, 2 << 30, 8 << 30, nbytes):
            for variant, name, grid in [(2, "u8_nt", 8192), (1, "u4_nt", 1024), (1, "u4_nt", 4096)]:
                gbps, ms = timeit(lambda: lib.probe_copy(a.data_ptr(), b.data_ptr(), sz, grid, variant, st))
                sweep[f"copy_{name}_g{grid}_{sz >> 20}MiB"] = [round(gbps * sz / nbytes, 1), ms]
            for grid in (1024, 4096, 8192):
                gbps, ms = timeit(lambda: lib.probe_copy(a.data_ptr(), b.data_ptr(), sz, grid, 3, st))
                sweep[f"read_g{grid}_{sz >> 20}MiB"] = [round(gbps * sz / nbytes / 2, 1), ms]
                gbps, ms = timeit(lambda: lib.probe_copy(a.data_ptr(), b.data_ptr(), sz, grid, 4, st))
                sweep[f"write_g{grid}_{sz >> 20}MiB"] = [round(gbps * sz / nbytes / 2, 1), ms]
        print(json.dumps({"sweep_GBps_ms": sweep}), flush=True)
