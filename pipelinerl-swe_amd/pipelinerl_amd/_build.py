"""Build libprl_hip.so (HIP, gfx950 only) in-tree with hipcc.

    python -m pipelinerl_amd._build [--resource-usage]

The library is the C-ABI declared in include/prl_hip.h.  libprl_comm.so (include/prl_comm.h,
csrc/comm.cpp) is the separate RCCL-linked communicator library.  It is built next to this file so
it travels with the repository snapshot to the GPU box (a JIT cache would not).
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parents[1]
INCLUDE = REPO / "include"
CSRC = PKG / "csrc"
LIB = PKG / "libprl_hip.so"
COMM_LIB = PKG / "libprl_comm.so"
GEMM_LIB = PKG / "libprl_gemm.so"
DATA_LIB = PKG / "libprl_data.so"
ARCH = "gfx950"
SOURCES = ["grpo_loss.hip", "flat_pack.hip", "model_ops.hip", "attn_bwd.hip", "adamw.hip"]
# per-source compiler flags (beside the common ones below)
FILE_FLAGS: dict[str, list[str]] = {}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the MI355X library cannot be built")


def _stale() -> bool:
    if not LIB.exists():
        return True
    mt = LIB.stat().st_mtime
    deps = list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + [INCLUDE / "prl_hip.h", Path(__file__)]
    return any(d.stat().st_mtime > mt for d in deps)


VARIANT_DIR = PKG / "variants"


def build_comm(force: bool = False) -> Path:
    """libprl_comm.so: host code over RCCL (no device code), rpath to the ROCm libraries."""
    src, hdr = CSRC / "comm.cpp", INCLUDE / "prl_comm.h"
    if not force and COMM_LIB.exists() and COMM_LIB.stat().st_mtime > max(src.stat().st_mtime,
                                                                           hdr.stat().st_mtime):
        return COMM_LIB
    rocm = Path(hipcc()).resolve().parents[1]
    tmp = COMM_LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{INCLUDE}", f"-I{rocm / 'include'}",
           str(src), "-o", str(tmp), f"-L{rocm / 'lib'}", "-lrccl", f"-Wl,-rpath,{rocm / 'lib'}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for comm.cpp:\n{r.stderr[-8000:]}")
    os.replace(tmp, COMM_LIB)
    return COMM_LIB


def build_gemm(force: bool = False) -> Path:
    """libprl_gemm.so: host code over hipBLASLt (no device code).  It does not link hipBLASLt: it
    dlopens the ROCm installation's copy (path baked in here) at first use, next to the copy torch
    bundles; its HIP runtime dependency resolves to the one torch loaded."""
    src, hdr = CSRC / "gemm.cpp", INCLUDE / "prl_gemm.h"
    if not force and GEMM_LIB.exists() and GEMM_LIB.stat().st_mtime > max(src.stat().st_mtime,
                                                                           hdr.stat().st_mtime):
        return GEMM_LIB
    rocm = Path(hipcc()).resolve().parents[1]
    tmp = GEMM_LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}", f"-I{INCLUDE}",
           f"-I{rocm / 'include'}", f"-DPRL_HIPBLASLT_PATH=\"{rocm / 'lib' / 'libhipblaslt.so.1'}\"", str(src),
           "-o", str(tmp), "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for gemm.cpp:\n{r.stderr[-8000:]}")
    os.replace(tmp, GEMM_LIB)
    return GEMM_LIB


def build_data(force: bool = False) -> Path:
    """libprl_data.so: host-only C++ (the stream codec and preprocessing arithmetic,
    include/prl_data.h); g++, no HIP."""
    src, hdr, pyconv = CSRC / "data.cpp", INCLUDE / "prl_data.h", CSRC / "pyconv.cpp"
    if not force and DATA_LIB.exists() and DATA_LIB.stat().st_mtime > max(
            src.stat().st_mtime, hdr.stat().st_mtime, pyconv.stat().st_mtime):
        return DATA_LIB
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no C++ compiler found for libprl_data.so")
    tmp = DATA_LIB.with_suffix(".so.tmp")
    import sysconfig
    pyinc = Path(sysconfig.get_paths()["include"])
    # the Python-object helpers (pyconv.cpp) need Python.h; their symbols resolve against the
    # interpreter that loads the library
    extra = [f"-I{pyinc}", str(pyconv)] if (pyinc / "Python.h").exists() else []
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{INCLUDE}", str(src), *extra, "-o", str(tmp),
           "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{cxx} failed for data.cpp:\n{r.stderr[-8000:]}")
    os.replace(tmp, DATA_LIB)
    return DATA_LIB


def build(force: bool = False, resource_usage: bool = False, verbose: bool = False,
          defines: dict[str, str] | None = None, out: Path | None = None, extra_flags: list[str] | None = None) -> Path:
    target = out or LIB
    if out is None and not force and not resource_usage and not _stale():
        return LIB
    cc = hipcc()
    objdir = PKG / "build" / (target.stem if out is not None else "main")
    objdir.mkdir(parents=True, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}",
             "-Wall", "-Wno-unused-function"]
    if resource_usage:
        flags.append("-Rpass-analysis=kernel-resource-usage")
    for k, v in (defines or {}).items():
        flags.append(f"-D{k}={v}")
    flags += list(extra_flags or [])

    def compile_one(src: str):
        obj = objdir / (Path(src).stem + ".o")
        cmd = [cc, *flags, *FILE_FLAGS.get(src, []), "-c", str(CSRC / src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
        return obj, r.stderr

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        results = list(ex.map(compile_one, SOURCES))
    if resource_usage or verbose:
        for (_, err), src in zip(results, SOURCES):
            (objdir / (Path(src).stem + ".resource.txt")).write_text(err)
    target.parent.mkdir(parents=True, exist_ok=True)
    tmp = target.with_suffix(".so.tmp")
    cmd = [cc, "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *[str(o) for o, _ in results]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
    os.replace(tmp, target)
    return target


def build_variant(name: str, defines: dict[str, str], extra_flags: list[str] | None = None) -> Path:
    """An experiment build (e.g. cache-policy A/B) at variants/libprl_hip_<name>.so; load it
    with PRL_LIB=<path>."""
    return build(defines=defines, out=VARIANT_DIR / f"libprl_hip_{name}.so", extra_flags=extra_flags)


if __name__ == "__main__":
    out = build(force=True, resource_usage="--resource-usage" in sys.argv, verbose=True)
    print(out)
    print(build_comm(force=True))
    print(build_gemm(force=True))
    print(build_data(force=True))
