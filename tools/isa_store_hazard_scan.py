"""Scan gfx950 ISA for the VMEM store-data write-after-read hazard (NV = 24 root cause).

A vector-memory store with more than 8 bytes of data (dwordx3 / dwordx4) reads its data VGPRs
after it issues; a VALU instruction that overwrites one of them in the very next issue slot can
replace the data the store writes (observed on MI355X: tools/nv24_probe.py, profiles/r03_nv24_*).
LLVM's hazard recognizer inserts the wait state for stores WITHOUT a register in soffset only
(it assumes an SGPR soffset removes the hazard), so ``buffer_store_dwordx4 v[..], v, s[..], sN``
followed directly by a VALU write of its data is emitted with no wait state.

Reports every store(x3/x4) whose next instruction (no s_nop / other instruction between) is a
VALU writing one of its data VGPRs.  Usage: python tools/isa_store_hazard_scan.py file.s [...]
(or import ``scan`` / ``compile_isa``)."""
from __future__ import annotations

import re
import subprocess
import sys
from pathlib import Path

STORE = re.compile(r"^\s*(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\s+(.*)$")
VRANGE = re.compile(r"v\[(\d+):(\d+)\]")
FUNC = re.compile(r"^([A-Za-z_$][\w$.]*):\s*(;.*)?$")


def _regs(tok: str) -> set[int]:
    m = VRANGE.fullmatch(tok.strip())
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok.strip())
    return {int(m.group(1))} if m else set()


def _data_operand(kind: str, ops: list[str]) -> str:
    # buffer_store: vdata, vaddr, srsrc, soffset ; global_store: vaddr, vdata, saddr|off ;
    # flat_store: vaddr, vdata ; scratch_store: vaddr|off, vdata, saddr|off
    return ops[0] if kind == "buffer" else ops[1]


def scan(isa: str) -> list[dict]:
    out, func = [], None
    lines = isa.split("\n")
    for i, line in enumerate(lines):
        fm = FUNC.match(line)
        if fm and not line.startswith("."):
            func = fm.group(1)
        m = STORE.match(line)
        if not m:
            continue
        ops = [o.strip() for o in m.group(3).split(";")[0].split(",")]
        data = _regs(_data_operand(m.group(1), ops))
        soffset_sgpr = m.group(1) == "buffer" and len(ops) > 3 and re.match(r"s\d+|s\[", ops[3]) is not None
        j = i + 1
        while j < len(lines):  # the next instruction (skip blank lines, comments, labels)
            t = lines[j].strip()
            if t and not t.startswith(";") and not t.startswith(".") and not FUNC.match(t):
                break
            j += 1
        if j >= len(lines):
            continue
        nxt = lines[j].strip()
        name = nxt.split()[0] if nxt else ""
        if not name.startswith("v_") or name.startswith("v_readlane") or name.startswith("v_cmp"):
            continue
        dst = nxt[len(name):].split(",")[0]
        if _regs(dst) & data:
            out.append({"function": func, "line": i + 1, "store": line.strip(), "next": nxt,
                        "soffset_sgpr": bool(soffset_sgpr)})
    return out


def compile_isa(src: Path, defines: dict[str, str] | None = None, include: list[Path] = ()) -> str:
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", "-",
           *[f"-I{p}" for p in include], *[f"-D{k}={v}" for k, v in (defines or {}).items()], str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    return r.stdout


if __name__ == "__main__":
    bad = 0
    for f in sys.argv[1:]:
        hits = scan(Path(f).read_text())
        bad += len(hits)
        for h in hits:
            print(f"{f}:{h['line']} [{h['function']}] {h['store']}  ->  {h['next']}")
    sys.exit(1 if bad else 0)
