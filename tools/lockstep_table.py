"""Regenerate workloads.LOCKSTEP_EFFICIENCY: the lockstep protocol's efficiency (the loop's order)
of an optimizer step of C3 (4096 samples) at N data-parallel ranks, from workloads.lockstep_cost on
the preprocessor's own packing of C3's rollouts (a few minutes per N on one CPU core).

    python tools/lockstep_table.py [N ...]
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))


def main() -> None:
    from pipelinerl_amd import workloads

    ns = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    print(json.dumps({n: workloads.lockstep_cost("c3", n, 4096 // n)["efficiency"]["loop"] for n in ns}))


if __name__ == "__main__":
    main()
