"""F5 fixture: the preprocessor's zero-advantage group filter (pipelinerl/preprocess.py:287-324,
applied when ``rl.filter_zero_advantage_groups`` is set, :509-513) on synthetic populated chunks.

Run in the build container only (reads /root/reference; writes data):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_f5.py

preprocess.py itself does not import here (litellm, tapeagents), so the one function is taken
from the file's syntax tree and run on its own (it uses no imports); nothing else of the module
is executed.  Inputs cover: groups with every advantage zero, tiny (|a| <= 1e-6) and just-over
values, negative values, NaN, interleaved group ids, empty advantage lists, an all-zero chunk.
"""

from __future__ import annotations

import ast
import json
import math
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference/pipelinerl/preprocess.py")


def reference_filter():
    tree = ast.parse(REF.read_text())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "filter_zero_advantage_groups")
    ns: dict = {}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), str(REF), "exec"), ns)
    return ns["filter_zero_advantage_groups"]


def chunks() -> list[list[dict]]:
    rng = np.random.default_rng(5)
    out = []
    for c in range(6):
        data = []
        n_groups = int(rng.integers(1, 6))
        for i in range(int(rng.integers(1, 24))):
            g = int(rng.integers(0, n_groups))
            n = int(rng.integers(0, 6))
            kind = rng.integers(0, 6)
            if kind == 0:
                adv = rng.normal(0, 1, n).tolist()
            elif kind == 1:
                adv = [0.0] * n
            elif kind == 2:
                adv = rng.choice([1e-7, -1e-6, 1e-6, -2e-6, 1.5e-6], n).tolist()
            elif kind == 3:
                adv = [float("nan")] * n
            else:
                adv = ([0.0] * n)
            data.append({"group_id": f"g{g}_{c}", "rollout_index": i, "advantages": adv})
        if c == 5:
            for e in data:
                e["advantages"] = [0.0] * len(e["advantages"])
        out.append(data)
    return out


def enc(x):
    return "nan" if isinstance(x, float) and math.isnan(x) else x


def main():
    f = reference_filter()
    cases = []
    for data in chunks():
        kept, dropped = f(data, 1e-6)
        cases.append({"input": [{**e, "advantages": [enc(a) for a in e["advantages"]]} for e in data],
                      "kept": [[e["group_id"], e["rollout_index"]] for e in kept], "dropped": dropped})
    (HERE / "f5_zero_adv_filter.json").write_text(json.dumps({"source": "pipelinerl/preprocess.py:287-324",
                                                               "epsilon": 1e-6, "cases": cases}))
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
