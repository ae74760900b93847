"""The trainer's stats/* and throughput/* keys against the reference's own expression
(finetune_loop.py:725-764), evaluated at world size 2 into F7 (tests/golden/make_f7.py)."""

from __future__ import annotations

import json
import math
import types
from pathlib import Path

import pytest

from pipelinerl_amd.finetune.types import TrainingMetrics
from pipelinerl_amd.finetune_loop import step_metrics

F7 = Path(__file__).parent / "golden" / "f7_step_metrics.json"


@pytest.mark.parametrize("case", json.loads(F7.read_text()), ids=lambda c: f"world{c['inputs']['world']}")
def test_step_metrics_match_the_reference_formulas(case):
    c = case["inputs"]
    m = TrainingMetrics(**c["metrics"])
    q = types.SimpleNamespace(qsize=lambda: c["qsize"])
    got = step_metrics(m, dict(c["lag"]), q, c["tokens"], c["passes"], c["mbs"], c["world"], c["samples_per_step"],
                       c["step_took"])
    exp = case["expected"]
    assert set(exp) <= set(got)
    for k, v in exp.items():
        assert math.isclose(float(got[k]), float(v), rel_tol=1e-12, abs_tol=0), (k, got[k], v)
    # the one added key: the whole job's rate over the step's wall time
    assert set(got) - set(exp) == {"throughput/real_tokens_per_sec_all_ranks"}
    assert math.isclose(got["throughput/real_tokens_per_sec_all_ranks"],
                        exp["throughput/real_tokens_per_sec"] * c["world"], rel_tol=1e-12)
