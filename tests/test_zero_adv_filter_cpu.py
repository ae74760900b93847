"""The preprocessor's zero-advantage group filter vs the reference's own outputs (F5 fixture,
tests/golden/make_f5.py: pipelinerl/preprocess.py:287-324 run on the same chunks)."""
import json
from pathlib import Path

from pipelinerl_amd.finetune.packing import filter_zero_advantage_groups

GOLDEN = Path(__file__).resolve().parent / "golden" / "f5_zero_adv_filter.json"


def _dec(x):
    return float("nan") if x == "nan" else x


def test_filter_matches_reference_fixture():
    d = json.loads(GOLDEN.read_text())
    for case in d["cases"]:
        data = [{**e, "advantages": [_dec(a) for a in e["advantages"]]} for e in case["input"]]
        kept, dropped = filter_zero_advantage_groups(data, d["epsilon"])
        assert [[e["group_id"], e["rollout_index"]] for e in kept] == case["kept"]
        assert dropped == case["dropped"]
        assert all(k is next(e for e in data if e is k) for k in kept)  # the same dicts, not copies


def test_filter_edges():
    assert filter_zero_advantage_groups([]) == ([], 0)
    one = [{"group_id": "a", "advantages": [0.0, 2e-6]}, {"group_id": "b", "advantages": [1e-6]}]
    kept, dropped = filter_zero_advantage_groups(one)
    assert [e["group_id"] for e in kept] == ["a"] and dropped == 1
