"""The trainer-input packing protocol (finetune/packing.py MicroBatchPacker) vs the reference's own
write loop (F6 fixture, tests/golden/make_f6.py: pipelinerl/preprocess.py:557-613 executed on the
same rollouts, chunk by chunk): the same writes, to the same lead trainers, in the same order —
micro-batch contents, sequence boundaries, padding, sentinels and their model versions."""
import copy
import json
import types
from pathlib import Path

import pytest

from pipelinerl_amd.finetune.packing import MicroBatchPacker

GOLDEN = json.loads((Path(__file__).resolve().parent / "golden" / "f6_packing.json").read_text())
FIELDS = ["input_ids", "labels", "position_ids", "attention_mask", "rewards", "advantages", "ref_logprobs",
          "old_logprobs", "group_tokens", "num_labels", "overflow"]


def _encode(tid, b):
    rec = {"trainer": int(tid), "sentinel": bool(b.sentinel), "model_version": int(b.model_version),
           "padding": int(b.padding), "is_packed": bool(b.is_packed),
           "seq_boundaries": [int(x) for x in b.seq_boundaries.tolist()]}
    for f in FIELDS:
        v = getattr(b, f, None)
        if v is not None:
            rec[f] = [float(x) for x in v.reshape(-1).tolist()] if v.is_floating_point() else \
                [int(x) for x in v.reshape(-1).tolist()]
    return rec


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_packer_matches_reference_write_loop(case):
    packer = MicroBatchPacker(case["num_trainers"], case["seq_length"], case["samples_per_lead_per_step"],
                              types.SimpleNamespace(eos_token_id=GOLDEN["eos"]), seq_parallel=case["seq_parallel"])
    data = copy.deepcopy(case["input"])
    writes, pos = [], 0
    for size in case["chunks"]:
        writes += packer.feed(data[pos:pos + size])
        pos += size
    got = [_encode(t, b) for t, b in writes]
    want = case["writes"]
    assert [(w["trainer"], w["sentinel"]) for w in got] == [(w["trainer"], w["sentinel"]) for w in want]
    for i, (g, w) in enumerate(zip(got, want)):
        assert set(g) == set(w), (i, set(g) ^ set(w))
        for k in w:
            assert g[k] == w[k], (i, k)
    sp = case["seq_parallel"]
    for i, ((t, b), want_slices) in enumerate(zip(writes, case["slices"])):  # types.py:144-180
        got_slices = [_encode(t + j, s) for j, s in enumerate(b.make_slices(sp))] if sp > 1 else []
        assert len(got_slices) == len(want_slices), i
        for j, (g, w) in enumerate(zip(got_slices, want_slices)):
            assert set(g) == set(w) and all(g[k] == w[k] for k in w), (i, j, [k for k in w if g.get(k) != w[k]])
