"""Pin the numpy oracle (oracle/grpo_oracle.py) to the reference's own outputs.

Golden vectors come from running the reference rl_step in the build container
(tests/golden/make_golden.py).  Tolerances: fp32 reference vs float64 oracle, 2e-5
relative on per-token values and sums, 2e-6 absolute on dlogits (|dlogits| <= 1/batch).
"""

import json

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import grpo_oracle, synth


def _close(a, b, rtol=2e-5, atol=2e-6):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol)


def test_f1_oracle_matches_reference(f1):
    batches, out, cases = f1
    assert len(cases) >= 39
    for i, c in enumerate(cases):
        b = batches[c["batch"]]
        vals = b["values"] if c["value_head"] else None
        r = grpo_oracle.rl_step_oracle(b["logits"], b, c["cfg"], c["step"], c["max_step"], values=vals)
        assert abs(r["loss"] - c["loss"]) <= 2e-5 * max(1.0, abs(c["loss"])), (i, r["loss"], c["loss"])
        assert set(r["stats"]) == set(c["stats"]), (i, set(r["stats"]) ^ set(c["stats"]))
        for k, v in c["stats"].items():
            assert abs(r["stats"][k] - v) <= 2e-5 * max(1.0, abs(v)), (i, k, r["stats"][k], v)
        _close(r["new_logprobs"], out[f"case{i}__new_logprobs"])
        _close(r["entropy"], out[f"case{i}__entropy"])
        _close(r["dlogits"], out[f"case{i}__dlogits"], rtol=1e-4, atol=2e-7)
        if c["value_head"]:
            _close(r["dvalues"], out[f"case{i}__dvalues"], atol=1e-7)


def f2_batch():
    meta = json.loads((GOLDEN / "f2_meta.json").read_text())
    T, V, seed = meta["T"], meta["V"], meta["seed"]
    b = synth.packed_rl_batch(seed, [8, 8], [3, 3], id_range=151643, eos=151643)
    ids = b["input_ids"][0]
    lg = synth.to_bf16(synth.logits_rows(seed, np.arange(T), V, ids))
    x = lg[:-1].astype(np.float64)
    lse = np.log(np.exp(x - x.max(-1, keepdims=True)).sum(-1)) + x.max(-1)
    tl = x[np.arange(T - 1), ids[1:]] - lse
    lab = b["labels"][0] != -100
    u = synth.normal(seed + 3, np.arange(2 * T, dtype=np.uint64))
    old = np.zeros(T, np.float32)
    ref = np.zeros(T, np.float32)
    old[1:] = tl + 0.1 * u[:T - 1]
    ref[1:] = tl + 0.2 * u[T:2 * T - 1]
    old[~lab] = 0
    ref[~lab] = 0
    b["old_logprobs"] = old[None]
    b["ref_logprobs"] = ref[None]
    return meta, lg[None].astype(np.float32), b


@pytest.mark.slow
def test_f2_oracle_matches_reference_full_vocab():
    meta, lg, b = f2_batch()
    out = np.load(GOLDEN / "f2_outputs.npz")
    r = grpo_oracle.rl_step_oracle(lg, b, meta["cfg"], meta["step"], meta["max_step"])
    ref = meta["fp32"]
    assert abs(r["loss"] - ref["loss"]) <= 1e-5 * max(1, abs(ref["loss"]))
    for k, v in ref["stats"].items():
        assert abs(r["stats"][k] - v) <= 1e-4 * max(1.0, abs(v)), (k, r["stats"][k], v)
    _close(r["new_logprobs"], out["fp32__new_logprobs"], rtol=1e-5, atol=1e-5)
    _close(r["entropy"], out["fp32__entropy"], rtol=1e-5, atol=1e-5)
    d = r["dlogits"][0]
    T = meta["T"]
    tgt = b["input_ids"][0, 1:]
    _close(d[np.arange(T - 1), tgt], out["fp32__d_target"], rtol=1e-4, atol=1e-7)
    _close(d[:, :1024], out["fp32__d_cols"], rtol=1e-3, atol=1e-9)
    # bf16 reference path: log-softmax in bf16, so compare at the bf16 tolerance (relative 1e-2)
    _close(r["new_logprobs"], out["bf16__new_logprobs"], rtol=1e-2, atol=1e-2)
    _close(r["entropy"], out["bf16__entropy"], rtol=1e-2, atol=1e-2)


def test_oracle_error_behaviour(f1):
    batches, _, _ = f1
    b = batches["packed"]
    with pytest.raises(ValueError):
        grpo_oracle.rl_step_oracle(b["logits"], b, {"policy_loss": "nope", "batch_size": 4}, 0, 10)
    lg = b["logits"].copy()
    lg[0, 3, 5] = np.inf
    with pytest.raises(AssertionError):
        grpo_oracle.rl_step_oracle(lg, b, {"batch_size": 4}, 0, 10)
