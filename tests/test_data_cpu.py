"""populate_rl_data / prepare_rl_fields / collate_packed / sentinel batches vs the reference's
own outputs (fixture F3, tests/golden/make_golden.py)."""

import copy
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN


@pytest.fixture(scope="module")
def f3():
    return json.loads((GOLDEN / "f3_rl_data.json").read_text())


def test_populate_rl_data_matches_reference(f3):
    from pipelinerl_amd.finetune.rl import RLConfig, populate_rl_data

    for divide in (False, True):
        out = populate_rl_data(copy.deepcopy(f3["inputs"]), f3["eos"], RLConfig(divide_advantage_by_std=divide))
        want = f3["populate"][f"divide_{divide}"]
        assert len(out) == len(want)
        for got, exp in zip(out, want):
            for k in ("advantages", "group_tokens", "overflow", "num_labels"):
                np.testing.assert_allclose(np.asarray(got[k], np.float64), np.asarray(exp[k], np.float64),
                                           rtol=1e-12, atol=1e-12, err_msg=k)


def test_collate_packed_matches_reference(f3):
    import types

    from pipelinerl_amd.finetune.data import collate_packed
    from pipelinerl_amd.finetune.rl import RLConfig, populate_rl_data

    out = populate_rl_data(copy.deepcopy(f3["inputs"]), f3["eos"], RLConfig())
    tok = types.SimpleNamespace(eos_token_id=f3["eos"])
    for sp in (1, 4):
        b = collate_packed(out[:5], tok, sp)
        want = f3["collate_packed"][f"sp{sp}"]
        got = {k: (v.tolist() if isinstance(v, torch.Tensor) else v) for k, v in b.model_dump().items() if v is not None}
        assert set(got) == set(want), set(got) ^ set(want)
        for k, v in want.items():
            if isinstance(v, list):
                np.testing.assert_allclose(np.asarray(got[k], np.float64), np.asarray(v, np.float64), err_msg=k)
            else:
                assert got[k] == v, k


def test_prepare_rl_fields_and_errors():
    from pipelinerl_amd.finetune.rl import prepare_rl_fields

    enc = {"input_ids": [1, 2, 3, 4], "labels": [-100, -100, 3, 4]}
    out = prepare_rl_fields(dict(enc), 1.0, [-0.5, -0.25], [-0.6, -0.2])
    assert out["old_logprobs"] == [0, 0, -0.5, -0.25]
    assert out["num_labels"] == [0, 0, 1, 1]
    with pytest.raises(AssertionError):
        prepare_rl_fields(dict(enc), 1.0, [-0.5], [-0.6])


def test_sentinel_batch_layout():
    import types

    from pipelinerl_amd.finetune.utils import create_sentinel_batch

    b = create_sentinel_batch(tokenizer=types.SimpleNamespace(eos_token_id=9), model_version=4)
    assert b.sentinel and b.is_packed and b.model_version == 4
    assert b.input_ids.tolist() == [[9] * 8] and b.labels.eq(-100).all()
    assert b.seq_boundaries.tolist() == [0, 8]


def test_pipeline_batch_encoding_roundtrip_and_slices():
    from pipelinerl_amd.finetune.types import PipelineBatchEncoding
    from pipelinerl_amd.streams import dumps

    T = 12
    b = PipelineBatchEncoding(input_ids=list(range(T)), attention_mask=[1] * T, labels=[-100] * 3 + list(range(3, T)),
                              position_ids=list(range(T)), rewards=[1.0] * T, advantages=[0.5] * T,
                              ref_logprobs=[0.0] * T, old_logprobs=[0.0] * T, group_tokens=[12.0] * T,
                              num_labels=[9.0] * T, overflow=[0.0] * T, model_version=2, is_packed=True,
                              seq_boundaries=[0, T])
    b = PipelineBatchEncoding(**{k: v for k, v in b.model_dump().items()})  # tensors accepted too
    d = json.loads(dumps(b))
    b2 = PipelineBatchEncoding(**d)
    assert torch.equal(b2.labels, b.labels) and b2.input_ids.dtype == torch.long
    assert b2.rewards.dtype == torch.float32 and b2.seq_boundaries.dtype == torch.int32
    with pytest.raises(ValueError):
        b.make_slices(5)


def test_label_rows_from_host_and_to_device():
    """PipelineBatchEncoding.label_rows_from_host: the loss rows q = b*(L-1)+t with a label
    (rl/__init__.py:152-153's mask, flattened), carried through to_device."""
    import torch

    from pipelinerl_amd.finetune.types import PipelineBatchEncoding

    lab = torch.tensor([[-100, -100, 5, 6, -100, 7], [-100, 1, 2, -100, -100, -100]])
    z = torch.zeros(2, 6)
    b = PipelineBatchEncoding(input_ids=lab.clamp(min=0), attention_mask=torch.ones_like(lab), labels=lab,
                              rewards=z, advantages=z, ref_logprobs=z, old_logprobs=z, group_tokens=z + 1,
                              num_labels=z, overflow=z, model_version=0)
    rows = b.label_rows_from_host()
    assert rows.tolist() == [1, 2, 4, 5, 6]  # row 0: t = 1, 2, 4; row 1: t = 0, 1 (q = 5 + t)
    b.to_device("cpu")
    assert b._label_rows is rows or torch.equal(b._label_rows, rows)
