"""Checkpoints of a value-head model (reference conf/finetune/ppo.yaml, actor_critic.yaml) whose
parameters were re-homed into one flat buffer (finetune.flat_parameters, weight_update.py): the
saved LM has the LM's own key names (vLLM and from_pretrained load it), the value head goes to
value_head.pt, and a resume loads both back (value_model.py:124-192)."""

from __future__ import annotations

import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))


def _args(model_dir: Path):
    from pipelinerl_amd.config import Cfg

    return Cfg.wrap(dict(config_name=str(model_dir), load_as_bf16=True, attn_implementation="sdpa",
                         gradient_checkpointing=False))


@pytest.mark.parametrize("flat", [True, False], ids=["flat", "plain"])
def test_value_head_checkpoint_round_trip(tmp_path, flat):
    from loop_helpers import tiny_model_dir
    from safetensors.torch import load_file

    from pipelinerl_amd.finetune.checkpoints import load_model, save_model_and_tokenizer
    from pipelinerl_amd.weight_update import rehome_parameters

    vh_class = "causal-language-modeling-with-value-head"
    torch.manual_seed(0)
    model = load_model(_args(tiny_model_dir(tmp_path)), vh_class, tmp_path / "none", torch.device("cpu"))
    if flat:
        assert rehome_parameters(model) is not None
        assert model.pretrained_model._prl_flat_params
    with torch.no_grad():
        for i, p in enumerate(model.parameters()):
            p.add_(0.01 * (i + 1))
    want = {n: p.detach().clone() for n, p in model.state_dict().items()}
    out = tmp_path / "current"
    save_model_and_tokenizer(out, model, object(), safe_serialization=True)

    saved = load_file(str(out / "model.safetensors"))
    lm_keys = {k[len("pretrained_model."):] for k in want if k.startswith("pretrained_model.")}
    assert set(saved) <= lm_keys and not any(k.startswith(("pretrained_model.", "value_head.")) for k in saved)
    assert "lm_head.weight" not in saved  # tied to the embedding (tie_word_embeddings)
    for k, t in saved.items():
        assert torch.equal(t, want["pretrained_model." + k]), k
    head = torch.load(out / "value_head.pt", weights_only=True)
    assert set(head) == {"output.weight", "output.bias"}

    torch.manual_seed(1)  # a different random head: the saved one must replace it
    back = load_model(_args(tiny_model_dir(tmp_path)), vh_class, out, torch.device("cpu"))
    got = back.state_dict()
    assert set(got) == set(want)
    for k in want:
        assert torch.equal(got[k], want[k]), k


def test_value_head_state_dict_split_rejects_foreign_keys():
    from pipelinerl_amd.finetune.value_model import split_value_head_state_dict

    lm, vh = split_value_head_state_dict({"pretrained_model.a": 1, "value_head.b": 2})
    assert lm == {"a": 1} and vh == {"b": 2}
    with pytest.raises(ValueError, match="Unexpected key"):
        split_value_head_state_dict({"model.a": 1})
