"""Causal LM + scalar value head (contract of pipelinerl/finetune/value_model.py:40-211).

values = Linear(H -> 1)(last hidden state).squeeze(-1); rl_step feeds them to the fused loss
head, which returns d loss / d values (value loss and the advantage-baseline statistics).
"""

from __future__ import annotations

import types

import torch
from torch import nn


class ValueHead(nn.Module):
    def __init__(self, hidden_size: int):
        super().__init__()
        self.output = nn.Linear(hidden_size, 1)
        g = torch.Generator().manual_seed(42)
        with torch.no_grad():
            self.output.weight.normal_(0.0, 1e-3, generator=g)
            self.output.bias.zero_()

    def forward(self, hidden_states: torch.Tensor) -> torch.Tensor:
        return self.output(hidden_states).squeeze(-1)


class AutoModelForCausalLMWithValueHead(nn.Module):
    def __init__(self, pretrained_model):
        super().__init__()
        self.pretrained_model = pretrained_model
        self.config = pretrained_model.config
        self.value_head = ValueHead(self.config.hidden_size).to(next(pretrained_model.parameters()).dtype)
        self.main_input_name = getattr(pretrained_model, "main_input_name", "input_ids")

    def forward(self, input_ids, attention_mask=None, position_ids=None, **kw):
        out = self.pretrained_model(input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids,
                                    output_hidden_states=True, return_dict=True, **kw)
        values = self.value_head(out.hidden_states[-1])
        return types.SimpleNamespace(logits=out.logits, value=values, loss=getattr(out, "loss", None))

    def gradient_checkpointing_enable(self, gradient_checkpointing_kwargs=None):
        self.pretrained_model.gradient_checkpointing_enable(gradient_checkpointing_kwargs)

    def save_pretrained(self, save_directory, safe_serialization: bool = True, state_dict: dict | None = None, **kw):
        """value_model.py:124-172: the LM (loadable by vLLM as is) and ``value_head.pt`` apart; a
        given ``state_dict`` is in this wrapper's namespace (``pretrained_model.*`` / ``value_head.*``)
        and split by prefix, any other key raising ValueError."""
        if state_dict is None:
            state_dict = self.state_dict()
        lm, vh = split_value_head_state_dict(state_dict)
        self.pretrained_model.save_pretrained(save_directory, safe_serialization=safe_serialization, state_dict=lm,
                                              **kw)
        torch.save(vh, f"{save_directory}/value_head.pt")

    def load_value_head(self, directory) -> bool:
        """value_model.py:189-192: the saved head, when ``directory`` holds one (plain tensors only)."""
        path = f"{directory}/value_head.pt"
        try:
            sd = torch.load(path, map_location="cpu", weights_only=True)
        except FileNotFoundError:
            return False
        self.value_head.load_state_dict(sd)
        return True


def split_value_head_state_dict(state_dict: dict) -> tuple[dict, dict]:
    """(the LM's state dict in its own namespace, the value head's) from the wrapper's."""
    lm, vh = {}, {}
    for k, v in state_dict.items():
        if k.startswith("value_head."):
            vh[k[len("value_head."):]] = v
        elif k.startswith("pretrained_model."):
            lm[k[len("pretrained_model."):]] = v
        else:
            raise ValueError(f"Unexpected key in state dict: {k}. "
                             "Expected keys should start with 'value_head.' or 'pretrained_model.'.")
    return lm, vh
