"""patch_model on a CPU model: every patched path (RMSNorm, SwiGLU MLP, the q/k/v group, the
decoder-layer forward with the fused residual adds) must fall back to the eager HF code off the
GPU and leave the model's outputs and gradients bit-identical (no HIP call is made: the kernels'
preconditions fail on CPU tensors).  The GPU tests cover the fused paths themselves."""

import copy

import torch


def test_patched_cpu_model_equals_eager(tmp_path):
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd.finetune.model_ops import patch_model

    cfg = AutoConfig.from_pretrained(tiny_model_dir(tmp_path, vocab=128))
    torch.manual_seed(0)
    eager = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32)
    patched = copy.deepcopy(eager)
    counts = patch_model(patched)
    n = cfg.num_hidden_layers
    assert counts["rmsnorm"] == 2 * n + 1 and counts["swiglu_mlp"] == n
    assert counts["qkv_groups"] == n and counts["add_norm_layers"] == n
    ids = torch.randint(0, 128, (1, 24))
    outs = []
    for m in (eager, patched):
        lg = m(input_ids=ids, use_cache=False).logits
        lg.pow(2).mean().backward()
        outs.append(lg.detach())
    assert torch.equal(outs[0], outs[1])
    for (name, p), (_, q) in zip(eager.named_parameters(), patched.named_parameters()):
        assert torch.equal(p.grad, q.grad), name
    # no hand-over left pending on any norm after a full forward
    assert all(m.__dict__.get("_prl_pending") is None for m in patched.modules())


def test_decoder_patch_keeps_the_installed_layer_contract(tmp_path):
    """transformers 5.x layers return a tensor; 4.x layers (the reference pins 4.51.1,
    pyproject.toml:20) return a tuple that Qwen2Model indexes with [0], and gradient
    checkpointing passes their arguments positionally.  The patched forward must return what
    the original returns, for either contract."""
    import types

    from pipelinerl_amd.finetune import model_ops

    class Norm(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.weight = torch.nn.Parameter(torch.ones(8))
            self.variance_epsilon = 1e-6

        def forward(self, x):
            return x * 2.0

    class Attn(torch.nn.Module):
        def forward(self, hidden_states, position_embeddings=None, attention_mask=None, past_key_value=None,
                    cache_position=None, **kwargs):
            self.seen = dict(kwargs, attention_mask=attention_mask, past_key_value=past_key_value,
                             position_embeddings=position_embeddings)
            return hidden_states + 1.0, "weights"

    class Layer4x(torch.nn.Module):  # transformers 4.51 Qwen2DecoderLayer.forward contract
        def __init__(self):
            super().__init__()
            self.input_layernorm, self.post_attention_layernorm = Norm(), Norm()
            self.self_attn, self.mlp = Attn(), torch.nn.Identity()

        def forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                    output_attentions=False, use_cache=False, cache_position=None, position_embeddings=None,
                    **kwargs):
            r = hidden_states
            a, w = self.self_attn(hidden_states=self.input_layernorm(hidden_states), attention_mask=attention_mask,
                                  position_ids=position_ids, past_key_value=past_key_value,
                                  output_attentions=output_attentions, use_cache=use_cache,
                                  cache_position=cache_position, position_embeddings=position_embeddings, **kwargs)
            h = r + a
            h = h + self.mlp(self.post_attention_layernorm(h))
            return (h, w) if output_attentions else (h,)

    class Layer5x(Layer4x):  # transformers 5.x contract: tensor out, past_key_values
        def forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_values=None,
                    use_cache=False, position_embeddings=None, **kwargs):
            r = hidden_states
            a, _ = self.self_attn(hidden_states=self.input_layernorm(hidden_states), attention_mask=attention_mask,
                                  position_ids=position_ids, past_key_values=past_key_values, use_cache=use_cache,
                                  position_embeddings=position_embeddings, **kwargs)
            h = r + a
            return h + self.mlp(self.post_attention_layernorm(h))

    x = torch.randn(1, 5, 8)
    pe = (torch.zeros(1, 5, 8), torch.ones(1, 5, 8))
    for cls in (Layer4x, Layer5x):
        layer = cls()
        want = layer(x, None, None, None, position_embeddings=pe) if cls is Layer5x else \
            layer(x, None, None, None, False, False, None, pe)
        layer.__dict__["_prl_orig_forward"] = layer.forward
        layer.forward = types.MethodType(model_ops._decoder_forward, layer)
        if cls is Layer4x:
            got = layer(x, None, None, None, False, False, None, pe)  # checkpointing: positional
            assert isinstance(got, tuple) and len(got) == 1 and torch.equal(got[0], want[0])
            got = layer(x, attention_mask=None, position_embeddings=pe, output_attentions=True)
            assert isinstance(got, tuple) and got[1] == "weights" and torch.equal(got[0], want[0])
            assert layer.self_attn.seen["position_embeddings"] is pe
        else:
            got = layer(x, position_embeddings=pe, past_key_values=None)
            assert isinstance(got, torch.Tensor) and torch.equal(got, want)


def test_fused_weight_cache_invalidated_by_known_writers():
    """model_ops._fused_weight keys its cat(Wg, Wu) cache on version counters, which a write
    through ``p.data`` or a raw pointer does not move; the build's own writers also call
    weights_written() (PrlAdamW.step, HipFlatPacker.unflatten), which drops every cache."""
    import torch

    from pipelinerl_amd.finetune import model_ops

    holder = torch.nn.Module()
    wg = torch.nn.Parameter(torch.ones(2, 3))
    wu = torch.nn.Parameter(torch.zeros(2, 3))
    a = model_ops._fused_weight(holder, (wg, wu))
    assert model_ops._fused_weight(holder, (wg, wu)) is a  # cached
    wg.data.fill_(5.0)  # p.data has its own version counter: the parameter's does not move
    assert model_ops._fused_weight(holder, (wg, wu)) is a  # stale (the hazard)
    model_ops.weights_written()
    b = model_ops._fused_weight(holder, (wg, wu))
    assert b is not a and float(b[0, 0]) == 5.0
