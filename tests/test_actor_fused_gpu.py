"""The bucketed receive into vLLM's fused parameter layout on the GPU: one HIP unflatten pass writes
the trainer's q / k / v and gate / up tensors straight into the row blocks of the actor's
qkv_proj / gate_up_proj (actor.py StackedParamsModel.direct_target), bit-identical to vLLM's
per-name load_weights path (the fallback) and to the concatenation of the trainer's shards."""
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

pytestmark = pytest.mark.gpu


def _qwen(seed):
    from transformers import Qwen2Config, Qwen2ForCausalLM

    torch.manual_seed(seed)
    cfg = Qwen2Config(vocab_size=1000, hidden_size=896, intermediate_size=4864, num_hidden_layers=2,
                      num_attention_heads=14, num_key_value_heads=2, tie_word_embeddings=True)
    return Qwen2ForCausalLM(cfg).to(torch.bfloat16).cuda()


def test_bucketed_receive_unflattens_into_fused_rows():
    from pipelinerl_amd.actor import StandaloneWorker
    from pipelinerl_amd.weight_update import FlatLayout, HipFlatPacker, ParameterInfo

    trainer = _qwen(0)
    named = list(trainer.named_parameters())
    infos = [ParameterInfo(name=n, shape=list(p.shape), dtype=str(torch.bfloat16)) for n, p in named]
    layout = FlatLayout.from_infos(infos)
    flat = torch.empty(layout.total, dtype=torch.bfloat16, device="cuda")
    HipFlatPacker().flatten([p.detach() for _, p in named], layout.offsets, flat)

    direct = StandaloneWorker(_qwen(1), rank=0, device="cuda", layout="vllm")
    model = direct.model_runner.model
    assert direct._direct_targets(layout) is not None  # the HIP path, not the per-name fallback
    v0 = {n: p._version for n, p in model.params.items()}
    direct._apply_flat(flat, layout)
    torch.cuda.synchronize()
    assert all(model.params[n]._version > v0[n] for n in model.params)

    per_name = StandaloneWorker(_qwen(2), rank=0, device="cuda", layout="vllm")
    for name, shape, n, off in zip(layout.names, layout.shapes, layout.numels, layout.offsets):
        per_name._load_one(name, flat[off:off + n].view(shape))

    want = dict(named)
    for fname, p in model.params.items():
        assert torch.equal(p, per_name.model_runner.model.params[fname]), fname
    for i in range(2):
        pre = f"model.layers.{i}."
        assert torch.equal(model.params[pre + "self_attn.qkv_proj.weight"],
                           torch.cat([want[pre + f"self_attn.{x}_proj.weight"] for x in "qkv"]))
        assert torch.equal(model.params[pre + "self_attn.qkv_proj.bias"],
                           torch.cat([want[pre + f"self_attn.{x}_proj.bias"] for x in "qkv"]))
        assert torch.equal(model.params[pre + "mlp.gate_up_proj.weight"],
                           torch.cat([want[pre + "mlp.gate_proj.weight"], want[pre + "mlp.up_proj.weight"]]))
    for n in ("model.embed_tokens.weight", "model.norm.weight", "model.layers.1.mlp.down_proj.weight"):
        assert torch.equal(model.params[n], want[n])


@pytest.mark.parametrize("multi_step", [False, True], ids=["Worker", "MultiStepWorker"])
def test_v0_worker_unflattens_into_fused_rows(multi_step):
    """vLLM v0's worker classes (make_worker_class over stand-ins of Worker / MultiStepWorker,
    tests/test_actor_v0_cpu.py): the bucketed receive resolves the fused layout through
    direct_target on both runner kinds — the multi-step runner's model is its base runner's
    (vllm0.py:90-93) — and the one HIP unflatten pass equals the per-name load."""
    sys.path.insert(0, str(ROOT / "tests"))
    from test_actor_v0_cpu import MultiStepWorker, Worker

    from pipelinerl_amd.actor import make_worker_class
    from pipelinerl_amd.weight_update import FlatLayout, HipFlatPacker, ParameterInfo

    cls = make_worker_class(multi_step, MultiStepWorker if multi_step else Worker)
    trainer = _qwen(0)
    named = list(trainer.named_parameters())
    layout = FlatLayout.from_infos([ParameterInfo(name=n, shape=list(p.shape), dtype=str(torch.bfloat16))
                                    for n, p in named])
    flat = torch.empty(layout.total, dtype=torch.bfloat16, device="cuda")
    HipFlatPacker().flatten([p.detach() for _, p in named], layout.offsets, flat)
    w = cls(_qwen(1), device="cuda")
    assert (w.model_runner._base_model_runner.model if multi_step else w.model_runner.model) is w._inference_model()
    assert w._direct_targets(layout) is not None
    w._apply_flat(flat, layout)
    ref = cls(_qwen(2), device="cuda")
    for name, shape, n, off in zip(layout.names, layout.shapes, layout.numels, layout.offsets):
        ref._load_one(name, flat[off:off + n].view(shape))
    torch.cuda.synchronize()
    got, want = w._inference_model().params, ref._inference_model().params
    assert set(got) == set(want)
    for fname in got:
        assert torch.equal(got[fname], want[fname]), fname
