"""Gradient-checkpointing plan (finetune/recompute.py): the reference config sets
gradient_checkpointing (conf/finetune/base.yaml:44-48); the build skips the recompute when the
micro-batch's activations fit the device.  Models are built on the meta device at the published
Qwen2.5 shapes (no memory), the device size is given."""

import types

import pytest
import torch

GB = 10 ** 9


def _meta_model(name):
    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd.trainer_probe import QWEN

    with torch.device("meta"):
        return AutoModelForCausalLM.from_config(Qwen2Config(**QWEN[name]), dtype=torch.bfloat16)


def _args(**kw):
    d = dict(gradient_checkpointing=True, seq_length=12000)
    d.update(kw)

    class A(dict):
        def __getattr__(self, k):
            return self[k]

    return A(d)


@pytest.fixture(scope="module")
def m7b():
    return _meta_model("7b")


def test_7b_c3_fits_mi355x(m7b):
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    from pipelinerl_amd.finetune.recompute import ModelStateTooLarge

    p = plan_gradient_checkpointing(_args(), m7b, torch.device("cuda"), device_bytes=288 * GB)
    assert not p.checkpoint, p.as_dict()
    # 7.6 B parameters x (bf16 weight + grad, fp32 master + 2 moments: the reference default's
    # optimizer state); activations of 12 000 tokens over 28 layers
    assert 121 * GB < p.state_bytes < 123 * GB
    assert 60 * GB < p.activation_bytes < 75 * GB
    # pure bf16 state (finetune.master_weights=false): 8 B per parameter
    pb = plan_gradient_checkpointing(_args(master_weights=False), m7b, torch.device("cuda"), device_bytes=288 * GB)
    assert 60 * GB < pb.state_bytes < 62 * GB
    # the same micro-batch on a 100 GB card recomputes (bf16 state), or cannot hold the fp32 state at
    # all; an 80 GB card cannot hold even the bf16 state beside one recomputed layer
    assert plan_gradient_checkpointing(_args(master_weights=False), m7b, torch.device("cuda"),
                                       device_bytes=100 * GB).checkpoint
    for dev_gb, master in ((100, True), (80, False)):
        with pytest.raises(ModelStateTooLarge, match="shard the model"):
            plan_gradient_checkpointing(_args(master_weights=master), m7b, torch.device("cuda"),
                                        device_bytes=dev_gb * GB)


def test_policy_and_reference_fallbacks(m7b):
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    cuda = torch.device("cuda")
    assert plan_gradient_checkpointing(_args(gradient_checkpointing_policy="always"), m7b, cuda,
                                       device_bytes=288 * GB).checkpoint
    assert not plan_gradient_checkpointing(_args(gradient_checkpointing=False), m7b, cuda,
                                           device_bytes=288 * GB).checkpoint
    # off the GPU, without a seq_length or without a decoder config: as the reference does
    assert plan_gradient_checkpointing(_args(), m7b, torch.device("cpu")).checkpoint
    assert plan_gradient_checkpointing(_args(seq_length=None), m7b, cuda, device_bytes=288 * GB).checkpoint
    assert plan_gradient_checkpointing(_args(), types.SimpleNamespace(parameters=lambda: iter(())), cuda,
                                       device_bytes=288 * GB).checkpoint
    with pytest.raises(ValueError):
        plan_gradient_checkpointing(_args(gradient_checkpointing_policy="never"), m7b, cuda, device_bytes=288 * GB)


def test_32b_needs_sharding():
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    m = _meta_model("32b")
    args = _args(seq_length=4096)
    cuda = torch.device("cuda")
    from pipelinerl_amd.finetune.recompute import ModelStateTooLarge

    # unsharded, the model state (524 GB with fp32 masters; 262 GB in pure bf16, which leaves no room
    # for even one layer's activations) does not fit: a named error pointing at FSDP, not a
    # recompute plan that would still run out of memory
    for master in (True, False):
        with pytest.raises(ModelStateTooLarge, match="use_fsdp"):
            plan_gradient_checkpointing(_args(seq_length=4096, master_weights=master), m, cuda, shard_world=1,
                                        device_bytes=288 * GB)
    p = plan_gradient_checkpointing(args, m, cuda, shard_world=4, device_bytes=288 * GB)
    assert not p.checkpoint, p.as_dict()
    assert 130 * GB < p.state_bytes < 132 * GB  # 524 GB / 4


def test_label_row_chunk_sizes_the_logits(m7b):
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    cuda = torch.device("cuda")
    a = plan_gradient_checkpointing(_args(), m7b, cuda, device_bytes=288 * GB)
    b = plan_gradient_checkpointing(_args(rl={"lm_head_chunk_rows": 4096}), m7b, cuda, device_bytes=288 * GB)
    assert a.logits_bytes == 12000 * 152064 * 2 and b.logits_bytes == 4096 * 152064 * 2


def test_build_buffers_are_counted(m7b, monkeypatch):
    """The fused gate/up weight cache (2 I H per layer, when fused at this micro-batch size and not
    sharded) and the lm_head dW staging ([V, H]: bf16 for one chunk, fp32 over several) enter the
    estimate: at the 7B shapes 7.6 GB + 1.1 GB; at 32B under FSDP, FSDP's unsharded
    working set instead (the larger of the backward's start — logits' gradient, root unit gathered,
    the lm_head's unsharded gradient, 2 decoder layers — and the root's reduce-scatter, 3 x the root
    unit: embedding, lm_head, norm)."""
    from pipelinerl_amd.finetune import model_ops
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    cuda = torch.device("cuda")
    monkeypatch.setattr(model_ops, "_FUSED_GATE_UP", True)
    nf = dict(flat_parameters=False)  # the cache exists only without flat parameter storage
    p = plan_gradient_checkpointing(_args(**nf), m7b, cuda, device_bytes=288 * GB)
    cache = 2 * 18944 * 3584 * 28 * 2
    assert p.buffer_bytes == cache + 152064 * 3584 * 2, p.as_dict()
    # flat parameters (the loop's default): the fused weight is a view, no cache
    assert plan_gradient_checkpointing(_args(), m7b, cuda, device_bytes=288 * GB).buffer_bytes == 152064 * 3584 * 2
    # several lm_head chunks: an fp32 accumulator
    p2 = plan_gradient_checkpointing(_args(rl={"lm_head_chunk_rows": 4096}, **nf), m7b, cuda, device_bytes=288 * GB)
    assert p2.buffer_bytes == cache + 152064 * 3584 * 4
    # above the fused size (12 288 tokens) the cache is not built
    p3 = plan_gradient_checkpointing(_args(seq_length=16384, **nf), m7b, cuda, device_bytes=288 * GB)
    assert p3.buffer_bytes == 152064 * 3584 * 2
    monkeypatch.setattr(model_ops, "_FUSED_GATE_UP", False)
    assert plan_gradient_checkpointing(_args(**nf), m7b, cuda, device_bytes=288 * GB).buffer_bytes == \
        152064 * 3584 * 2
    # a device the estimate barely fits without the buffers: with them, recompute
    monkeypatch.setattr(model_ops, "_FUSED_GATE_UP", True)
    base = p.state_bytes + p.activation_bytes + p.logits_bytes
    dev = int((base + (4 << 30) + cache // 2) / 0.95)
    assert plan_gradient_checkpointing(_args(**nf), m7b, cuda, device_bytes=dev).checkpoint
    # 32B under FSDP 4: no fused cache (off under sharding), FSDP's transients
    m32 = _meta_model("32b")
    p32 = plan_gradient_checkpointing(_args(seq_length=4096), m32, cuda, shard_world=4, device_bytes=288 * GB)
    root = (2 * 152064 * 5120 + 5120) * 2
    layer = (2 * 5120 * 5120 + 2 * 1024 * 5120 + 3 * 27648 * 5120 + 5120 + 2 * 1024 + 2 * 5120) * 2
    head = 152064 * 5120 * 2
    start = root + head + 2 * layer  # beyond the activations (the label-row head: dlogits in place)
    assert p32.buffer_bytes == max(start, 3 * root - p32.activation_bytes) and not p32.checkpoint, p32.as_dict()
    # the full-logits loss head (rl.fused_lm_head false) also holds the logits' gradient
    pf = plan_gradient_checkpointing(_args(seq_length=4096, rl={"fused_lm_head": False}), m32, cuda, shard_world=4,
                                     device_bytes=288 * GB)
    assert pf.buffer_bytes == max(pf.logits_bytes + start, 3 * root - pf.activation_bytes), pf.as_dict()


def test_plan_counts_the_allocator_rounding(m7b, monkeypatch):
    """Under the trainer loop's size rounding (devalloc.py) each term of the plan is sized with the
    allocator's own rounding at the micro-batch's largest shapes: a device between the unrounded
    and the rounded need recomputes only when the rounding is in force; the 32B FSDP plan at 8
    ranks (C5) still keeps its activations (a flat 1.25 allowance flipped it to recomputing)."""
    from pipelinerl_amd import devalloc
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    for k in devalloc.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    cuda = torch.device("cuda")
    monkeypatch.setattr(devalloc, "_applied", None)
    raw = plan_gradient_checkpointing(_args(), m7b, cuda, device_bytes=288 * GB).need_bytes
    monkeypatch.setattr(devalloc, "_applied", devalloc.DEFAULT_SETTINGS)
    rounded = plan_gradient_checkpointing(_args(), m7b, cuda, device_bytes=288 * GB).need_bytes
    assert raw < rounded < raw * 1.1, (raw, rounded)
    from pipelinerl_amd.finetune.recompute import HEADROOM_BYTES, HEADROOM_FRAC

    # the terms without the headroom (5 % of the device + 4 GiB), then a device between the two
    core = [n - int(HEADROOM_FRAC * 288 * GB) - HEADROOM_BYTES for n in (raw, rounded)]
    dev = int((sum(core) / 2 + HEADROOM_BYTES) / (1 - HEADROOM_FRAC))
    assert plan_gradient_checkpointing(_args(), m7b, cuda, device_bytes=dev).checkpoint
    monkeypatch.setattr(devalloc, "_applied", None)
    assert not plan_gradient_checkpointing(_args(), m7b, cuda, device_bytes=dev).checkpoint
    monkeypatch.setattr(devalloc, "_applied", devalloc.DEFAULT_SETTINGS)
    m32 = _meta_model("32b")
    p = plan_gradient_checkpointing(_args(master_weights=False), m32, cuda, shard_world=8, device_bytes=288 * 2 ** 30)
    assert not p.checkpoint, p.as_dict()
    # with fp32 masters (65.5 GB of state per rank instead of 32.8) a few layers recompute
    pm = plan_gradient_checkpointing(_args(), m32, cuda, shard_world=8, device_bytes=288 * 2 ** 30)
    assert pm.checkpoint and 48 <= pm.keep_layers < 64, pm.as_dict()


def test_round_size_follows_the_allocator():
    """devalloc.round_size against PyTorch's rule (the GPU test checks two of these on the device)."""
    from pipelinerl_amd import devalloc

    S = devalloc.DEFAULT_SETTINGS
    assert devalloc.division_table(S) == [16] * 9 + [4] * 7
    assert devalloc.division_table("roundup_power2_divisions:8") == [8] * 16
    assert devalloc.division_table("max_split_size_mb:64") == [0] * 16
    assert devalloc.round_size(int(1.1 * 2 ** 30), S) == 5 * 2 ** 28  # 4 divisions above 512 MiB
    assert devalloc.round_size(300 * 10 ** 6, S) == 288 << 20  # 16 below
    assert devalloc.round_size(2 ** 27, S) == 2 ** 27  # powers of two are kept
    assert devalloc.round_size(1000, S) == 1024 and devalloc.round_size(100, S) == 512
    assert devalloc.round_size(300 * 10 ** 6, "") == -(-300 * 10 ** 6 // 512) * 512  # no rounding configured


def test_partial_recompute_keeps_the_layers_that_fit(monkeypatch):
    """C5 on 4 trainer ranks (32B, 12 000 tokens) does not fit whole: instead of recomputing all 64
    layers the plan keeps the activations of the largest K that fits — need(K) <= device <
    need(K + 1) — and finetune.gradient_checkpointing_keep_layers sets K directly."""
    from pipelinerl_amd import devalloc
    from pipelinerl_amd.finetune.recompute import plan_gradient_checkpointing

    for k in devalloc.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(devalloc, "_applied", devalloc.DEFAULT_SETTINGS)
    m32 = _meta_model("32b")
    cuda, dev = torch.device("cuda"), 288 * 2 ** 30
    p = plan_gradient_checkpointing(_args(), m32, cuda, shard_world=4, device_bytes=dev)
    assert p.checkpoint and 0 < p.keep_layers < 64, p.as_dict()
    assert p.need_bytes <= dev
    nxt = plan_gradient_checkpointing(_args(gradient_checkpointing_keep_layers=p.keep_layers + 1), m32, cuda,
                                      shard_world=4, device_bytes=dev)
    assert nxt.need_bytes > dev and nxt.keep_layers == p.keep_layers + 1
    # fewer kept layers need less; keeping all 64 is the no-recompute plan
    lo = plan_gradient_checkpointing(_args(gradient_checkpointing_keep_layers=0), m32, cuda, shard_world=4,
                                     device_bytes=dev)
    # (before the spare memory goes to FSDP layers kept gathered, plan_fsdp_gathering)
    assert lo.checkpoint and lo.keep_layers == 0 and lo.need_bytes - lo.gathered_bytes < p.need_bytes - p.gathered_bytes
    allk = plan_gradient_checkpointing(_args(gradient_checkpointing_keep_layers=64), m32, cuda, shard_world=4,
                                       device_bytes=dev)
    assert not allk.checkpoint
    # "always" is the reference's behaviour: every layer recomputes
    assert plan_gradient_checkpointing(_args(gradient_checkpointing_policy="always"), m32, cuda, shard_world=4,
                                       device_bytes=dev).keep_layers == 0


def test_keep_activations_flags_the_last_layers_and_gradients_are_unchanged():
    """checkpoints.keep_activations after HF's gradient_checkpointing_enable: the last K decoder
    layers stop recomputing; the gradients of a tiny fp32 Qwen2 on CPU are bit-identical for
    every K (the recomputed forward is the same computation)."""
    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd.finetune.checkpoints import keep_activations

    cfg = Qwen2Config(vocab_size=64, hidden_size=32, intermediate_size=64, num_hidden_layers=4,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
    ids = torch.randint(0, 64, (1, 24), generator=torch.Generator().manual_seed(0))
    grads = {}
    for keep in (None, 0, 2, 4):
        torch.manual_seed(0)
        m = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32)
        m.train()
        if keep is not None:
            m.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
            assert keep_activations(m, keep) == keep
            flags = [layer.gradient_checkpointing for layer in m.model.layers]
            assert flags == [True] * (4 - keep) + [False] * keep
        m(input_ids=ids, labels=ids).loss.backward()
        grads[keep] = {n: p.grad.clone() for n, p in m.named_parameters()}
    for keep in (0, 2, 4):
        for n, g in grads[None].items():
            assert torch.equal(g, grads[keep][n]), (keep, n)


def test_fsdp_gathered_layers_spend_the_spare_memory(monkeypatch):
    """plan_fsdp_gathering: under FSDP the spare device memory after the recompute plan keeps the
    last R decoder layers' unsharded parameters from forward to backward (R = spare // a layer's
    rounded unsharded bytes); need_bytes grows by them and stays within the device; the explicit
    int overrides, 0 turns it off; unsharded (shard_world 1) or unsized plans keep FSDP's default."""
    from pipelinerl_amd import devalloc
    from pipelinerl_amd.finetune.recompute import gathered_layer_bytes, plan_gradient_checkpointing

    for k in devalloc.ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(devalloc, "_applied", devalloc.DEFAULT_SETTINGS)
    m32 = _meta_model("32b")
    cuda, dev = torch.device("cuda"), 288 * 2 ** 30
    per = gathered_layer_bytes(m32)
    raw = (2 * 5120 * 5120 + 2 * 1024 * 5120 + 3 * 27648 * 5120 + 5120 + 2 * 1024 + 2 * 5120) * 2
    assert raw <= per <= 1.1 * raw
    # C5 on 8 ranks at 4 096 tokens: no recompute, the spare holds every layer
    p8 = plan_gradient_checkpointing(_args(seq_length=4096), m32, cuda, shard_world=8, device_bytes=dev)
    base = plan_gradient_checkpointing(_args(seq_length=4096, fsdp_keep_gathered_layers=0), m32, cuda,
                                       shard_world=8, device_bytes=dev)
    assert not p8.checkpoint and base.gathered_layers == 0
    assert p8.gathered_layers == min(64, (dev - base.need_bytes) // per) > 0, p8.as_dict()
    assert p8.need_bytes == base.need_bytes + p8.gathered_layers * per <= dev
    # C5 on 4 ranks at 12 000 tokens (partial recompute): what is left after the kept activations
    p4 = plan_gradient_checkpointing(_args(), m32, cuda, shard_world=4, device_bytes=dev)
    assert p4.checkpoint and 0 <= p4.gathered_layers <= (dev - (p4.need_bytes - p4.gathered_bytes)) // per
    assert p4.need_bytes <= dev
    # a tighter device gathers fewer: as many as fit, not one more
    tdev = base.need_bytes + 3 * per + per // 2
    tight = plan_gradient_checkpointing(_args(seq_length=4096), m32, cuda, shard_world=8, device_bytes=tdev)
    assert 0 < tight.gathered_layers < p8.gathered_layers, tight.as_dict()
    assert tight.need_bytes <= tdev < tight.need_bytes + per
    # explicit R; unsharded; unsized (policy always); invalid values
    assert plan_gradient_checkpointing(_args(seq_length=4096, fsdp_keep_gathered_layers=5), m32, cuda,
                                       shard_world=8, device_bytes=dev).gathered_layers == 5
    assert plan_gradient_checkpointing(_args(seq_length=4096), m32, cuda, shard_world=1,
                                       device_bytes=4 * dev).gathered_layers == 0
    assert plan_gradient_checkpointing(_args(gradient_checkpointing_policy="always"), m32, cuda, shard_world=8,
                                       device_bytes=dev).gathered_layers == 0
    for bad in (-1, "all", True):
        with pytest.raises(ValueError):
            plan_gradient_checkpointing(_args(fsdp_keep_gathered_layers=bad), m32, cuda, shard_world=8,
                                        device_bytes=dev)
