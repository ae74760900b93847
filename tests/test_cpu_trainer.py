"""The CPU trainer-step baseline (oracle/cpu_trainer.py, bench.py cpu_baseline.trainer_step):
driving the model backward with the oracle's d loss / d logits gives the same parameter gradients
as autograd through a torch restatement of the loss (tests/cpu_rl_step.py), and the timed step
runs end to end on a 2-layer 0.5B-shaped model."""

import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]


def test_oracle_dlogits_drive_the_same_gradients():
    sys.path[:0] = [str(ROOT / "tests")]
    from cpu_rl_step import cpu_rl_step
    from transformers import Qwen2Config, Qwen2ForCausalLM

    from oracle import cpu_trainer, grpo_oracle
    from pipelinerl_amd.finetune.rl import RLConfig
    from pipelinerl_amd.finetune.types import PipelineBatchEncoding

    cfg = Qwen2Config(vocab_size=96, hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, max_position_embeddings=128, tie_word_embeddings=True)
    torch.manual_seed(0)
    m = Qwen2ForCausalLM(cfg).float()
    b = cpu_trainer.micro_batch(3, 20, 5, 96)
    rl = dict(cpu_trainer.GRPO, batch_size=3)
    # autograd through the torch loss
    enc = PipelineBatchEncoding(**{k: torch.as_tensor(v) for k, v in b.items()
                                   if k not in ("is_packed", "model_version", "seq_boundaries")},
                                is_packed=False, model_version=0)
    loss_t, _ = cpu_rl_step(m, enc, 0, 100, RLConfig(**rl))
    loss_t.backward()
    ga = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    # oracle dlogits into the model backward
    ids = torch.from_numpy(b["input_ids"])
    out = m(input_ids=ids, attention_mask=torch.ones_like(ids), use_cache=False)
    o = grpo_oracle.rl_step_oracle(out.logits.detach().numpy(), b, rl, 0, 100)
    assert abs(o["loss"] - float(loss_t)) < 1e-5
    out.logits.backward(torch.from_numpy(o["dlogits"]).float())
    for n, p in m.named_parameters():
        err = float((p.grad - ga[n]).abs().max())
        assert err <= 1e-4 * float(ga[n].abs().max()) + 1e-7, (n, err)


def test_cpu_trainer_step_runs():
    from oracle import cpu_trainer

    r = cpu_trainer.cpu_trainer_step(n_seq=2, seq=64, prompt=16, threads=4, layers=2)
    assert r["value"] > 0 and r["kind"] == "port" and np.isfinite(r["loss"]) and r["cores"] == 4
