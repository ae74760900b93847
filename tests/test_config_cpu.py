"""The trainer entrypoint's config loader on the config the reference launcher saves.

The fixture ``golden/exp_config_math_grpo.yaml`` is what ``OmegaConf.save`` writes at
pipelinerl/launch.py:547 for ``math finetune=grpo`` (composed by golden/make_exp_config.py from
conf/base.yaml + conf/math.yaml + conf/finetune/{base,grpo}.yaml, interpolations unresolved).
OmegaConf semantics: ``${.x}`` = sibling, ``${..x}`` = the parent's child, ``${...x}`` one more
level up (conf/finetune/base.yaml:5, :96, :103).
"""

from __future__ import annotations

import pytest
import yaml

from conftest import GOLDEN
from pipelinerl_amd.config import load_config, resolve
from pipelinerl_amd.entrypoints import run_finetune
from pipelinerl_amd.finetune.rl import RLConfig

FIX = GOLDEN / "exp_config_math_grpo.yaml"


def test_composed_reference_config_resolves():
    raw = yaml.safe_load(FIX.read_text())
    cfg = load_config(GOLDEN, "exp_config_math_grpo")
    ft = cfg.finetune
    # ${..rl.kl_coef} inside finetune.rl -> finetune.rl.kl_coef (conf/finetune/base.yaml:96)
    assert ft.rl.final_kl_coef == raw["finetune"]["rl"]["kl_coef"] == 0.0
    # ${...llm.parameters.temperature} inside finetune.rl -> root llm.parameters.temperature (:103)
    assert ft.rl.temperature == raw["llm"]["parameters"]["temperature"] == 1.0
    # ${..model_path} inside finetune -> root model_path (:5)
    assert ft.config_name == raw["model_path"] == "Qwen/Qwen2.5-7B"
    assert ft.output_dir == "/tmp/exp/finetune"
    assert ft.seed == raw["seed"] == 42
    assert ft.pop_old_data is True and ft.max_lag is None
    # absolute interpolation at the root: attempts: ${finetune.attempts} (conf/base.yaml:106)
    assert cfg.attempts == ft.attempts == 8
    # the GRPO choice (conf/finetune/grpo.yaml) over finetune/base.yaml
    assert ft.rl.policy_loss == "ppo"
    assert ft.seq_length == 12000 and ft.gradient_clipping_threshold == 0.3
    # every rl key the reference config sets is accepted by RLConfig with the same value
    rl = RLConfig(**dict(ft.rl))
    for k, v in ft.rl.items():
        if hasattr(rl, k):
            assert getattr(rl, k) == v, k


def test_overrides_and_sibling_interpolation(tmp_path):
    cfg = load_config(GOLDEN, "exp_config_math_grpo",
                      ["+me.weight_update_group_init_method=tcp://127.0.0.1:9000",
                       "+me.weight_update_group_world_size=5", "finetune.rl.kl_coef=0.001",
                       "llm.parameters.temperature=0.7"])
    assert cfg.me.weight_update_group_world_size == 5
    assert cfg.me.weight_update_group_init_method == "tcp://127.0.0.1:9000"
    assert cfg.finetune.rl.final_kl_coef == 0.001  # the interpolation sees the override
    assert cfg.finetune.rl.temperature == 0.7
    r = resolve({"a": {"x": 3, "y": "${.x}", "z": "v${.x}w", "b": {"c": "${..x}", "d": "${...top}"}},
                 "top": "t"})
    assert r.a.y == 3 and r.a.z == "v3w" and r.a.b.c == 3 and r.a.b.d == "t"


def test_interpolation_above_root_raises():
    with pytest.raises(KeyError):
        resolve({"a": {"b": "${...x}"}, "x": 1})


def test_entrypoint_reads_reference_config(monkeypatch):
    seen = {}
    monkeypatch.setattr(run_finetune, "run_finetuning_loop", lambda cfg: seen.setdefault("cfg", cfg))
    rc = run_finetune.main(["--config-dir", str(GOLDEN), "--config-name", "exp_config_math_grpo",
                            "--local_rank=0", "+me.llm_urls=http://a:8080+http://b:8080"])
    assert rc == 0
    cfg = seen["cfg"]
    assert cfg.finetune.rl.final_kl_coef == 0.0 and cfg.me.llm_urls.split("+") == ["http://a:8080", "http://b:8080"]
