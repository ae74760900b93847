"""Compose the experiment config the reference launcher saves (exp/conf/exp_config.yaml) from the
reference's own Hydra config tree, WITHOUT resolving interpolations — what
``OmegaConf.save(cfg, config_dir / "exp_config.yaml")`` writes (pipelinerl/launch.py:547), so
the trainer entrypoint has to resolve ``${..x}`` / ``${...x}`` itself.

Run in the build container only (reads /root/reference/conf; the output is a data fixture):

    python tests/golden/make_exp_config.py

Composition follows Hydra's defaults lists for ``--config-name math finetune=grpo
output_dir=/tmp/exp model_path=Qwen/Qwen2.5-7B``:
  math.yaml       defaults [base, _self_]
  base.yaml       defaults [finetune: actor_critic -> overridden to grpo, rewards: pure_success,
                            streams: files, _self_]
  finetune/grpo.yaml  defaults [base, _self_]  (placed under the ``finetune`` key)
Later entries deep-merge over earlier ones; the ``hydra`` node is dropped as Hydra does.
"""

from __future__ import annotations

import sys
from pathlib import Path

import yaml

CONF = Path("/root/reference/conf")
OUT = Path(__file__).resolve().parent / "exp_config_math_grpo.yaml"


def merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in b.items():
        out[k] = merge(out[k], v) if isinstance(out.get(k), dict) and isinstance(v, dict) else v
    return out


def load(rel: str) -> tuple[list, dict]:
    d = yaml.safe_load((CONF / rel).read_text()) or {}
    return d.pop("defaults", []), d


def compose_group(group: str, name: str) -> dict:
    defaults, body = load(f"{group}/{name}.yaml")
    acc: dict = {}
    for item in defaults:
        if item == "_self_":
            acc = merge(acc, body)
        else:
            acc = merge(acc, compose_group(group, item))
    if "_self_" not in defaults:
        acc = merge(acc, body)
    return acc


def compose_primary(name: str, group_choices: dict) -> dict:
    defaults, body = load(f"{name}.yaml")
    acc: dict = {}
    for item in defaults:
        if item == "_self_":
            acc = merge(acc, body)
        elif isinstance(item, dict):
            (group, choice), = item.items()
            acc = merge(acc, {group: compose_group(group, group_choices.get(group, choice))})
        else:
            acc = merge(acc, compose_primary(item, group_choices))
    return acc


def main() -> int:
    if not CONF.exists():
        print("reference config tree not present", file=sys.stderr)
        return 1
    cfg = compose_primary("math", {"finetune": "grpo"})
    cfg.pop("hydra", None)
    cfg = merge(cfg, {"output_dir": "/tmp/exp", "model_path": "Qwen/Qwen2.5-7B"})
    OUT.write_text(yaml.safe_dump(cfg, sort_keys=False))
    print(f"wrote {OUT}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
