"""Experiment config for the trainer entrypoint (replaces Hydra/OmegaConf, which the trainer
only uses to read a frozen YAML: launch.py writes exp/conf/exp_config.yaml and starts
``run_finetune.py --config-dir exp/conf --config-name exp_config +me.k=v ...``).

Supports what that file needs: nested mappings, ``${a.b.c}`` absolute and ``${.x}`` / ``${..x}``
relative interpolation (OmegaConf semantics: ``${.x}`` is a sibling of the key, in the node that
holds it; each further leading dot goes one level up, so ``finetune.rl.final_kl_coef:
${..rl.kl_coef}`` reads ``finetune.rl.kl_coef``, conf/finetune/base.yaml:96), and Hydra-style
``key=value`` / ``+key=value`` overrides.
"""

from __future__ import annotations

import re
from pathlib import Path
from typing import Any

import yaml

_INTERP = re.compile(r"\$\{([^}]+)\}")


class Cfg(dict):
    """dict with attribute access (cfg.finetune.rl.kl_coef) and dict semantics ("x" in cfg)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x: Any) -> Any:
        if isinstance(x, Cfg):
            return x
        if isinstance(x, dict):
            return Cfg({k: Cfg.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [Cfg.wrap(v) for v in x]
        return x

    def to_dict(self) -> dict:
        def un(x):
            if isinstance(x, dict):
                return {k: un(v) for k, v in x.items()}
            if isinstance(x, list):
                return [un(v) for v in x]
            return x
        return un(self)


def _lookup(root: dict, path: list[str]) -> Any:
    node: Any = root
    for p in path:
        if isinstance(node, list):
            node = node[int(p)]
        else:
            node = node[p]
    return node


def _resolve_value(root: dict, here: list[str], value: Any, depth: int = 0) -> Any:
    if depth > 32:
        raise ValueError("interpolation cycle")
    if not isinstance(value, str) or "${" not in value:
        return value

    def target(expr: str) -> Any:
        expr = expr.strip()
        if expr.startswith("."):
            up = len(expr) - len(expr.lstrip(".")) - 1  # one dot = the containing node itself
            if up > len(here):
                raise KeyError(f"interpolation ${{{expr}}} at {'.'.join(here) or '<root>'} goes above the root")
            base = here[:len(here) - up]
            path = base + [p for p in expr.lstrip(".").split(".") if p]
        else:
            path = expr.split(".")
        v = _lookup(root, path)
        return _resolve_value(root, path[:-1], v, depth + 1)

    m = _INTERP.fullmatch(value.strip())
    if m:
        return target(m.group(1))
    return _INTERP.sub(lambda mm: str(target(mm.group(1))), value)


def resolve(cfg: dict) -> Cfg:
    def walk(node: Any, path: list[str]) -> Any:
        if isinstance(node, dict):
            return {k: walk(v, path + [k]) for k, v in node.items()}
        if isinstance(node, list):
            return [walk(v, path + [str(i)]) for i, v in enumerate(node)]
        return _resolve_value(cfg, path[:-1], node)

    return Cfg.wrap(walk(cfg, []))


def _parse_scalar(s: str) -> Any:
    return yaml.safe_load(s) if s != "" else ""


def apply_overrides(cfg: dict, overrides: list[str]) -> dict:
    for ov in overrides:
        key, _, val = ov.lstrip("+~").partition("=")
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = _parse_scalar(val)
    return cfg


def load_config(config_dir: str | Path, config_name: str, overrides: list[str] | None = None) -> Cfg:
    path = Path(config_dir) / (config_name if config_name.endswith((".yaml", ".yml")) else config_name + ".yaml")
    with open(path) as f:
        raw = yaml.safe_load(f) or {}
    raw.pop("defaults", None)
    raw.pop("hydra", None)
    return resolve(apply_overrides(raw, overrides or []))
