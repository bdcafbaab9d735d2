"""Configuration loading (reference ballbot_gym/core/config.py:1-196).

Same YAML conventions as the reference so its training configs load unchanged:
* load_config: yaml.safe_load, empty file -> {}, missing file -> FileNotFoundError;
* merge_configs: recursive dict merge, override wins;
* load_training_config: a training config names its env config with
  `env_config` (required, ValueError otherwise; "configs/..." resolves from the
  working directory, other relative paths from the training config's
  grand-parent directory); the env config is the base, the training config
  overrides it, and the env config's terrain/reward are copied under `problem`;
* get_component_config: "problem.<kind>" first, then top level; a bare string
  is the type; missing "type" -> default_type or ValueError.
"""
from __future__ import annotations

import copy
from pathlib import Path
from typing import Any, Dict, Optional

import yaml


def load_config(config_path: str) -> Dict[str, Any]:
    path = Path(config_path)
    if not path.exists():
        raise FileNotFoundError(f"Configuration file not found: {config_path}")
    with path.open("r") as f:
        data = yaml.safe_load(f)
    return data if data is not None else {}


def merge_configs(base: Dict[str, Any], override: Dict[str, Any]) -> Dict[str, Any]:
    out = dict(base)
    for k, v in override.items():
        out[k] = merge_configs(out[k], v) if isinstance(out.get(k), dict) and isinstance(v, dict) else v
    return out


def load_training_config(config_path: str) -> Dict[str, Any]:
    cfg = load_config(config_path)
    env_ref = cfg.get("env_config")
    if not env_ref:
        raise ValueError(
            "Training config must specify 'env_config' key pointing to an environment config.\n"
            "Example: env_config: 'configs/env/perlin_directional.yaml'\n"
            f"Config file: {config_path}")
    env_path = Path(env_ref)
    if not env_path.is_absolute():
        env_path = (Path.cwd() / env_ref) if str(env_ref).startswith("configs/") \
            else Path(config_path).parent.parent / env_ref
    env_cfg = load_config(str(env_path))
    merged = merge_configs(env_cfg, cfg)
    problem = merged.setdefault("problem", {})
    for kind in ("terrain", "reward"):
        if kind in env_cfg and kind not in problem:
            problem[kind] = env_cfg[kind]
    merged.pop("env_config", None)
    return merged


def get_component_config(config: Dict[str, Any], component_type: str,
                         default_type: Optional[str] = None) -> Dict[str, Any]:
    comp = (config.get("problem", {}) or {}).get(component_type, {})
    if not comp:
        comp = config.get(component_type, {})
    if isinstance(comp, str):
        return {"type": comp, "config": {}}
    if not comp and default_type:
        return {"type": default_type, "config": {}}
    if not isinstance(comp, dict) or "type" not in comp:
        if default_type:
            return {"type": default_type, "config": comp if isinstance(comp, dict) else {}}
        raise ValueError(f"Component config for '{component_type}' must have 'type' key or be a string, "
                         f"got: {comp}")
    comp = copy.copy(comp)
    comp.setdefault("config", {})
    return comp
