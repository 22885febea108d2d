"""`.roundtable/config.json` loading, validation and generation.

Parity: `src/utils/config.ts:13-86` (load + validate, same error messages) and
`src/commands/init.ts:138-220` (generated defaults). The schema is accepted
unchanged; unknown fields are tolerated.

MI355X extension: every ``adapter_config[<adapter id>]`` may carry an ``engine``
object that tells the local engine how to host that knight, and a top-level
``engine`` object holds defaults::

    "engine": {"default_model": "llama3-8b", "dtype": "bf16", "weights": "random:0",
               "kv_block_size": 32, "max_new_tokens": 512, "temperature": 0.7,
               "top_p": 0.95, "top_k": 0, "seed": 0, "stop_on_consensus": true},
    "adapter_config": {"claude-cli": {"command": "claude", "args": [],
                                      "engine": {"model": "llama3-8b", "gpus": [0], "tp": 1}}}

Vendor fields (``command``, ``args``, ``env_key``, vendor ``model`` names) are
ignored: no subprocess or HTTPS call is ever made.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional

from .errors import ConfigError
from .types import RoundtableConfig, dumps_js
from .utils.atomic import read_text

DEFAULT_CAPABILITIES = {
    "Claude": ["architecture", "refactoring", "logic", "debugging", "testing"],
    "Gemini": ["docs", "ui-ux", "summarization", "review", "planning"],
    "GPT": ["communication", "content", "explanation"],
}

ENGINE_DEFAULTS: Dict[str, Any] = {
    "default_model": "llama3-8b",
    "dtype": "bf16",
    "weights": "random:0",
    "kv_block_size": 32,
    "max_new_tokens": 512,
    "temperature": 0.7,
    "top_p": 0.95,
    "top_k": 0,
    "seed": 0,
    "stop_on_consensus": True,
    "ignore_eos": False,
    "kv_cache_fraction": 0.85,
}


def config_path(project_root: str) -> str:
    return os.path.join(project_root, ".roundtable", "config.json")


def load_config(project_root: str) -> RoundtableConfig:
    p = config_path(project_root)
    if not os.path.exists(p):
        raise ConfigError("No .roundtable/config.json found.", hint='Run "roundtable init" first.')
    try:
        raw = json.loads(read_text(p))
    except ValueError:
        raise ConfigError("Invalid config.json — could not parse JSON.",
                          hint="Check for syntax errors in .roundtable/config.json")
    validate_config(raw)
    return RoundtableConfig.from_dict(raw)


def _is_num(v: Any) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def validate_config(cfg: Dict[str, Any]) -> None:
    if not isinstance(cfg, dict):
        raise ConfigError("config.json must be a JSON object.")
    if not cfg.get("version"):
        raise ConfigError("config.json missing 'version' field.")
    knights = cfg.get("knights")
    if not isinstance(knights, list) or not knights:
        raise ConfigError("config.json must have at least one knight.")
    for k in knights:
        if not isinstance(k, dict) or not k.get("name") or not k.get("adapter"):
            raise ConfigError(f"Knight missing required fields (name, adapter): {json.dumps(k)}")
        if not isinstance(k.get("capabilities"), list):
            raise ConfigError(f'Knight "{k["name"]}" missing capabilities array.')
        if not _is_num(k.get("priority")):
            raise ConfigError(f'Knight "{k["name"]}" missing numeric priority.')
    rules = cfg.get("rules")
    if not rules:
        raise ConfigError("config.json missing 'rules' section.")
    if not _is_num(rules.get("max_rounds")) or rules["max_rounds"] < 1:
        raise ConfigError("rules.max_rounds must be a positive number.")
    ct = rules.get("consensus_threshold")
    if not _is_num(ct) or ct < 0 or ct > 10:
        raise ConfigError("rules.consensus_threshold must be between 0 and 10.")
    tpt = rules.get("timeout_per_turn_seconds")
    if not _is_num(tpt) or tpt < 1:
        raise ConfigError("rules.timeout_per_turn_seconds must be a positive number.")
    if rules.get("round_mode", "sequential") not in ("sequential", "parallel"):
        raise ConfigError("rules.round_mode must be 'sequential' or 'parallel'.")
    if rules.get("prompt_layout", "reference") not in ("reference", "append", "shared"):
        raise ConfigError("rules.prompt_layout must be 'reference', 'append' or 'shared'.")
    if rules.get("placeholder_semantics", "literal") not in ("literal", "reference"):
        raise ConfigError("rules.placeholder_semantics must be 'literal' or 'reference'.")
    if not cfg.get("adapter_config") and cfg.get("adapter_config") != {}:
        raise ConfigError("config.json missing 'adapter_config' section.")
    if cfg.get("adapter_config") is None:
        raise ConfigError("config.json missing 'adapter_config' section.")


def engine_settings(config: RoundtableConfig, adapter_id: str) -> Dict[str, Any]:
    """Effective engine settings for one adapter id: defaults <- config.engine <- adapter engine."""
    out = dict(ENGINE_DEFAULTS)
    top = config.raw.get("engine") if isinstance(config.raw, dict) else None
    if isinstance(top, dict):
        out.update(top)
    ac = config.adapter_config.get(adapter_id) or {}
    eng = ac.get("engine") if isinstance(ac, dict) else None
    if isinstance(eng, dict):
        out.update(eng)
    if "model" not in out or not out.get("model"):
        out["model"] = resolve_model_name(ac.get("model") if isinstance(ac, dict) else None,
                                          out["default_model"])
    return out


_MODEL_ALIASES = {
    "llama3-8b": ("llama-3-8b", "llama3-8b", "llama-3.1-8b", "meta-llama-3-8b"),
    "llama3-70b": ("llama-3-70b", "llama3-70b", "llama-3.1-70b", "meta-llama-3-70b"),
    "mistral-7b": ("mistral-7b", "mistral-7b-instruct"),
    "gpt2-small": ("gpt2", "gpt-2", "gpt2-small"),
    "tiny-llama": ("tiny-llama", "tiny"),
}


def resolve_model_name(name: Optional[str], default: str) -> str:
    """Map an ``adapter_config.model`` string onto an engine preset (vendor names -> default)."""
    if not name:
        return default
    low = str(name).lower()
    for preset, aliases in _MODEL_ALIASES.items():
        if any(a in low for a in aliases):
            return preset
    return default


def generate_config(project: str, language: str, knights: List[Dict[str, Any]],
                    engine: Optional[Dict[str, Any]] = None,
                    adapter_engine: Optional[Dict[str, Dict[str, Any]]] = None) -> Dict[str, Any]:
    """Build a config dict in the reference's shape (init.ts:138-220) + engine extensions.

    ``knights`` items: ``{"name", "adapter", "fallback"?, "capabilities"?}``.
    """
    out_knights = []
    for i, k in enumerate(knights, start=1):
        d = {"name": k["name"], "adapter": k["adapter"],
             "capabilities": k.get("capabilities") or DEFAULT_CAPABILITIES.get(k["name"], ["general"]),
             "priority": i}
        if k.get("fallback"):
            d["fallback"] = k["fallback"]
        out_knights.append(d)
    adapter_config: Dict[str, Any] = {
        "claude-cli": {"command": "claude", "args": ["-p", "{prompt}", "--print"]},
        "claude-api": {"model": "claude-sonnet-4-6", "env_key": "ANTHROPIC_API_KEY"},
        "gemini-cli": {"command": "gemini", "args": ["-p", "{prompt}"], "model": "gemini-2.5-pro"},
        "gemini-api": {"model": "gemini-2.5-flash", "env_key": "GEMINI_API_KEY"},
        "openai-cli": {"command": "codex", "args": ["exec", "{prompt}"]},
        "openai-api": {"model": "gpt-5.2", "env_key": "OPENAI_API_KEY"},
    }
    for aid, eng in (adapter_engine or {}).items():
        adapter_config.setdefault(aid, {})["engine"] = eng
    cfg = {
        "version": "1.0", "project": project, "language": language, "knights": out_knights,
        "rules": {"max_rounds": 5, "consensus_threshold": 9, "timeout_per_turn_seconds": 120,
                  "escalate_to_user_after": 3, "auto_execute": False,
                  "ignore": [".git", "node_modules", "dist", "build", ".next"],
                  "round_mode": "sequential", "prompt_layout": "reference"},
        "chronicle": ".roundtable/chronicle.md",
        "adapter_config": adapter_config,
    }
    if engine:
        cfg["engine"] = engine
    return cfg


def write_config(project_root: str, cfg: Dict[str, Any]) -> None:
    from .utils.atomic import atomic_write_text
    atomic_write_text(config_path(project_root), dumps_js(cfg))
