"""Local model discovery: find HF-format checkpoints on this machine and map them to engine presets.

The reference discovers *running model servers* (`src/utils/local-detect.ts:103-134`: probe
LM Studio / Ollama ports, fall back to ``ollama list``) and seats each chat model as a
``local-llm-<slug>`` knight (`src/commands/init.ts:361-373`). Here the engine itself hosts
knights, so discovery looks for *weights*: directories holding ``config.json`` plus
``*.safetensors`` under

* ``$ROUNDTABLE_MODELS_DIR`` (``os.pathsep``-separated),
* ``./models`` of the project,
* the Hugging Face hub cache (``$HF_HOME``/``~/.cache/huggingface/hub/models--*/snapshots/*``).

Each hit is read (JSON only — nothing from a checkpoint is executed) and matched to a preset
(Llama-3-8B/70B, Mistral-7B, Qwen2.5-7B/0.5B, GPT-2) or described as a preset plus shape overrides; embedding /
reranker / speech models are skipped, as the reference's ``isNonChatModel`` does.
Running servers are still supported from the other side: ``roundtable serve`` speaks the
LM Studio / Ollama dialects.
"""
from __future__ import annotations

import glob
import json
import math
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional

from ..models.config import PRESETS

NON_CHAT = re.compile(r"(^|[^a-z])(embed|embedding|tts|whisper|rerank|reranker|clip)([^a-z]|$)", re.I)


@dataclass
class LocalModel:
    name: str                 # display name, e.g. "Meta Llama 3 8B Instruct"
    model_id: str             # directory-derived id, e.g. "meta-llama/Meta-Llama-3-8B-Instruct"
    path: str                 # checkpoint directory (engine ``weights`` spec)
    preset: Optional[str]     # matching engine preset, or the closest architecture preset
    overrides: Dict[str, Any] = field(default_factory=dict)   # ModelConfig fields that differ
    source: str = "checkpoint"

    def adapter_slug(self) -> str:
        return re.sub(r"[^a-z0-9]+", "-", self.model_id.split("/")[-1].lower()).strip("-")


def prettify_model_name(model_id: str) -> str:
    """``"meta-llama/Meta-Llama-3-8B-instruct"`` -> ``"Meta Llama 3 8B Instruct"``."""
    raw = model_id.rsplit("/", 1)[-1]
    words = [w for w in re.split(r"[-_\s]+", raw) if w]
    out = []
    for w in words:
        if re.fullmatch(r"\d+(\.\d+)?[bBmM]", w):
            out.append(w[:-1] + w[-1].upper())
        else:
            out.append(w[:1].upper() + w[1:])
    return " ".join(out)


def is_non_chat_model(model_id: str) -> bool:
    return bool(NON_CHAT.search(model_id))


def _rope_scaling(hf: Dict[str, Any]):
    """config.json ``rope_scaling`` -> ModelConfig.rope_scaling; False when the type is unknown
    (the checkpoint is then not offered: a silently different RoPE would be wrong text)."""
    # transformers >= 5 writes "rope_parameters" (rope_theta inside), older files "rope_scaling"
    rs = hf.get("rope_scaling") or hf.get("rope_parameters")
    if not isinstance(rs, dict):
        return None
    kind = str(rs.get("rope_type", rs.get("type", "default"))).lower()
    orig = int(rs.get("original_max_position_embeddings") or hf.get("max_position_embeddings", 8192))
    if kind == "default":
        return None
    if kind == "linear":
        return ("linear", float(rs["factor"]))
    if kind == "llama3":
        return ("llama3", float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)),
                float(rs.get("high_freq_factor", 4.0)), orig)
    if kind == "yarn":
        factor = float(rs.get("factor") or hf.get("max_position_embeddings", orig) / orig)

        def mscale(scale, m=1.0):
            return 1.0 if scale <= 1 else 0.1 * m * math.log(scale) + 1.0
        att = rs.get("attention_factor")
        if att is None:
            att = (mscale(factor, rs["mscale"]) / mscale(factor, rs["mscale_all_dim"])
                   if rs.get("mscale") and rs.get("mscale_all_dim") else mscale(factor))
        return ("yarn", factor, orig, float(rs.get("beta_fast") or 32.0), float(rs.get("beta_slow") or 1.0), float(att))
    return False


def _rope_theta(hf: Dict[str, Any], default: float = 10000.0) -> float:
    rp = hf.get("rope_parameters") if isinstance(hf.get("rope_parameters"), dict) else {}
    return float(hf.get("rope_theta") or rp.get("rope_theta") or default)


def _shape_from_hf(hf: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    mt = str(hf.get("model_type", "")).lower()
    if mt in ("llama", "mistral", "qwen2"):
        if hf.get("attention_bias") or hf.get("mlp_bias"):
            return None   # biased o / MLP projections (Llama variants): not in the engine's layer
        scaling = _rope_scaling(hf)
        if scaling is False:
            return None   # a RoPE scaling the engine does not implement
        h = int(hf["hidden_size"])
        nh = int(hf["num_attention_heads"])
        return {"arch": "llama", "n_layers": int(hf["num_hidden_layers"]), "hidden": h, "n_heads": nh,
                "n_kv_heads": int(hf.get("num_key_value_heads", nh)), "head_dim": int(hf.get("head_dim", h // nh)),
                "ffn": int(hf["intermediate_size"]), "vocab": int(hf["vocab_size"]),
                "max_pos": int(hf.get("max_position_embeddings", 8192)),
                "rope_theta": _rope_theta(hf), "norm_eps": float(hf.get("rms_norm_eps", 1e-5)),
                "tie_embeddings": bool(hf.get("tie_word_embeddings", False)),
                "qkv_bias": mt == "qwen2", "rope_scaling": scaling}
    if mt == "gpt2":
        h = int(hf["n_embd"])
        nh = int(hf["n_head"])
        return {"arch": "gpt2", "n_layers": int(hf["n_layer"]), "hidden": h, "n_heads": nh, "n_kv_heads": nh,
                "head_dim": h // nh, "ffn": int(hf.get("n_inner") or 4 * h), "vocab": int(hf["vocab_size"]),
                "max_pos": int(hf.get("n_positions", 1024)), "rope_theta": 0.0,
                "norm_eps": float(hf.get("layer_norm_epsilon", 1e-5)), "tie_embeddings": True}
    return None


def match_preset(shape: Dict[str, Any]) -> (Optional[str], Dict[str, Any]):
    """Preset with the same architecture and fewest differing fields, plus those differences."""
    best, best_diff = None, None
    for name, cfg in PRESETS.items():
        if cfg.arch != shape["arch"] or name.startswith("tiny"):
            continue
        diff = {k: v for k, v in shape.items() if k != "arch" and getattr(cfg, k) != v}
        if best_diff is None or len(diff) < len(best_diff):
            best, best_diff = name, diff
    return best, (best_diff or {})


def checkpoint_model(path: str) -> Optional[tuple]:
    """(engine preset, ModelConfig overrides) for an HF checkpoint directory, from its
    ``config.json`` alone; None if it is not a recognised Llama / Mistral / Qwen2 / GPT-2 checkpoint."""
    try:
        with open(os.path.join(path, "config.json"), encoding="utf-8") as f:
            shape = _shape_from_hf(json.load(f))
    except (OSError, ValueError, KeyError, TypeError):
        return None
    if shape is None:
        return None
    preset, diff = match_preset(shape)
    return (preset, diff) if preset else None


def resolve_model(model: str, weights: str, overrides: Optional[Dict[str, Any]] = None) -> tuple:
    """(preset, overrides) to build an engine for ``weights``: a checkpoint directory defines the
    architecture unless the config pins ``model_overrides`` explicitly."""
    if overrides:
        return model, dict(overrides)
    if weights and os.path.isdir(weights):
        found = checkpoint_model(weights)
        if found is not None:
            return found[0], dict(found[1])
    return model, {}


def _model_id(path: str) -> str:
    m = re.search(r"models--([^/]+)--([^/]+)/snapshots/", path.replace(os.sep, "/"))
    if m:
        return f"{m.group(1)}/{m.group(2)}"
    return os.path.basename(os.path.normpath(path))


def default_search_dirs(project_root: Optional[str] = None) -> List[str]:
    dirs: List[str] = []
    env = os.environ.get("ROUNDTABLE_MODELS_DIR")
    if env:
        dirs.extend(d for d in env.split(os.pathsep) if d)
    if project_root:
        dirs.append(os.path.join(project_root, "models"))
    hf_home = os.environ.get("HF_HOME") or os.path.join(os.path.expanduser("~"), ".cache", "huggingface")
    dirs.append(os.path.join(hf_home, "hub"))
    return dirs


def _candidates(root: str) -> Iterable[str]:
    if not os.path.isdir(root):
        return []
    pats = [os.path.join(root, "config.json"), os.path.join(root, "*", "config.json"),
            os.path.join(root, "*", "*", "config.json"), os.path.join(root, "models--*", "snapshots", "*", "config.json")]
    seen = set()
    for pat in pats:
        for cfg in sorted(glob.glob(pat)):
            d = os.path.dirname(cfg)
            if d not in seen and glob.glob(os.path.join(d, "*.safetensors")):
                seen.add(d)
                yield d


def detect_local_models(search_dirs: Optional[List[str]] = None, project_root: Optional[str] = None) -> List[LocalModel]:
    out: List[LocalModel] = []
    seen_ids = set()
    for root in (search_dirs if search_dirs is not None else default_search_dirs(project_root)):
        for d in _candidates(root):
            mid = _model_id(d)
            if mid in seen_ids or is_non_chat_model(mid):
                continue
            try:
                with open(os.path.join(d, "config.json"), encoding="utf-8") as f:
                    hf = json.load(f)
                shape = _shape_from_hf(hf)
            except (OSError, ValueError, KeyError, TypeError):
                continue
            if shape is None:
                continue
            preset, diff = match_preset(shape)
            seen_ids.add(mid)
            out.append(LocalModel(prettify_model_name(mid), mid, d, preset, diff))
    return out


# ---- running model servers (reference behaviour, `src/utils/local-detect.ts:43-134`) ------------
LOCAL_SERVERS = (("LM Studio", "http://localhost:1234"), ("Ollama", "http://localhost:11434"))


@dataclass
class ServerModel:
    name: str                 # prettified display name
    model_id: str             # id the server reports
    endpoint: str
    source: str               # "LM Studio" | "Ollama"

    def adapter_slug(self) -> str:
        return re.sub(r"[^a-z0-9]+", "-", self.model_id.split("/")[-1].lower()).strip("-")

    def adapter_config(self) -> Dict[str, Any]:
        """``adapter_config`` entry for an external local-llm seat (knights/external.py)."""
        return {"endpoint": self.endpoint, "model": self.model_id, "name": self.name, "source": self.source}


def fetch_models_from_endpoint(endpoint: str, source: str, timeout_s: float = 3.0, http=None) -> List[ServerModel]:
    """``GET <endpoint>/v1/models`` (local-detect.ts:43-71); chat models only, [] on any failure."""
    from ..knights.external import http_request
    try:
        r = (http or http_request)("GET", f"{endpoint}/v1/models", None, {}, timeout_s)
        if not r.ok:
            return []
        data = r.json().get("data") or []
    except Exception:  # noqa: BLE001 - server absent / not JSON
        return []
    out = []
    for m in data:
        mid = m.get("id") if isinstance(m, dict) else None
        if isinstance(mid, str) and mid and not is_non_chat_model(mid):
            out.append(ServerModel(prettify_model_name(mid), mid, endpoint, source))
    return out


def fetch_models_from_ollama_cli(endpoint: str = "http://localhost:11434", run=None) -> List[ServerModel]:
    """Parse ``ollama list`` (local-detect.ts:77-97): first column after the header, ``:latest`` stripped."""
    import subprocess
    try:
        if run is None:
            proc = subprocess.run(["ollama", "list"], capture_output=True, text=True, timeout=5)
            if proc.returncode != 0:
                return []
            text = proc.stdout
        else:
            text = run()
    except (OSError, subprocess.SubprocessError):
        return []
    out = []
    for line in text.splitlines()[1:]:
        cols = line.split()
        if cols:
            mid = re.sub(r":latest$", "", cols[0])
            out.append(ServerModel(prettify_model_name(mid), mid, endpoint, "Ollama"))
    return out


def detect_local_servers(servers=LOCAL_SERVERS, http=None, ollama_cli=None) -> List[ServerModel]:
    """Probe LM Studio and Ollama concurrently; fall back to ``ollama list`` (local-detect.ts:103-134)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=max(1, len(servers))) as ex:
        results = list(ex.map(lambda s: fetch_models_from_endpoint(s[1], s[0], http=http), servers))
    found: List[ServerModel] = [m for r in results for m in r]
    if not any(m.source == "Ollama" for m in found) and any(src == "Ollama" for src, _ in servers):
        ep = next(e for src, e in servers if src == "Ollama")
        found.extend(fetch_models_from_ollama_cli(ep, run=ollama_cli))
    return found
