"""Weight materialization: seeded random init (benchmarks: no network, no checkpoints) or safetensors.

``random:<seed>`` generates every tensor directly on the target device with a
generator seeded by (seed, tensor name, tp rank) — an 8B model materializes in well
under a second on MI355X. ``random-full:<seed>`` builds the *unsharded* tensors on CPU
first and then shards them, so TP=1 and TP=N see identical math (TP equivalence
tests). ``random-dev:<seed>`` does the same with the full tensors generated on the target
device, one tensor at a time (GPU TP checks at 8B / 70B shapes, where CPU generation of the
unsharded model would take minutes and tens of GB of host memory per rank).
A path loads HF-named safetensors (Llama/Mistral/Qwen2/GPT-2 naming) and shards it.
"""
from __future__ import annotations

import hashlib
import os
from typing import Callable, Dict, Optional, Tuple

import torch

from ..parallel.tp import TPInfo, shard_cols, shard_rows
from .config import ModelConfig

# (shape, init-kind, parallel-kind); kinds: "normal", "ones", "zeros"; parallel: None|"row"|"col"|"qkv"|"gateup"|"vocab"


def _seed_for(base: int, name: str, rank: int) -> int:
    h = hashlib.sha256(f"{base}:{name}:{rank}".encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 63) - 1)


def llama_layout(cfg: ModelConfig) -> Dict[str, Tuple[Tuple[int, ...], str, Optional[str]]]:
    H, D = cfg.hidden, cfg.head_dim
    lay: Dict[str, Tuple[Tuple[int, ...], str, Optional[str]]] = {
        "embed": ((cfg.vocab, H), "normal", None),
        "final_norm": ((H,), "ones", None),
        "lm_head": ((cfg.vocab, H), "normal", "vocab"),
    }
    for i in range(cfg.n_layers):
        p = f"layers.{i}."
        lay[p + "attn_norm"] = ((H,), "ones", None)
        lay[p + "wqkv"] = (((cfg.n_heads + 2 * cfg.n_kv_heads) * D, H), "normal", "qkv")
        if cfg.qkv_bias:
            lay[p + "bqkv"] = (((cfg.n_heads + 2 * cfg.n_kv_heads) * D,), "normal", "qkv")
        lay[p + "wo"] = ((H, cfg.n_heads * D), "normal", "col")
        lay[p + "ffn_norm"] = ((H,), "ones", None)
        lay[p + "w_gate_up"] = ((2 * cfg.ffn, H), "normal", "gateup")
        lay[p + "w_down"] = ((H, cfg.ffn), "normal", "col")
    return lay


def gpt2_layout(cfg: ModelConfig) -> Dict[str, Tuple[Tuple[int, ...], str, Optional[str]]]:
    H, F = cfg.hidden, cfg.ffn
    lay: Dict[str, Tuple[Tuple[int, ...], str, Optional[str]]] = {
        "wte": ((cfg.vocab, H), "normal", None),
        "wpe": ((cfg.max_pos, H), "normal", None),
        "ln_f.w": ((H,), "ones", None), "ln_f.b": ((H,), "zeros", None),
    }
    for i in range(cfg.n_layers):
        p = f"layers.{i}."
        lay[p + "ln1.w"] = ((H,), "ones", None)
        lay[p + "ln1.b"] = ((H,), "zeros", None)
        lay[p + "w_qkv"] = ((3 * H, H), "normal", "qkv")
        lay[p + "b_qkv"] = ((3 * H,), "zeros", "qkv")
        lay[p + "w_o"] = ((H, H), "normal", "col")
        lay[p + "b_o"] = ((H,), "zeros", None)
        lay[p + "ln2.w"] = ((H,), "ones", None)
        lay[p + "ln2.b"] = ((H,), "zeros", None)
        lay[p + "w_fc"] = ((F, H), "normal", "row")
        lay[p + "b_fc"] = ((F,), "zeros", "row")
        lay[p + "w_proj"] = ((H, F), "normal", "col")
        lay[p + "b_proj"] = ((H,), "zeros", None)
    return lay


def layout_for(cfg: ModelConfig):
    return gpt2_layout(cfg) if cfg.arch == "gpt2" else llama_layout(cfg)


def shard_tensor(name: str, w: torch.Tensor, kind: Optional[str], cfg: ModelConfig, tp: TPInfo) -> torch.Tensor:
    if tp.size == 1 or kind is None:
        return w
    if kind in ("row", "vocab"):
        if kind == "vocab" and w.shape[0] % tp.size:
            pad = tp.size - w.shape[0] % tp.size
            w = torch.cat([w, w.new_zeros((pad,) + tuple(w.shape[1:]))])
        return shard_rows(w, tp)
    if kind == "col":
        return shard_cols(w, tp)
    if kind == "gateup":
        g, u = w.chunk(2, dim=0)
        return torch.cat([shard_rows(g, tp), shard_rows(u, tp)])
    if kind == "qkv":
        D = cfg.head_dim
        q, k, v = w.split([cfg.n_heads * D, cfg.n_kv_heads * D, cfg.n_kv_heads * D], dim=0)
        h0, nh = tp.kv_head0(cfg.n_kv_heads), tp.kv_heads(cfg.n_kv_heads)
        return torch.cat([shard_rows(q, tp), k[h0 * D:(h0 + nh) * D], v[h0 * D:(h0 + nh) * D]])
    raise ValueError(kind)


def local_shape(shape, kind, cfg: ModelConfig, tp: TPInfo):
    if tp.size == 1 or kind is None:
        return shape
    s = list(shape)
    if kind in ("row", "gateup"):
        s[0] //= tp.size
    elif kind == "vocab":
        s[0] = (s[0] + tp.size - 1) // tp.size
    elif kind == "col":
        s[1] //= tp.size
    elif kind == "qkv":
        s[0] = (cfg.n_heads // tp.size + 2 * tp.kv_heads(cfg.n_kv_heads)) * cfg.head_dim
    return tuple(s)


def materialize(cfg: ModelConfig, spec: str, device, dtype=torch.bfloat16, tp: Optional[TPInfo] = None,
                std: float = 0.02) -> Dict[str, torch.Tensor]:
    tp = tp or TPInfo()
    lay = layout_for(cfg)
    out: Dict[str, torch.Tensor] = {}
    if spec.startswith(("random:", "random-full:", "random-dev:")):
        full = spec.startswith(("random-full:", "random-dev:"))
        gen_dev = torch.device(device) if spec.startswith("random-dev:") else torch.device("cpu")
        seed = int(spec.split(":", 1)[1] or 0)
        for name, (shape, init, kind) in lay.items():
            if full:
                g = torch.Generator(device=gen_dev).manual_seed(_seed_for(seed, name, 0))
                w = _init(shape, init, std, g, gen_dev, torch.float32)
                if init == "normal" and name in ("embed", "wte"):
                    w = w * 10  # unit-ish scale residual stream for the embedding
                out[name] = shard_tensor(name, w, kind, cfg, tp).to(device=device, dtype=dtype).contiguous()
                del w
            else:
                shp = local_shape(shape, kind, cfg, tp)
                dev = torch.device(device)
                g = torch.Generator(device=dev).manual_seed(_seed_for(seed, name, tp.rank))
                w = _init(shp, init, std, g, dev, dtype)
                if init == "normal" and name in ("embed", "wte"):
                    w.mul_(10)
                out[name] = w
        # GPT-2 reads its tied head from wte; a tied Llama-family model (random init) keeps an
        # independent vocab-parallel lm_head (checkpoints copy the embedding, load_safetensors)
        if cfg.tie_embeddings and cfg.arch == "gpt2" and "lm_head" in out:
            out.pop("lm_head")
        return out
    if os.path.isdir(spec) or spec.endswith(".safetensors"):
        return load_safetensors(cfg, spec, device, dtype, tp)
    raise ValueError(f"unknown weights spec '{spec}' (use random:<seed>, random-full:<seed>, or a path)")


def _init(shape, init, std, g, device, dtype):
    if init == "ones":
        return torch.ones(shape, device=device, dtype=dtype)
    if init == "zeros":
        return torch.zeros(shape, device=device, dtype=dtype)
    w = torch.empty(shape, device=device, dtype=dtype)
    w.normal_(0.0, std, generator=g)
    return w


# ---- safetensors (HF naming) -----------------------------------------------------------------

def _hf_llama_name_map(cfg: ModelConfig) -> Dict[str, Callable[[Dict[str, torch.Tensor]], torch.Tensor]]:
    m: Dict[str, Callable] = {
        "embed": lambda t: t["model.embed_tokens.weight"],
        "final_norm": lambda t: t["model.norm.weight"],
        "lm_head": lambda t: t.get("lm_head.weight", t["model.embed_tokens.weight"]),
    }
    for i in range(cfg.n_layers):
        p = f"model.layers.{i}."
        m[f"layers.{i}.attn_norm"] = lambda t, p=p: t[p + "input_layernorm.weight"]
        m[f"layers.{i}.ffn_norm"] = lambda t, p=p: t[p + "post_attention_layernorm.weight"]
        m[f"layers.{i}.wqkv"] = lambda t, p=p: torch.cat([t[p + "self_attn.q_proj.weight"],
                                                           t[p + "self_attn.k_proj.weight"],
                                                           t[p + "self_attn.v_proj.weight"]])
        if cfg.qkv_bias:
            m[f"layers.{i}.bqkv"] = lambda t, p=p: torch.cat([t[p + "self_attn.q_proj.bias"],
                                                               t[p + "self_attn.k_proj.bias"],
                                                               t[p + "self_attn.v_proj.bias"]])
        m[f"layers.{i}.wo"] = lambda t, p=p: t[p + "self_attn.o_proj.weight"]
        m[f"layers.{i}.w_gate_up"] = lambda t, p=p: torch.cat([t[p + "mlp.gate_proj.weight"],
                                                               t[p + "mlp.up_proj.weight"]])
        m[f"layers.{i}.w_down"] = lambda t, p=p: t[p + "mlp.down_proj.weight"]
    return m


def _hf_gpt2_name_map(cfg: ModelConfig):
    pre = "transformer."

    def g(t, n):
        return t[pre + n] if pre + n in t else t[n]

    m: Dict[str, Callable] = {"wte": lambda t: g(t, "wte.weight"), "wpe": lambda t: g(t, "wpe.weight"),
                              "ln_f.w": lambda t: g(t, "ln_f.weight"), "ln_f.b": lambda t: g(t, "ln_f.bias")}
    for i in range(cfg.n_layers):
        p = f"h.{i}."
        # HF GPT-2 uses Conv1D ([in, out]); transpose to [out, in]
        m[f"layers.{i}.ln1.w"] = lambda t, p=p: g(t, p + "ln_1.weight")
        m[f"layers.{i}.ln1.b"] = lambda t, p=p: g(t, p + "ln_1.bias")
        m[f"layers.{i}.w_qkv"] = lambda t, p=p: g(t, p + "attn.c_attn.weight").t()
        m[f"layers.{i}.b_qkv"] = lambda t, p=p: g(t, p + "attn.c_attn.bias")
        m[f"layers.{i}.w_o"] = lambda t, p=p: g(t, p + "attn.c_proj.weight").t()
        m[f"layers.{i}.b_o"] = lambda t, p=p: g(t, p + "attn.c_proj.bias")
        m[f"layers.{i}.ln2.w"] = lambda t, p=p: g(t, p + "ln_2.weight")
        m[f"layers.{i}.ln2.b"] = lambda t, p=p: g(t, p + "ln_2.bias")
        m[f"layers.{i}.w_fc"] = lambda t, p=p: g(t, p + "mlp.c_fc.weight").t()
        m[f"layers.{i}.b_fc"] = lambda t, p=p: g(t, p + "mlp.c_fc.bias")
        m[f"layers.{i}.w_proj"] = lambda t, p=p: g(t, p + "mlp.c_proj.weight").t()
        m[f"layers.{i}.b_proj"] = lambda t, p=p: g(t, p + "mlp.c_proj.bias")
    return m


def load_safetensors(cfg: ModelConfig, path: str, device, dtype, tp: TPInfo) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    files = [path] if path.endswith(".safetensors") else sorted(
        os.path.join(path, f) for f in os.listdir(path) if f.endswith(".safetensors"))
    tensors: Dict[str, torch.Tensor] = {}
    for f in files:
        tensors.update(load_file(f, device="cpu"))
    name_map = _hf_gpt2_name_map(cfg) if cfg.arch == "gpt2" else _hf_llama_name_map(cfg)
    lay = layout_for(cfg)
    out = {}
    for name, fn in name_map.items():
        if name == "lm_head" and cfg.tie_embeddings and cfg.arch == "gpt2":
            continue   # GPT-2 reads the tied head from wte; Llama-family models get a (sharded) copy
        w = fn(tensors)
        kind = lay[name][2]
        out[name] = shard_tensor(name, w.float(), kind, cfg, tp).to(device=device, dtype=dtype).contiguous()
    return out
