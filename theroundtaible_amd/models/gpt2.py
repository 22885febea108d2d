"""GPT-2 (learned positions, pre-LayerNorm, GELU-tanh MLP, MHA, tied lm_head).

Config 1 of BASELINE.json (2-knight discuss on CPU) runs this model through the same
engine (paged KV, chunked prefill, decode loop) on the PyTorch reference ops; on GPU
the same code path dispatches to the HIP kernels (head_dim 64 variants).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel.tp import TPInfo
from .config import ModelConfig
from .llama import AttnMeta


class GPT2Model:
    def __init__(self, cfg: ModelConfig, weights: Dict[str, torch.Tensor], device, dtype=torch.bfloat16,
                 tp: Optional[TPInfo] = None):
        self.cfg = cfg
        self.w = weights
        self.tp = tp or TPInfo()
        self.device = device
        self.dtype = dtype
        if cfg.n_heads % self.tp.size or cfg.ffn % self.tp.size:
            raise ValueError(f"{cfg.name}: {cfg.n_heads} heads / FFN {cfg.ffn} do not split over tp={self.tp.size}")
        self.n_heads = cfg.n_heads // self.tp.size
        self.n_kv_heads = self.n_heads
        self.head_dim = cfg.head_dim
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.layers = [{k.split(".", 2)[2]: v for k, v in weights.items() if k.startswith(f"layers.{i}.")}
                       for i in range(cfg.n_layers)]
        if self.tp.size > 1:
            vs = self.tp.shard((cfg.vocab + self.tp.size - 1) // self.tp.size * self.tp.size)
            wte = weights["wte"]
            pad = vs * self.tp.size - wte.shape[0]
            if pad:
                wte = torch.cat([wte, wte.new_zeros(pad, wte.shape[1])])
            self.lm_head = wte[self.tp.rank * vs:(self.tp.rank + 1) * vs].contiguous()
        else:
            self.lm_head = weights["wte"]

    @property
    def kv_heads_local(self) -> int:
        return self.n_kv_heads

    def forward(self, ids: torch.Tensor, positions: torch.Tensor, kv, meta: AttnMeta) -> torch.Tensor:
        cfg, tp = self.cfg, self.tp
        T = ids.shape[0]
        h = F.embedding(ids, self.w["wte"]) + F.embedding(positions.long(), self.w["wpe"])
        res = None
        for l, lw in enumerate(self.layers):
            if res is None:
                res = h
                x = ops.layer_norm(h, lw["ln1.w"], lw["ln1.b"], cfg.norm_eps)
            else:
                x, res = ops.fused_add_layer_norm(h, res, lw["ln1.w"], lw["ln1.b"], cfg.norm_eps)
            qkv = F.linear(x, lw["w_qkv"], lw["b_qkv"])
            q = ops.rope_and_cache(qkv, positions, None, kv.k_layer(l), kv.v_layer(l), meta.slot_mapping,
                                   self.n_heads, self.n_kv_heads, self.head_dim)
            if meta.kind == "decode":
                a = ops.paged_attention_decode(q, kv.k_layer(l), kv.v_layer(l), meta.block_tables, meta.ctx_lens,
                                               self.scale, meta.num_splits, meta.workspace, groups=meta.groups)
            else:
                a = ops.prefill_attention(q, kv.k_layer(l), kv.v_layer(l), meta.block_tables, meta.cu_q,
                                          meta.start_pos, self.scale, meta.tile_map)
            h = tp.all_reduce(F.linear(a.reshape(T, -1), lw["w_o"])) + lw["b_o"]
            x, res = ops.fused_add_layer_norm(h, res, lw["ln2.w"], lw["ln2.b"], cfg.norm_eps)
            m = ops.gelu_tanh(F.linear(x, lw["w_fc"], lw["b_fc"]))
            h = tp.all_reduce(F.linear(m, lw["w_proj"])) + lw["b_proj"]
        if meta.kind == "prefill" and meta.last_rows is not None:
            h = h.index_select(0, meta.last_rows)
            res = res.index_select(0, meta.last_rows)
        x, _ = ops.fused_add_layer_norm(h, res, self.w["ln_f.w"], self.w["ln_f.b"], cfg.norm_eps)
        logits = F.linear(x, self.lm_head)
        if meta.kind == "decode" and meta.local_logits:
            return logits
        logits = tp.all_gather_last(logits)
        return logits[:, :cfg.vocab]


def build_model(cfg: ModelConfig, weights, device, dtype=torch.bfloat16, tp: Optional[TPInfo] = None):
    if cfg.arch == "gpt2":
        return GPT2Model(cfg, weights, device, dtype, tp)
    from .llama import LlamaModel
    return LlamaModel(cfg, weights, device, dtype, tp)
