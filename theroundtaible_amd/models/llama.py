"""Llama-3 / Mistral decoder (dense, GQA, RoPE, SwiGLU, RMSNorm), TP-aware.

Per layer (decode and prefill share the code; only the attention op differs):

    x, res = fused_add_rms_norm(h, res)          K1 (HIP)
    qkv    = x @ Wqkv^T                          hipBLASLt (column-parallel)
    q      = rope_and_cache(qkv, ...)            K2 (HIP): RoPE on q/k + paged K/V scatter
    a      = paged_decode | prefill attention    K3 / K4 (HIP, MFMA)
    h      = a @ Wo^T ; all_reduce               hipBLASLt (row-parallel) + RCCL (C2)
    x, res = fused_add_rms_norm(h, res)          K1
    h      = silu_and_mul(x @ Wgu^T) @ Wd^T      hipBLASLt + K5 (HIP) + hipBLASLt ; all_reduce
    logits = final_norm(h) @ Wlm^T ; all_gather  hipBLASLt (vocab-parallel) + RCCL (C3)
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..ops.reference import rope_cos_sin
from ..parallel.tp import TPInfo
from .config import ModelConfig


@dataclass
class AttnMeta:
    """Per-forward attention metadata (device tensors)."""
    kind: str                               # "decode" | "prefill"
    slot_mapping: torch.Tensor              # [T] int64
    block_tables: torch.Tensor              # [S, max_blocks] int32
    ctx_lens: Optional[torch.Tensor] = None     # decode: [B] int32
    num_splits: int = 1                         # decode split-KV
    workspace: Optional[ops.DecodeWorkspace] = None
    cu_q: Optional[torch.Tensor] = None         # prefill: [S+1] int32
    start_pos: Optional[torch.Tensor] = None    # prefill: [S] int32
    tile_map: Optional[torch.Tensor] = None     # prefill: [n_tiles, 2] int32
    last_rows: Optional[torch.Tensor] = None    # prefill: rows whose logits are needed


class LlamaModel:
    def __init__(self, cfg: ModelConfig, weights: Dict[str, torch.Tensor], device, dtype=torch.bfloat16,
                 tp: Optional[TPInfo] = None):
        self.cfg = cfg
        self.w = weights
        self.tp = tp or TPInfo()
        self.device = device
        self.dtype = dtype
        self.n_heads = cfg.n_heads // self.tp.size
        self.n_kv_heads = cfg.n_kv_heads // self.tp.size
        self.head_dim = cfg.head_dim
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.cos_sin = rope_cos_sin(cfg.max_pos, cfg.head_dim, cfg.rope_theta, device)
        self.layers = [{k.split(".", 2)[2]: v for k, v in weights.items() if k.startswith(f"layers.{i}.")}
                       for i in range(cfg.n_layers)]

    @property
    def kv_heads_local(self) -> int:
        return self.n_kv_heads

    def attention(self, q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        if meta.kind == "decode":
            return ops.paged_attention_decode(q, kc, vc, meta.block_tables, meta.ctx_lens, self.scale,
                                              meta.num_splits, meta.workspace)
        return ops.prefill_attention(q, kc, vc, meta.block_tables, meta.cu_q, meta.start_pos, self.scale,
                                     meta.tile_map)

    def forward(self, ids: torch.Tensor, positions: torch.Tensor, kv, meta: AttnMeta) -> torch.Tensor:
        """Returns logits [rows, vocab] (all rows for decode, ``meta.last_rows`` for prefill)."""
        cfg, tp = self.cfg, self.tp
        T = ids.shape[0]
        h = F.embedding(ids, self.w["embed"])
        res = None
        for l, lw in enumerate(self.layers):
            if res is None:
                res = h
                x = ops.rms_norm(h, lw["attn_norm"], cfg.norm_eps)
            else:
                x, res = ops.fused_add_rms_norm(h, res, lw["attn_norm"], cfg.norm_eps)
            qkv = F.linear(x, lw["wqkv"])
            q = ops.rope_and_cache(qkv, positions, self.cos_sin, kv.k_layer(l), kv.v_layer(l), meta.slot_mapping,
                                   self.n_heads, self.n_kv_heads, self.head_dim)
            a = self.attention(q, kv.k_layer(l), kv.v_layer(l), meta)
            h = tp.all_reduce(F.linear(a.reshape(T, -1), lw["wo"]))
            x, res = ops.fused_add_rms_norm(h, res, lw["ffn_norm"], cfg.norm_eps)
            g = ops.silu_and_mul(F.linear(x, lw["w_gate_up"]))
            h = tp.all_reduce(F.linear(g, lw["w_down"]))
        if meta.kind == "prefill" and meta.last_rows is not None:
            h = h.index_select(0, meta.last_rows)
            res = res.index_select(0, meta.last_rows)
        x, _ = ops.fused_add_rms_norm(h, res.clone() if not res.is_cuda else res, self.w["final_norm"], cfg.norm_eps)
        logits = F.linear(x, self.w["lm_head"])
        logits = tp.all_gather_last(logits)
        return logits[:, :cfg.vocab]
