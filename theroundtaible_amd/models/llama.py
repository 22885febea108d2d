"""Llama-3 / Mistral / Qwen2 decoder (dense, GQA, RoPE, SwiGLU, RMSNorm; Qwen2: q/k/v bias), TP-aware.

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

import os

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
    prefill_split: Optional[tuple] = None       # prefill: ops.prefill_split_plan (items, cmap, parts) on device
    last_rows: Optional[torch.Tensor] = None    # prefill: rows whose logits are needed
    groups: Optional[torch.Tensor] = None       # decode: [B, 3] shared-prefix groups (ops.decode_groups)
    local_logits: bool = False                  # TP decode: return this rank's vocab shard (C3 greedy argmax)
    planned: bool = False                       # decode: the workspace holds this step's ops.attn_plan


class LlamaModel:
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
        self.n_kv_heads = self.tp.kv_heads(cfg.n_kv_heads)   # replicated when tp > KV heads
        self.head_dim = cfg.head_dim
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.cos_sin = rope_cos_sin(cfg.max_pos, cfg.head_dim, cfg.rope_theta, device, cfg.rope_scaling)
        self.layers = [{k.split(".", 2)[2]: v for k, v in weights.items() if k.startswith(f"layers.{i}.")}
                       for i in range(cfg.n_layers)]
        self.lm_rows = weights["lm_head"].shape[0]   # (vocab shard) rows of the lm_head

    @property
    def kv_heads_local(self) -> int:
        return self.n_kv_heads

    def attention(self, q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        if meta.kind == "decode":
            return ops.paged_attention_decode(q, kc, vc, meta.block_tables, meta.ctx_lens, self.scale,
                                              meta.num_splits, meta.workspace, groups=meta.groups,
                                              planned=meta.planned)
        return ops.prefill_attention(q, kc, vc, meta.block_tables, meta.cu_q, meta.start_pos, self.scale,
                                     meta.tile_map, split=meta.prefill_split)

    def fused_decode_ok(self, ids: torch.Tensor) -> bool:
        """The fused decode path takes up to 16 rows, up to 32 at tp 1 (serving batches: the skinny
        GEMMs' two-row-block launches, csrc/skinny_core.h gemm_tiles; the tensor-parallel epilogues
        stay at 16)."""
        cfg = self.cfg
        rows = 32 if self.tp.size == 1 and not self.force_tp_path else 16
        rows = min(rows, int(os.environ.get("ROUNDTABLE_FUSED_ROWS", rows)))   # A/B knob
        return (ids.is_cuda and 1 <= ids.shape[0] <= rows and self.use_fused
                and cfg.hidden % 32 == 0 and cfg.ffn % 32 == 0 and (cfg.n_heads * cfg.head_dim) % 32 == 0
                and self.lm_rows % 16 == 0)

    use_fused = True
    force_tp_path = False   # tests: run the tensor-parallel fused path at tp=1 (all-reduces are no-ops)
    _dec = None

    # shuffled-only residency: the row-major linears were dropped after shuffling (a knight whose
    # weights do not fit twice, e.g. Llama-3-70B on one GPU); prefill GEMMs rebuild each row-major
    # (gamma-folded) operand in a per-shape scratch buffer with ops.unshuffle_weight
    shuffled_only = False
    _scratch: Optional[Dict[tuple, torch.Tensor]] = None

    # (name, folded norm, shuffle kwargs) of the linears the fused decode path streams
    def _lin_specs(self):
        return (("wqkv", "attn_norm", {"rope_heads": self.n_heads + self.n_kv_heads, "head_dim": self.head_dim}),
                ("wo", None, {}), ("w_gate_up", "ffn_norm", {"swiglu": True}), ("w_down", None, {}))

    def decode_weights(self, drop_originals: bool = False):
        """Fragment-shuffled, norm-folded copies of every linear for the fused decode path (built
        lazily once). Default: +1x weight memory, affordable on 288 GB HBM for 7-8B knights.
        ``drop_originals``: shuffle one linear at a time and free its row-major tensor (peak +1
        tensor), so only ONE copy of the weights stays resident (see :attr:`shuffled_only`)."""
        if self._dec is None:
            with torch.no_grad():
                layers = []
                for i, lw in enumerate(self.layers):
                    d = {}
                    for name, norm, kw in self._lin_specs():
                        d[name] = ops.shuffle_weight(lw[name], lw[norm] if norm else None, **kw)
                        if drop_originals:
                            # drop BOTH references (the per-layer view and the flat dict) now, so the
                            # allocator reuses this tensor's memory for the next shuffle: the load peak
                            # stays one weight copy + one tensor
                            lw[name] = None
                            self.w[f"layers.{i}.{name}"] = None
                    if lw.get("bqkv") is not None:   # Qwen2: the bias the qkv epilogue adds before RoPE
                        d["bqkv"] = ops.rope_bias(lw["bqkv"], self.n_heads, self.n_kv_heads, self.head_dim)
                    layers.append(d)
                lm = ops.shuffle_weight(self.w["lm_head"], self.w["final_norm"])
                if drop_originals:
                    self.w["lm_head"] = None
                    for k in [k for k in self.w if k.startswith("layers.") and k.split(".", 2)[2] in
                              ("wqkv", "wo", "w_gate_up", "w_down")] + ["lm_head"]:
                        self.w[k] = None
                    self.shuffled_only = True
                    self._scratch = {}
                    if self.device.type == "cuda":
                        torch.cuda.empty_cache()
                # ONE split workspace for every decode GEMM of this model (they run in order on
                # the engine's stream; counters re-arm at the end of each call): split-K for shard
                # shapes with fewer tiles than CUs (tensor parallel), and the balanced launch of
                # gate_up, whose tile count (ffn/16) is rarely a multiple of the CU count
                ws = ops.split_workspace(lm.device) if lm.is_cuda else None
                self._dec = {"layers": layers, "lm_head": lm, "split_ws": ws}
        return self._dec

    def _row_major(self, l: Optional[int], name: str) -> torch.Tensor:
        """The row-major operand of a prefill / unfused GEMM: the resident tensor, or (shuffled-only
        residency) the gamma-folded weight unshuffled into a scratch buffer reused per shape."""
        if not self.shuffled_only:
            return self.layers[l][name] if l is not None else self.w[name]
        if l is None:
            Ws, kw = self._dec["lm_head"], {}
        else:
            Ws = self._dec["layers"][l][name]
            kw = next(k for n, _, k in self._lin_specs() if n == name)
        key = tuple(Ws.shape)
        buf = self._scratch.get(key)
        if buf is None:
            buf = self._scratch[key] = torch.empty_like(Ws)
        return ops.unshuffle_weight(Ws, out=buf, **kw)

    def _norm_w(self, l: Optional[int], name: str) -> torch.Tensor:
        """Norm weight of the unfused path: ones when gamma is folded into the next linear."""
        w = self.layers[l][name] if l is not None else self.w[name]
        if self.shuffled_only:
            ones = self._scratch.get(("ones", w.numel()))
            if ones is None:
                ones = self._scratch[("ones", w.numel())] = torch.ones_like(w)
            return ones
        return w

    accepts_hidden = True  # forward(..., hidden=) takes pre-gathered embedding rows (decode_prep)

    def forward_decode_fused(self, ids: torch.Tensor, positions: torch.Tensor, kv, meta: AttnMeta,
                             hidden: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Decode step with every norm / residual / activation fused into the MFMA GEMMs
        (csrc/gemm_skinny.hip): per layer qkv(+RMSNorm, +RoPE/KV-cache write) -> K3 (+ its split
        combine launch) -> o(+residual) -> gate_up(+RMSNorm, SwiGLU) -> down(+residual); no norm /
        rope / reduce kernels. (Folding the combine into the o launch measured slower:
        tools/experiments/combine_o.hip.)"""
        cfg = self.cfg
        eps = cfg.norm_eps
        dec = self.decode_weights()
        # the residual stream is updated in place by every RESID epilogue
        res = hidden if hidden is not None else F.embedding(ids, self.w["embed"]).contiguous()
        B = ids.shape[0]
        sw, SK, ALL = dec["split_ws"], ops.SPLIT_K, ops.SPLIT_K | ops.SPLIT_BALANCE
        for l, lw in enumerate(dec["layers"]):
            q = ops.skinny_gemm_rope(res, lw["wqkv"], ops.PRO_NORM, positions, self.cos_sin, kv.k_layer(l),
                                     kv.v_layer(l), meta.slot_mapping, self.n_heads, self.n_kv_heads,
                                     self.head_dim, eps, split_ws=sw, split_mode=SK, bias=lw.get("bqkv"))
            a = self.attention(q, kv.k_layer(l), kv.v_layer(l), meta)
            ops.skinny_gemm(a.reshape(B, -1), lw["wo"], ops.PRO_PLAIN, ops.EPI_RESID, res=res, split_ws=sw,
                            split_mode=SK)
            g = ops.skinny_gemm(res, lw["w_gate_up"], ops.PRO_NORM, ops.EPI_SWIGLU, eps=eps, split_ws=sw,
                                split_mode=ALL)
            ops.skinny_gemm(g, lw["w_down"], ops.PRO_PLAIN, ops.EPI_RESID, res=res, split_ws=sw, split_mode=SK)
        logits = ops.skinny_gemm(res, dec["lm_head"], ops.PRO_NORM, ops.EPI_STORE, eps=eps, split_ws=sw,
                                 split_mode=SK)
        return logits[:, :cfg.vocab]

    def forward_decode_fused_tp(self, ids: torch.Tensor, positions: torch.Tensor, kv, meta: AttnMeta,
                                hidden: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Tensor-parallel fused decode (Megatron split), the same 4 GEMMs per
        layer as tp 1: qkv (RMSNorm + RoPE/KV-cache epilogue) -> K3 -> o -> gate_up (RMSNorm +
        SwiGLU) -> down. o / down are row-parallel: their partial sums are all-reduced over the
        group (C2) and added into the residual stream in place by the same launch — the K9 exchange
        in the GEMM epilogue when the one-shot comm passed its fused self-test, else the GEMM + a
        K9 launch in its residual form (``tp.row_parallel(res=)``). The lm_head is vocab-parallel
        + all-gather (C3). Round 3 instead handed the partial to the next GEMM's NORM_ADD
        prologue, which re-added it in every workgroup: 1-3 us per GEMM at shard shapes
        (profiles/r04/gemm_variants.md). qkv never takes split-K (its seam cost more than the
        48-192 unsplit tiles lose; same table)."""
        cfg, tp = self.cfg, self.tp
        eps = cfg.norm_eps
        dec = self.decode_weights()
        # the residual stream is updated in place by every row-parallel launch
        res = hidden if hidden is not None else F.embedding(ids, self.w["embed"]).contiguous()
        B = ids.shape[0]
        sk = dict(split_ws=dec["split_ws"], split_mode=ops.SPLIT_K)
        for l, lw in enumerate(dec["layers"]):
            kc, vc = kv.k_layer(l), kv.v_layer(l)
            q = ops.skinny_gemm_rope(res, lw["wqkv"], ops.PRO_NORM, positions, self.cos_sin, kc, vc,
                                     meta.slot_mapping, self.n_heads, self.n_kv_heads, self.head_dim, eps,
                                     split_ws=dec["split_ws"], split_mode=0, bias=lw.get("bqkv"))
            a = self.attention(q, kc, vc, meta)
            tp.row_parallel(a.reshape(B, -1), lw["wo"], res=res, **sk)
            g = ops.skinny_gemm(res, lw["w_gate_up"], ops.PRO_NORM, ops.EPI_SWIGLU, eps=eps, **sk)
            tp.row_parallel(g, lw["w_down"], res=res, **sk)
        logits = ops.skinny_gemm(res, dec["lm_head"], ops.PRO_NORM, ops.EPI_STORE, eps=eps, **sk)
        if meta.local_logits:
            return logits
        logits = tp.all_gather_last(logits)
        return logits[:, :cfg.vocab]

    def forward(self, ids: torch.Tensor, positions: torch.Tensor, kv, meta: AttnMeta,
                hidden: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Returns logits [rows, vocab] (all rows for decode, ``meta.last_rows`` for prefill).
        ``hidden``: optional pre-gathered embedding rows (used by the fused decode path only)."""
        if meta.kind == "decode":
            # one attention work plan per decode step, read by all layers' launches
            meta.planned = ops.attn_plan(meta.block_tables, meta.ctx_lens, meta.num_splits, meta.workspace,
                                         self.n_heads, self.n_kv_heads, meta.groups, ids.shape[0])
        if meta.kind == "decode" and self.fused_decode_ok(ids):
            if self.tp.size > 1 or self.force_tp_path:
                return self.forward_decode_fused_tp(ids, positions, kv, meta, hidden)
            return self.forward_decode_fused(ids, positions, kv, meta, hidden)
        cfg, tp = self.cfg, self.tp
        T = ids.shape[0]
        h = F.embedding(ids, self.w["embed"])
        res = None
        for l, lw in enumerate(self.layers):
            if res is None:
                res = h
                x = ops.rms_norm(h, self._norm_w(l, "attn_norm"), cfg.norm_eps)
            else:
                x, res = ops.fused_add_rms_norm(h, res, self._norm_w(l, "attn_norm"), cfg.norm_eps)
            qkv = F.linear(x, self._row_major(l, "wqkv"), lw.get("bqkv"))
            q = ops.rope_and_cache(qkv, positions, self.cos_sin, kv.k_layer(l), kv.v_layer(l), meta.slot_mapping,
                                   self.n_heads, self.n_kv_heads, self.head_dim)
            a = self.attention(q, kv.k_layer(l), kv.v_layer(l), meta)
            h = tp.all_reduce(F.linear(a.reshape(T, -1), self._row_major(l, "wo")))
            x, res = ops.fused_add_rms_norm(h, res, self._norm_w(l, "ffn_norm"), cfg.norm_eps)
            g = ops.silu_and_mul(F.linear(x, self._row_major(l, "w_gate_up")))
            h = tp.all_reduce(F.linear(g, self._row_major(l, "w_down")))
        if meta.kind == "prefill" and meta.last_rows is not None:
            h = h.index_select(0, meta.last_rows)
            res = res.index_select(0, meta.last_rows)
        x, _ = ops.fused_add_rms_norm(h, res.clone() if not res.is_cuda else res, self._norm_w(None, "final_norm"),
                                      cfg.norm_eps)
        logits = F.linear(x, self._row_major(None, "lm_head"))
        if meta.kind == "decode" and meta.local_logits:
            return logits
        logits = tp.all_gather_last(logits)
        return logits[:, :cfg.vocab]
