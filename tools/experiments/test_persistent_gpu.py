"""EXPERIMENT (not adopted): persistent decode-layer kernel (decode_layer.hip) vs the five-launch
fused path. Needs ``python tools/experiments/build_exp.py`` first."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.engine import Engine, EngineConfig  # noqa: E402
from theroundtaible_amd.models.llama import AttnMeta  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _engine(**kw):
    cfg = dict(model="tiny-llama-128", weights="random-full:5", device=DEV, num_blocks=256, use_graphs=False)
    cfg.update(kw)
    return Engine(EngineConfig(**cfg))


def _decode_meta(e, seqs, splits):
    for s in seqs:
        e.kv.ensure_capacity(s, s.length + 1)
    pos = torch.tensor([s.length for s in seqs], device=DEV)
    slots = torch.tensor([s.blocks[p // 32] * 32 + p % 32 for s, p in zip(seqs, pos.tolist())], device=DEV)
    bt = torch.zeros(len(seqs), 16, dtype=torch.int32)
    for j, s in enumerate(seqs):
        bt[j, :len(s.blocks)] = torch.tensor(s.blocks)
    ws = ops.DecodeWorkspace(len(seqs), e.model.n_heads, e.cfg.head_dim, splits, DEV)
    return pos, AttnMeta("decode", slots, bt.to(DEV), (pos + 1).to(torch.int32), num_splits=splits, workspace=ws)


def _persistent_forward(e, ids, positions, meta):
    """The fused decode forward with every layer as ONE persistent launch (experiment module)."""
    import torch.nn.functional as F
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from build_exp import load
    exp = load()
    m, kv = e.model, e.kv
    dec = m.decode_weights()
    res = F.embedding(ids, m.w["embed"]).contiguous()
    M, D = res.shape[0], m.head_dim
    for l, lw in enumerate(dec["layers"]):
        q = torch.empty(M, m.n_heads, D, dtype=res.dtype, device=res.device)
        a = torch.empty(M, m.n_heads * D, dtype=res.dtype, device=res.device)
        g = torch.empty(M, lw["w_down"].shape[1], dtype=res.dtype, device=res.device)
        ws = meta.workspace
        exp.decode_layer(res, q, a, g, lw["wqkv"], lw["wo"], lw["w_gate_up"], lw["w_down"], positions, m.cos_sin,
                         kv.k_layer(l), kv.v_layer(l), meta.slot_mapping, meta.block_tables, meta.ctx_lens,
                         ws.partial_o, ws.partial_ml, ws.counters, ws.sync, ws.err, m.n_heads, m.n_kv_heads,
                         max(1, meta.num_splits), m.cfg.norm_eps, m.scale)
    logits = ops.skinny_gemm(res, dec["lm_head"], ops.PRO_NORM, ops.EPI_STORE, eps=m.cfg.norm_eps)
    return logits[:, :m.cfg.vocab]


@pytest.mark.parametrize("splits", [1, 4])
def test_persistent_layer_matches_five_launches(splits):
    e = _engine()
    ids = e.encode_prompt("persistent layer kernel versus five launches " * 6)
    seqs = [e.kv.seq("a"), e.kv.seq("b"), e.kv.seq("c")]
    e.prefill([(seqs[0], ids), (seqs[1], ids[:-5]), (seqs[2], ids[:40])])
    pos, meta = _decode_meta(e, seqs, splits)
    tok = torch.tensor([5, 7, 11], device=DEV)
    ref = e.model.forward(tok, pos, e.kv, meta).float()
    kc = e.kv.k_layer(0).clone()
    got = _persistent_forward(e, tok, pos, meta).float()
    torch.cuda.synchronize()
    assert int(meta.workspace.err.item()) == 0, "a phase poll expired"
    assert int(meta.workspace.sync.abs().sum()) == 0, "phase counters were not re-armed"
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert float(cos.min()) > 0.999
    # the K/V written by the persistent qkv phase equals the five-launch path's
    assert torch.allclose(e.kv.k_layer(0).float(), kc.float(), atol=2e-2, rtol=2e-2)
