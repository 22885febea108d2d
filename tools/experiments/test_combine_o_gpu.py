"""EXPERIMENT (not adopted): K3 split combine + o-projection + residual in one launch
(tools/experiments/combine_o.hip) vs the fp32 oracle: grouped (shared-prefix) and ungrouped decode, split counts that defer the combine and
one that does not (attention writes its rows itself), repeat launches (the grid barrier re-arms)
and the separate-launch path it replaces."""
import math
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.dirname(os.path.abspath(__file__))]
from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.ops import reference as ref  # noqa: E402
from test_kernels_gpu import DEV, bf, close, make_cache  # noqa: E402

pytestmark = pytest.mark.gpu


def attention_o_resid(q, kc, vc, bt, cl, scale, splits, ws, groups, Ws, res, fused=True):
    """Attention then ``res += attn . Wo^T``; ``fused``: the split combine inside the o launch."""
    import _exp
    B = q.shape[0]
    out = torch.empty_like(q)
    stride = ws.slot_stride if groups is not None else 0
    deferred = ops.native().paged_attention_decode(out, q, kc, vc, bt, cl, scale, int(splits), ws.partial_o,
                                                   ws.partial_ml, ws.counters, groups, stride, fused)
    if deferred:
        _exp.combine_o_gemm(out, ws.partial_o, ws.partial_ml, groups, stride, int(splits), int(kc.shape[1]), Ws,
                            res, ws.sync[6:8], ws.err)
    else:
        ops.skinny_gemm(out.reshape(B, -1), Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res)


def _case(hq, hkv, grouped, seed=3):
    d = 128
    G = hq // hkv
    g = torch.Generator().manual_seed(seed)
    if grouped:   # one table: 3 knights over a 1900-token shared prefix + private tails
        spec = [("A", 1900 // 32, [1900 + 7, 1900 + 300, 1900 + 33])]
    else:
        spec = [(None, 0, [700]), (None, 0, [2100]), (None, 0, [33])]
    lens, group_of, shared = [], [], []
    for label, sh, ls in spec:
        for l in ls:
            lens.append(l)
            group_of.append(label)
            shared.append(sh)
    B = len(lens)
    nb = sum(sh for _, sh, _ in spec) + sum((l + 31) // 32 for l in lens) + 4
    kc, vc = make_cache(nb, hkv, d, seed=31)
    perm = torch.randperm(nb, generator=g).tolist()
    bt = torch.zeros(B, max((l + 31) // 32 for l in lens), dtype=torch.int32)
    nxt = b = 0
    for label, sh, ls in spec:
        common = perm[nxt:nxt + sh]
        nxt += sh
        for l in ls:
            own = (l + 31) // 32 - sh
            bt[b, :sh + own] = torch.tensor(common + perm[nxt:nxt + own], dtype=torch.int32)
            nxt += own
            b += 1
    groups = ops.decode_groups(group_of, shared, G)[0].to(DEV) if grouped else None
    return B, d, kc, vc, bt, torch.tensor(lens, dtype=torch.int32), groups


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (4, 1)])
@pytest.mark.parametrize("grouped", [True, False])
@pytest.mark.parametrize("splits", [1, 8, 24])
def test_combine_o_matches_oracle(hq, hkv, grouped, splits):
    B, d, kc, vc, bt, cl, groups = _case(hq, hkv, grouped)
    N = 4096
    q = bf(B, hq, d, seed=41)
    Wo = bf(N, hq * d, scale=(hq * d) ** -0.5, seed=42)
    Ws = ops.shuffle_weight(Wo)
    res0 = bf(B, N, seed=43)
    scale = 1 / math.sqrt(d)
    G = hq // hkv
    ws = ops.DecodeWorkspace(B, hq, d, splits, DEV, max_group=16 // G if grouped else 1)
    # oracle: fp32 attention of each sequence alone, rounded to bf16 (the kernel's o operand)
    a = ref.paged_attention_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, cl, scale).to(torch.bfloat16).float()
    exp = res0.float().cpu() + a.reshape(B, -1) @ Wo.float().cpu().t()
    outs = []
    for _ in range(3):                     # the barrier and split counters re-arm every launch
        res = res0.clone()
        attention_o_resid(q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws, groups, Ws, res)
        torch.cuda.synchronize()
        outs.append(res)
    close(outs[0], exp.to(DEV).to(torch.bfloat16), 0.06, 0.03)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert int(ws.err.item()) == 0 and int(ws.sync[6:8].abs().sum()) == 0
    assert int(ws.counters.abs().sum()) == 0


def test_combine_o_equals_separate_launches():
    """Same numbers as attention (+ its separate combine launch) followed by the o GEMM, up to the
    merge order of the split partials (fp32)."""
    B, d, kc, vc, bt, cl, groups = _case(32, 8, True)
    q = bf(B, 32, d, seed=51)
    Ws = ops.shuffle_weight(bf(4096, 32 * d, scale=(32 * d) ** -0.5, seed=52))
    res0 = bf(B, 4096, seed=53)
    ws = ops.DecodeWorkspace(B, 32, d, 8, DEV, max_group=4)
    fused = res0.clone()
    attention_o_resid(q, kc, vc, bt.to(DEV), cl.to(DEV), 1 / math.sqrt(d), 8, ws, groups, Ws, fused)
    sep = res0.clone()
    attention_o_resid(q, kc, vc, bt.to(DEV), cl.to(DEV), 1 / math.sqrt(d), 8, ws, groups, Ws, sep, fused=False)
    torch.cuda.synchronize()
    close(fused, sep, 0.02, 0.01)
