"""Numerics of every HIP kernel vs the plain-PyTorch fp32 reference (ops/reference.py)."""
import math

import pytest
import torch

from theroundtaible_amd import ops
from theroundtaible_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def close(a, b, atol, rtol=0.0):
    d = (a.float() - b.float()).abs()
    tol = atol + rtol * b.float().abs()
    assert bool((d <= tol).all()), f"max err {d.max().item():.4g}"


def test_native_loaded():
    assert ops.native_available()
    assert ops.native().arch == "gfx950"


@pytest.mark.parametrize("H", [256, 768, 4096, 8192])
@pytest.mark.parametrize("rows", [1, 3, 17])
def test_rmsnorm(H, rows):
    x, w = bf(rows, H, seed=1), bf(H, seed=2)
    close(ops.rms_norm(x, w, 1e-5), ref.rms_norm(x.cpu(), w.cpu(), 1e-5).to(DEV), 0.02, 0.01)
    r = bf(rows, H, seed=3)
    exp_o, exp_r = ref.fused_add_rms_norm(x.cpu(), r.cpu(), w.cpu(), 1e-5)
    o, r2 = ops.fused_add_rms_norm(x, r, w, 1e-5)
    close(r2, exp_r.to(DEV), 0.0)
    close(o, exp_o.to(DEV), 0.02, 0.01)


@pytest.mark.parametrize("H", [128, 768])
def test_layernorm(H):
    x, w, b = bf(5, H, seed=1), bf(H, seed=2), bf(H, seed=4)
    close(ops.layer_norm(x, w, b, 1e-5), ref.layer_norm(x.cpu(), w.cpu(), b.cpu(), 1e-5).to(DEV), 0.03, 0.01)
    r = bf(5, H, seed=3)
    eo, er = ref.fused_add_layer_norm(x.cpu(), r.cpu(), w.cpu(), b.cpu(), 1e-5)
    o, r2 = ops.fused_add_layer_norm(x, r, w, b, 1e-5)
    close(r2, er.to(DEV), 0.0)
    close(o, eo.to(DEV), 0.03, 0.01)


def test_activations():
    x = bf(7, 2 * 1024, seed=5)
    close(ops.silu_and_mul(x), ref.silu_and_mul(x.cpu()).to(DEV), 0.02, 0.01)
    close(ops.gelu_tanh(x), ref.gelu_tanh(x.cpu()).to(DEV), 0.02, 0.01)


def make_cache(nb, hkv, d, seed=0):
    kc = bf(nb, hkv, 32, d, seed=seed)
    vc = bf(nb, hkv, d, 32, seed=seed + 1)
    return kc, vc


@pytest.mark.parametrize("hq,hkv,d,rope", [(32, 8, 128, True), (12, 12, 64, False), (8, 1, 128, True)])
def test_rope_and_cache(hq, hkv, d, rope):
    T, nb = 37, 16
    qkv = bf(T, (hq + 2 * hkv) * d, seed=7)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    perm = torch.randperm(nb * 32, device=DEV)[:T]
    cs = ref.rope_cos_sin(4096, d, 500000.0, DEV) if rope else None
    kc, vc = make_cache(nb, hkv, d)
    kc2, vc2 = kc.cpu().clone(), vc.cpu().clone()
    q = ops.rope_and_cache(qkv, pos, cs, kc, vc, perm, hq, hkv, d)
    qr = ref.rope_and_cache(qkv.cpu(), pos.cpu(), cs.cpu() if cs is not None else None, kc2, vc2, perm.cpu(),
                            hq, hkv, d)
    close(q, qr.to(DEV), 0.02, 0.01)
    close(kc, kc2.to(DEV), 0.02, 0.01)
    close(vc, vc2.to(DEV), 0.0)


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (64, 8, 128), (12, 12, 64), (8, 2, 128), (4, 1, 128),
                                      (8, 1, 128), (28, 4, 128), (14, 2, 64), (24, 8, 128)])
@pytest.mark.parametrize("splits", [1, 3, 8, 64])
def test_paged_decode(hq, hkv, d, splits):
    lens = [1, 31, 32, 33, 257, 1500]
    B = len(lens)
    nb = sum((l + 31) // 32 for l in lens) + 4
    kc, vc = make_cache(nb, hkv, d, seed=11)
    perm = torch.randperm(nb).tolist()
    maxb = max((l + 31) // 32 for l in lens)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    i = 0
    for b, l in enumerate(lens):
        n = (l + 31) // 32
        bt[b, :n] = torch.tensor(perm[i:i + n], dtype=torch.int32)
        i += n
    q = bf(B, hq, d, seed=12)
    cl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(d)
    ws = ops.DecodeWorkspace(B, hq, d, splits, DEV)
    out = ops.paged_attention_decode(q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws)
    exp = ref.paged_attention_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, cl, scale)
    close(out, exp.to(DEV), 0.02, 0.02)
    # the in-kernel split combine re-arms its arrival counters: a second launch on the same
    # workspace must reproduce the first bit for bit
    out2 = ops.paged_attention_decode(q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws)
    assert torch.equal(out, out2)
    assert int(ws.counters.abs().sum()) == 0
    _check_planned(out, q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws, hq, hkv)


def _check_planned(out, q, kc, vc, bt, cl, scale, splits, ws, hq, hkv, groups=None):
    """The per-step work plan (ops.attn_plan, csrc/attention_decode.hip attn_plan_kernel) must give
    the same bits as the launch that derives its own ranges (same partials, same merge order)."""
    assert ops.attn_plan(bt, cl, splits, ws, hq, hkv, groups, q.shape[0])
    planned = ops.paged_attention_decode(q, kc, vc, bt, cl, scale, splits, ws, groups=groups, planned=True)
    assert torch.equal(out, planned)
    assert int(ws.counters.abs().sum()) == 0


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (64, 8, 128), (8, 2, 128), (12, 12, 64), (4, 1, 128),
                                      (28, 4, 128), (24, 8, 128)])
@pytest.mark.parametrize("splits", [1, 3, 10, 64])
@pytest.mark.parametrize("layout", ["table3", "mixed"])
def test_paged_decode_shared_prefix_groups(hq, hkv, d, splits, layout):
    """Knights sharing a KV prefix (same leading block ids) decode it once per group: the
    grouped kernel must equal the fp32 oracle of each sequence alone, for groups of 1..4, a
    shared prefix longer / shorter than the private tails, and groups wider than 16 columns
    (cut into sub-groups)."""
    G = hq // hkv
    if layout == "table3":      # one table: 3 knights, 1900-token shared prefix + private tails
        spec = [("A", 1900 // 32, [1900 + 7, 1900 + 300, 1900 + 33])]
    else:                        # two groups of different size + a lone sequence
        spec = [("A", 40, [40 * 32 + 1, 40 * 32 + 500]), (None, 0, [700]), ("B", 3, [3 * 32 + 5, 96 + 64, 96 + 1, 96 + 900])]
    g = torch.Generator().manual_seed(5)
    lens, group_of, shared = [], [], []
    for label, sh, ls in spec:
        for l in ls:
            lens.append(l)
            group_of.append(label)
            shared.append(sh)
    B = len(lens)
    nb = sum(sh for _, sh, _ in spec) + sum((l + 31) // 32 for l in lens) + 4
    kc, vc = make_cache(nb, hkv, d, seed=21)
    perm = torch.randperm(nb, generator=g).tolist()
    maxb = max((l + 31) // 32 for l in lens)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    nxt = 0
    b = 0
    for label, sh, ls in spec:
        common = perm[nxt:nxt + sh]
        nxt += sh
        for l in ls:
            own = (l + 31) // 32 - sh
            bt[b, :sh + own] = torch.tensor(common + perm[nxt:nxt + own], dtype=torch.int32)
            nxt += own
            b += 1
    groups, nmax = ops.decode_groups(group_of, shared, G)
    assert nmax <= max(1, 16 // G)
    q = bf(B, hq, d, seed=22)
    cl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(d)
    ws = ops.DecodeWorkspace(B, hq, d, splits, DEV, max_group=16 // G)
    out = ops.paged_attention_decode(q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws, groups=groups.to(DEV))
    exp = ref.paged_attention_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, cl, scale)
    close(out, exp.to(DEV), 0.02, 0.02)
    out2 = ops.paged_attention_decode(q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws, groups=groups.to(DEV))
    assert torch.equal(out, out2)
    assert int(ws.counters.abs().sum()) == 0
    _check_planned(out, q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws, hq, hkv, groups.to(DEV))


@pytest.mark.parametrize("splits", [1, 2, 5])
def test_paged_decode_long_context(splits):
    """Contexts of 20K / 33K keys: at splits=1 a wave walks > 64 tiles, exercising the per-lane
    block-id refill; block tables are a random permutation over the whole pool."""
    hq, hkv, d = 32, 8, 128
    lens = [20000, 33000, 40]
    B = len(lens)
    nb = sum((l + 31) // 32 for l in lens) + 2
    kc, vc = make_cache(nb, hkv, d, seed=21)
    perm = torch.randperm(nb, generator=torch.Generator().manual_seed(5)).tolist()
    maxb = max((l + 31) // 32 for l in lens)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    i = 0
    for b, l in enumerate(lens):
        n = (l + 31) // 32
        bt[b, :n] = torch.tensor(perm[i:i + n], dtype=torch.int32)
        i += n
    q = bf(B, hq, d, seed=22)
    cl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(d)
    ws = ops.DecodeWorkspace(B, hq, d, splits, DEV)
    out = ops.paged_attention_decode(q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws)
    exp = ref.paged_attention_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, cl, scale)
    close(out, exp.to(DEV), 0.02, 0.02)
    # planned: items longer than the plan row (512 tiles) read the rest from the block tables
    _check_planned(out, q, kc, vc, bt.to(DEV), cl.to(DEV), scale, splits, ws, hq, hkv)


def test_paged_decode_spike():
    """Force the online-softmax rescale path: a key that dominates late in the sequence."""
    hq, hkv, d, L = 32, 8, 128, 700
    nb = 32
    kc, vc = make_cache(nb, hkv, d, seed=3)
    q = bf(1, hq, d, seed=4)
    # make key 650 align strongly with every query of kv head 0
    blk, off = 650 // 32, 650 % 32
    ref.set_k_row(kc, blk, 0, off, (q[0, :4].float().mean(0) * 8).to(torch.bfloat16))
    bt = torch.arange(nb, dtype=torch.int32)[None]
    cl = torch.tensor([L], dtype=torch.int32)
    for splits in (1, 4):
        out = ops.paged_attention_decode(q, kc, vc, bt.to(DEV), cl.to(DEV), 1 / math.sqrt(d), splits)
        exp = ref.paged_attention_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, cl, 1 / math.sqrt(d))
        close(out, exp.to(DEV), 0.03, 0.02)


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (64, 8, 128), (12, 12, 64), (8, 4, 128), (16, 1, 128),
                                      (28, 4, 128), (14, 2, 64), (12, 4, 128), (12, 1, 64)])
def test_prefill_varlen(hq, hkv, d):
    """Includes GQA groups that are not powers of two (Qwen2.5: G = 7; Llama-3.2-3B: G = 3; 12):
    D = 128 groups up to 8 run the 32x32 kernel in the next power of two of head slots, the others
    the 16x16 kernel; surplus head slots stay idle in both."""
    # (start_pos, new tokens): prefix already cached + delta chunk
    specs = [(0, 1), (0, 45), (100, 70), (31, 33), (500, 17)]
    S = len(specs)
    nb_each = [(sp + n + 31) // 32 for sp, n in specs]
    nb = sum(nb_each) + 2
    kc, vc = make_cache(nb, hkv, d, seed=21)
    perm = torch.randperm(nb).tolist()
    maxb = max(nb_each)
    bt = torch.zeros(S, maxb, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb_each):
        bt[s, :n] = torch.tensor(perm[i:i + n], dtype=torch.int32)
        i += n
    cu = [0]
    for _, n in specs:
        cu.append(cu[-1] + n)
    cu_t = torch.tensor(cu, dtype=torch.int32)
    st = torch.tensor([sp for sp, _ in specs], dtype=torch.int32)
    q = bf(cu[-1], hq, d, seed=22)
    scale = 1 / math.sqrt(d)
    out = ops.prefill_attention(q, kc, vc, bt.to(DEV), cu_t.to(DEV), st.to(DEV), scale)
    exp = ref.prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), bt, cu_t, st, scale)
    close(out, exp.to(DEV), 0.02, 0.02)


def test_prefill_long_prefix():
    """Delta chunks over long paged prefixes (30K / 12K keys) mixed with a fresh sequence."""
    hq, hkv, d = 32, 8, 128
    specs = [(30000, 200), (0, 300), (12345, 129)]
    S = len(specs)
    nb_each = [(sp + n + 31) // 32 for sp, n in specs]
    nb = sum(nb_each) + 2
    kc, vc = make_cache(nb, hkv, d, seed=41)
    perm = torch.randperm(nb, generator=torch.Generator().manual_seed(6)).tolist()
    bt = torch.zeros(S, max(nb_each), dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb_each):
        bt[s, :n] = torch.tensor(perm[i:i + n], dtype=torch.int32)
        i += n
    cu = [0]
    for _, n in specs:
        cu.append(cu[-1] + n)
    cu_t = torch.tensor(cu, dtype=torch.int32)
    st = torch.tensor([sp for sp, _ in specs], dtype=torch.int32)
    q = bf(cu[-1], hq, d, seed=42)
    scale = 1 / math.sqrt(d)
    out = ops.prefill_attention(q, kc, vc, bt.to(DEV), cu_t.to(DEV), st.to(DEV), scale)
    exp = ref.prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), bt, cu_t, st, scale)
    close(out, exp.to(DEV), 0.02, 0.02)


@pytest.mark.parametrize("hq,hkv", [(4, 1), (8, 2), (8, 1), (32, 8), (28, 4), (12, 4)])
@pytest.mark.parametrize("min_chunk", [1, 3, 8])
def test_prefill_key_split(hq, hkv, min_chunk):
    """Key-split prefill (tensor-parallel shard head counts: few tiles x KV heads): work items
    over key-tile ranges leave unnormalised partials merged by the combine launch
    (attention_prefill32.hip); long tiles cut into 2..many parts, short ones whole, a fresh
    sequence (causal diagonal inside a part) and delta chunks over long prefixes — vs the fp32
    oracle and vs the whole-tile kernel."""
    d = 128
    specs = [(9000, 300), (0, 257), (2345, 129), (31, 1)]
    S = len(specs)
    nb_each = [(sp + n + 31) // 32 for sp, n in specs]
    nb = sum(nb_each) + 2
    kc, vc = make_cache(nb, hkv, d, seed=51)
    perm = torch.randperm(nb, generator=torch.Generator().manual_seed(7)).tolist()
    bt = torch.zeros(S, max(nb_each), dtype=torch.int32)
    i = 0
    for s, n in enumerate(nb_each):
        bt[s, :n] = torch.tensor(perm[i:i + n], dtype=torch.int32)
        i += n
    cu = [0]
    for _, n in specs:
        cu.append(cu[-1] + n)
    cu_t = torch.tensor(cu, dtype=torch.int32)
    st = torch.tensor([sp for sp, _ in specs], dtype=torch.int32)
    q = bf(cu[-1], hq, d, seed=52)
    scale = 1 / math.sqrt(d)
    rows = ops.native().prefill_rows_per_tile(hq // hkv, d)
    plan = ops.prefill_split_plan(cu_t, rows, st, hkv, num_cus=1 << 20, min_chunk_tiles=min_chunk)
    assert plan is not None and plan[2] >= 2
    split = (plan[0].to(DEV), plan[1].to(DEV), plan[2])
    out = ops.prefill_attention(q, kc, vc, bt.to(DEV), cu_t.to(DEV), st.to(DEV), scale, split=split)
    whole = ops.prefill_attention(q, kc, vc, bt.to(DEV), cu_t.to(DEV), st.to(DEV), scale)
    exp = ref.prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), bt, cu_t, st, scale)
    close(out, exp.to(DEV), 0.02, 0.02)
    close(out, whole, 0.02, 0.02)
    again = ops.prefill_attention(q, kc, vc, bt.to(DEV), cu_t.to(DEV), st.to(DEV), scale, split=split)
    assert torch.equal(out, again)


def test_sample_greedy_and_topk1():
    B, V = 5, 128256
    # fp32 logits: bf16 random rows contain exact ties at the max, where top-k=1 legitimately
    # keeps both tied tokens (threshold semantics) while argmax picks the lowest index.
    logits = bf(B, V, scale=3.0, seed=31).float() + torch.arange(V, device=DEV).float() * 1e-6
    z = torch.zeros(B, device=DEV)
    one = torch.ones(B, device=DEV)
    k0 = torch.zeros(B, dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV)
    offs = torch.arange(B, dtype=torch.int64, device=DEV) + 7
    am = logits.float().argmax(-1)
    assert torch.equal(ops.sample(logits, z, one, k0, seeds, offs), am)
    k1 = torch.ones(B, dtype=torch.int32, device=DEV)
    assert torch.equal(ops.sample(logits, one * 0.8, one, k1, seeds, offs), am)


def test_sample_matches_reference():
    B, V = 8, 32000
    logits = bf(B, V, scale=2.0, seed=41).float()
    temp = torch.full((B,), 0.7, device=DEV)
    top_p = torch.tensor([1.0, 0.9, 0.5, 0.95, 1.0, 0.8, 0.99, 0.3], device=DEV)
    top_k = torch.tensor([0, 0, 0, 50, 10, 0, 1000, 0], dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 1000 + 1
    offs = torch.arange(B, dtype=torch.int64, device=DEV) + 123
    got = ops.sample(logits, temp, top_p, top_k, seeds, offs).cpu()
    exp = ref.sample(logits.cpu(), temp.cpu(), top_p.cpu(), top_k.cpu(), seeds.cpu(), offs.cpu())
    assert (got == exp).sum() >= B - 1, (got, exp)
    # determinism
    again = ops.sample(logits, temp, top_p, top_k, seeds, offs).cpu()
    assert torch.equal(got, again)


def test_sample_fast_path_matches_reference():
    """Accept pass (csrc/sampling.hip launch 2): the whole-vocabulary Gumbel argmax is taken
    when it lies in the nucleus, the histogram path decides otherwise; both must agree with the
    fp64 reference over many draws (Llama-3 vocabulary, peaked and flat rows)."""
    B, V = 16, 128256
    logits = bf(B, V, scale=3.0, seed=77).float()
    logits[::2] *= 3.0          # peaked rows: small nuclei, frequent fallbacks
    temp = torch.full((B,), 0.7, device=DEV)
    top_p = torch.full((B,), 0.9, device=DEV)
    top_k = torch.zeros(B, dtype=torch.int32, device=DEV)
    hits = total = 0
    for rep in range(4):
        seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 7919 + rep
        offs = torch.arange(B, dtype=torch.int64, device=DEV) + 1000 * rep
        got = ops.sample(logits, temp, top_p, top_k, seeds, offs).cpu()
        exp = ref.sample(logits.cpu(), temp.cpu(), top_p.cpu(), top_k.cpu(), seeds.cpu(), offs.cpu())
        hits += int((got == exp).sum())
        total += B
    assert hits >= total - 2, (hits, total)


def test_sample_rejection_paths_match_reference():
    """Low top-p (most whole-vocabulary draws rejected: the histogram-resolved nucleus, the
    candidate test and the threshold search all run) and near-flat rows (random-init models: the
    histogram grid scale adapts after the first call on a persistent workspace) agree with the
    fp64 reference draw for draw."""
    B, V = 8, 128256
    logits = bf(B, V, scale=2.0, seed=91).float()
    logits[1::2] *= 0.05
    temp = torch.full((B,), 0.8, device=DEV)
    top_p = torch.tensor([0.3, 0.3, 0.5, 0.5, 0.95, 0.95, 0.99, 0.7], device=DEV)
    top_k = torch.zeros(B, dtype=torch.int32, device=DEV)
    ws = ops.sample_workspace(B, DEV)
    hits = total = 0
    for rep in range(6):
        seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 104729 + rep
        offs = torch.arange(B, dtype=torch.int64, device=DEV) + 777 * rep
        got = ops.sample(logits, temp, top_p, top_k, seeds, offs, ws=ws).cpu()
        exp = ref.sample(logits.cpu(), temp.cpu(), top_p.cpu(), top_k.cpu(), seeds.cpu(), offs.cpu())
        hits += int((got == exp).sum())
        total += B
    assert hits >= total - 2, (hits, total)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_sample_topk_lists_match_reference(dtype):
    """Top-k rows with k <= 64 (csrc/sampling.hip: every chunk publishes its own top k, the
    decider merges the lists — no pass over the row), alone and with top-p inside the top-k set,
    on bf16 (16-bit order keys) and fp32 logits; a tie-heavy row (quantised logits: chunks drop
    ties at the cut, so the histogram path decides) and a near-flat row. Draw for draw against
    the fp64 reference."""
    B, V = 8, 128256
    B = 11
    logits = bf(B, V, scale=2.0, seed=123).float()
    logits[1] *= 0.05
    logits[2] = torch.round(logits[2] * 2) / 2
    # rows whose whole top k is NEGATIVE (log-prob-like inputs), with many exact ties at the
    # chunks' k-th value: a negative value's order key must compare EQUAL to a tie at the cut,
    # not above it (advisor r4: the 'above' list then overflowed its LDS slots)
    logits[8] = torch.round(logits[8] * 4) / 4 - 20.0
    logits[9] = torch.round(logits[9]) - 9.0
    logits[10] = torch.round(logits[10] * 8) / 8 - 3.0
    logits = logits.to(dtype)
    temp = torch.full((B,), 0.8, device=DEV)
    top_k = torch.tensor([1, 5, 40, 64, 40, 64, 2, 17, 40, 64, 9], dtype=torch.int32, device=DEV)
    top_p = torch.tensor([1.0, 1.0, 1.0, 0.9, 0.5, 1.0, 0.7, 0.95, 1.0, 0.9, 1.0], device=DEV)
    ws = ops.sample_workspace(B, DEV)
    hits = total = 0
    for rep in range(6):
        seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 7907 + rep
        offs = torch.arange(B, dtype=torch.int64, device=DEV) + 333 * rep
        got = ops.sample(logits, temp, top_p, top_k, seeds, offs, ws=ws).cpu()
        exp = ref.sample(logits.cpu(), temp.cpu(), top_p.cpu(), top_k.cpu(), seeds.cpu(), offs.cpu())
        hits += int((got == exp).sum())
        total += B
        assert torch.equal(got, ops.sample(logits, temp, top_p, top_k, seeds, offs, ws=ws).cpu())
    assert hits >= total - 2, (hits, total)


def test_sample_top_p_nucleus():
    V = 1000
    logits = torch.full((1, V), -10.0, device=DEV)
    logits[0, :3] = torch.tensor([5.0, 4.9, 4.8], device=DEV)
    hits = set()
    for s in range(64):
        tok = ops.sample(logits, torch.ones(1, device=DEV), torch.tensor([0.5], device=DEV),
                         torch.zeros(1, dtype=torch.int32, device=DEV), torch.tensor([s], device=DEV),
                         torch.tensor([s], device=DEV))
        hits.add(int(tok))
    assert hits <= {0, 1} and len(hits) == 2



@pytest.mark.parametrize("mode", ["greedy", "top_p", "top_k"])
def test_sample_advance_equals_sample_then_advance(mode):
    """The captured step's fused K6 + bookkeeping launch (csrc/sampling.hip sample_advance) equals
    sample -> decode_advance(prep) run separately, bit for bit, over several chained steps on ONE
    persistent workspace (its tickets re-arm: no memset between replays)."""
    B, V, H, bs, maxb = 5, 128256, 256, 32, 8
    g = torch.Generator(device=DEV).manual_seed(3)
    embed = (torch.randn(V, H, generator=g, device=DEV)).to(torch.bfloat16)
    bt = torch.randperm(64, device=DEV)[:B * maxb].to(torch.int32).reshape(B, maxb)
    temp = torch.full((B,), 0.0 if mode == "greedy" else 0.8, device=DEV)
    top_p = torch.full((B,), 0.9 if mode == "top_p" else 1.0, device=DEV)
    top_k = torch.full((B,), 40 if mode == "top_k" else 0, dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 31 + 5

    def state():
        pos = torch.tensor([3, 40, 77, 100, 31], dtype=torch.int64, device=DEV)
        return dict(out=torch.zeros(16, B, dtype=torch.int64, device=DEV), ids=torch.zeros(B, dtype=torch.int64, device=DEV),
                    pos=pos, ctx=(pos + 1).to(torch.int32), step=torch.zeros(1, dtype=torch.int64, device=DEV),
                    slots=torch.zeros(B, dtype=torch.int64, device=DEV), offs=pos + 1,
                    res=torch.zeros(B, H, dtype=torch.bfloat16, device=DEV))
    a, r = state(), state()
    ws = ops.sample_workspace(B, DEV)
    nxt = torch.zeros(B, dtype=torch.int64, device=DEV)
    for step in range(4):
        logits = bf(B, V, scale=3.0, seed=100 + step)
        ops.sample_advance(logits, temp, top_p, top_k, seeds, a["offs"], ws, nxt, a["out"], a["ids"], a["pos"],
                           a["ctx"], a["step"], a["slots"], a["res"], bt, embed, bs)
        t = ops.sample(logits, temp, top_p, top_k, seeds, r["offs"])
        ops.decode_advance(r["out"], r["ids"], r["pos"], r["ctx"], r["step"], t,
                           prep=(r["slots"], r["offs"], r["res"], bt, embed, bs))
        assert torch.equal(nxt, t), (step, nxt, t)
    for k in a:
        assert torch.equal(a[k], r[k]), k
    assert int(a["step"]) == 4
    wsi = ws.view(torch.int32)
    assert int(wsi[-4]) == 0                                       # rows-done ticket re-armed
    row = (ws.numel() - 4) // B
    assert all(int(wsi[b * row + 5 * 32]) == 0 for b in range(B))   # row tickets (W_CNT) re-armed


def test_paging_guard_matches_reference():
    g = torch.Generator().manual_seed(3)
    for trial in range(40):
        B, maxb, nb, bs = 3, 6, 16, 32
        bt = torch.randint(0, nb, (B, maxb), generator=g, dtype=torch.int32)
        ctx = torch.randint(1, maxb * bs + 1, (B,), generator=g, dtype=torch.int32)
        pos = (ctx - 1).to(torch.int64)
        slots = torch.tensor([int(bt[b, int(p) // bs]) * bs + int(p) % bs for b, p in enumerate(pos)])
        kind = trial % 5
        if kind == 1:
            bt[trial % B, 0] = nb + trial            # out of the pool
        elif kind == 2:
            slots[trial % B] += 1                    # wrong write slot
        elif kind == 3:
            ctx[trial % B] = maxb * bs + 5           # beyond the table
        elif kind == 4:
            pos[trial % B] += 2                      # position / length mismatch
        want = torch.zeros(1, dtype=torch.int32)
        ref.paging_guard(bt, ctx, pos, slots, want, nb, bs)
        got = torch.zeros(1, dtype=torch.int32, device=DEV)
        ops.paging_guard(bt.to(DEV), ctx.to(DEV), pos.to(DEV), slots.to(DEV), got, nb, bs)
        assert int(got.item()) == int(want[0]), (trial, kind)
        assert (kind == 0) == (int(want[0]) == 0)


def test_decode_prep_and_fused_advance_match_reference():
    """csrc/decode_step.hip: decode_prep and decode_advance (plain and with the fused next-step
    prep) against the PyTorch semantics in ops/reference.py, including a row whose advanced
    position runs past its block table."""
    torch.manual_seed(3)
    B, maxb, bs, H, V = 5, 4, 32, 4096, 1000
    bt = torch.randint(0, 50, (B, maxb), dtype=torch.int32)
    pos = torch.tensor([0, 31, 64, 100, maxb * bs - 1])
    ids = torch.tensor([1, 999, 5, 1200, -3])
    emb = torch.randn(V, H).bfloat16()
    out = torch.zeros(8, B, dtype=torch.int64)
    ctx = (pos + 1).to(torch.int32)
    step = torch.zeros(1, dtype=torch.int64)
    nxt = torch.tensor([7, 8, 9, 10, 11])
    st_ref = [t.clone() for t in (out, ids, pos, ctx, step)]
    st_gpu = [t.cuda() for t in (out, ids, pos, ctx, step)]
    bufs_ref = [torch.zeros(B, dtype=torch.int64), torch.zeros(B, dtype=torch.int64), torch.zeros(B, H).bfloat16()]
    bufs_gpu = [t.cuda() for t in bufs_ref]
    ref.decode_prep(*bufs_ref, st_ref[1], st_ref[2], bt, emb, bs)
    ops.decode_prep(*bufs_gpu, st_gpu[1], st_gpu[2], bt.cuda(), emb.cuda(), bs)
    for a, b in zip(bufs_ref, bufs_gpu):
        assert torch.equal(a, b.cpu())
    ref.decode_advance(*st_ref, nxt, prep=(*bufs_ref, bt, emb, bs))
    ops.decode_advance(*st_gpu, nxt.cuda(), prep=(*bufs_gpu, bt.cuda(), emb.cuda(), bs))
    ref.decode_advance(*st_ref, nxt + 1)
    ops.decode_advance(*st_gpu, nxt.cuda() + 1)
    torch.cuda.synchronize()
    for a, b in zip(st_ref + bufs_ref, st_gpu + bufs_gpu):
        assert torch.equal(a, b.cpu())
    assert bufs_ref[0][4].item() == (maxb * bs) % bs   # past the table: block 0
