"""Decode GEMM (csrc/gemm_skinny.hip): shuffled weights + fused norm / residual / SwiGLU vs fp32 reference."""
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


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("N,K", [(256, 512), (4096, 4096), (1024, 14336), (48, 96), (65536, 512)])
def test_skinny_gemm_modes(M, N, K):
    # weight orders (skinny_core.h weight_order): (1024, 14336) k-major, (65536, 512) k-chunks of
    # 16 (lm_head rule), SwiGLU chunks of 16 where K allows, the rest tile-major
    x = bf(M, K, seed=51)
    W = bf(N, K, scale=0.05, seed=52)
    gam = bf(K, seed=53)
    Ws = ops.shuffle_weight(W)
    close(ops.skinny_gemm(x, Ws), ref.skinny_gemm(x.cpu(), W.cpu()).to(DEV), 0.05, 0.02)
    # RMSNorm prologue with gamma folded into the weights
    Wg = ops.shuffle_weight(W, gam)
    Wf = ref.fold_gamma(W.cpu(), gam.cpu())
    close(ops.skinny_gemm(x, Wg, ops.PRO_NORM, eps=1e-5), ref.skinny_gemm(x.cpu(), Wf, 1, eps=1e-5).to(DEV), 0.05, 0.02)
    # residual epilogue, in place
    res = bf(M, N, seed=54)
    res_ref = res.cpu().clone()
    ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res)
    ref.skinny_gemm(x.cpu(), W.cpu(), 0, 1, res=res_ref)
    close(res, res_ref.to(DEV), 0.06, 0.02)
    # SwiGLU epilogue over [gate; up]
    W2 = bf(2 * N, K, scale=0.05, seed=55)
    got = ops.skinny_gemm(x, ops.shuffle_weight(W2, gam, swiglu=True), ops.PRO_NORM, ops.EPI_SWIGLU)
    exp = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W2.cpu(), gam.cpu()), 1, 2)
    close(got, exp.to(DEV), 0.05, 0.03)


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("N,K", [(14336, 4096), (300 * 16, 1024), (257 * 16, 2048)])
def test_skinny_gemm_balanced_split(M, N, K):
    """CU-balanced launch (tiles mod CUs run as two K-halves): same results as the fp32
    reference on every epilogue, and the workspace counters re-arm (three calls agree)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert (N // 16) % cus != 0
    x = bf(M, K, seed=61)
    gam = bf(K, seed=62)
    ws = ops.split_workspace(DEV)
    W2 = bf(2 * N, K, scale=0.05, seed=63)
    Ws2 = ops.shuffle_weight(W2, gam, swiglu=True)
    exp = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W2.cpu(), gam.cpu()), 1, 2).to(DEV)
    outs = [ops.skinny_gemm(x, Ws2, ops.PRO_NORM, ops.EPI_SWIGLU, split_ws=ws) for _ in range(3)]
    for o in outs:
        close(o, exp, 0.05, 0.03)
        assert torch.equal(o, outs[0])
    assert int(ws[:256].abs().sum()) == 0, "split counters must re-arm to zero"
    W = bf(N, K, scale=0.05, seed=64)
    Wg = ops.shuffle_weight(W, gam)
    close(ops.skinny_gemm(x, Wg, ops.PRO_NORM, split_ws=ws),
          ref.skinny_gemm(x.cpu(), ref.fold_gamma(W.cpu(), gam.cpu()), 1, eps=1e-5).to(DEV), 0.05, 0.02)
    Ws = ops.shuffle_weight(W)
    res = bf(M, N, seed=65)
    res_ref = res.cpu().clone()
    ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res, split_ws=ws)
    ref.skinny_gemm(x.cpu(), W.cpu(), 0, 1, res=res_ref)
    close(res, res_ref.to(DEV), 0.06, 0.02)
    # no workspace: the plain launch gives the same SwiGLU output up to summation order
    close(ops.skinny_gemm(x, Ws2, ops.PRO_NORM, ops.EPI_SWIGLU), outs[0], 0.02, 0.02)


@pytest.mark.parametrize("M", [5, 8, 12, 16, 20, 32])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 14336), (128256, 4096), (6144, 4096)])
def test_skinny_gemm_serving_batch_multi_tile(M, N, K):
    """Serving batches (M > 4): several tiles per workgroup share each activation fragment
    (skinny_core.h gemm_tiles) — o / down (256 tiles, M > 8) as two tiles over two K halves with
    the split hand-off, qkv-sized (384 tiles) two tiles, lm_head-sized four. Against the fp32 oracle
    on the norm / residual / SwiGLU epilogues, deterministic over repeats, counters re-armed;
    the same GEMMs with the multi-tile launches off (RT_SKINNY_TN=1 is read once per process, so
    the one-tile launch is checked through M = 3 rows of the same operands instead). 17..32 rows
    run as two 16-row blocks per MFMA pass (one weight stream for both)."""
    x = bf(M, K, seed=71)
    gam = bf(K, seed=72)
    ws = ops.split_workspace(DEV)
    W = bf(N, K, scale=0.05, seed=73)
    Wg = ops.shuffle_weight(W, gam)
    exp = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W.cpu(), gam.cpu()), 1, eps=1e-5).to(DEV)
    outs = [ops.skinny_gemm(x, Wg, ops.PRO_NORM, split_ws=ws) for _ in range(3)]
    for o in outs:
        close(o, exp, 0.05, 0.02)
        assert torch.equal(o, outs[0])
    assert int(ws[:256].abs().sum()) == 0, "split counters must re-arm to zero"
    # the first 3 rows through the M <= 4 one-tile launch: same values up to summation order
    close(ops.skinny_gemm(x[:3].contiguous(), Wg, ops.PRO_NORM, split_ws=ws), outs[0][:3], 0.02, 0.02)
    Ws = ops.shuffle_weight(W)
    res = bf(M, N, seed=74)
    res_ref = res.cpu().clone()
    ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res, split_ws=ws)
    ref.skinny_gemm(x.cpu(), W.cpu(), 0, 1, res=res_ref)
    close(res, res_ref.to(DEV), 0.06, 0.02)
    if N <= 14336:
        W2 = bf(2 * N, K, scale=0.05, seed=75)
        got = ops.skinny_gemm(x, ops.shuffle_weight(W2, gam, swiglu=True), ops.PRO_NORM, ops.EPI_SWIGLU, split_ws=ws)
        close(got, ref.skinny_gemm(x.cpu(), ref.fold_gamma(W2.cpu(), gam.cpu()), 1, 2).to(DEV), 0.05, 0.03)
    assert int(ws[:256].abs().sum()) == 0


@pytest.mark.parametrize("M", [12, 20])
@pytest.mark.parametrize("N", [4112, 6160, 12304])
def test_skinny_gemm_serving_batch_odd_tile_counts(M, N):
    """Tile counts that do not divide by the tiles per workgroup: 257 tiles on the two-K-half path
    (a last group with one real tile), 385 on two tiles, 769 on four — the past-the-end tile of a
    workgroup is computed on a clamped copy and never stored (skinny_core.h gemm_tiles)."""
    K = 4096
    x = bf(M, K, seed=81)
    W = bf(N, K, scale=0.05, seed=82)
    ws = ops.split_workspace(DEV)
    Ws = ops.shuffle_weight(W)
    res = bf(M, N, seed=83)
    res_ref = res.cpu().clone()
    ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res, split_ws=ws)
    ref.skinny_gemm(x.cpu(), W.cpu(), 0, 1, res=res_ref)
    close(res, res_ref.to(DEV), 0.06, 0.02)
    got = ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, split_ws=ws)
    close(got, ref.skinny_gemm(x.cpu(), W.cpu(), 0).to(DEV), 0.05, 0.02)
    assert int(ws[:256].abs().sum()) == 0


def test_shuffle_layout():
    N, K = 32, 64
    W = torch.arange(N * K, device=DEV).reshape(N, K).to(torch.float32).to(torch.bfloat16)
    Ws = ops.shuffle_weight(W).reshape(N // 16, K // 32, 64, 8)
    t, s, l = 1, 1, 37
    expect = W[16 * t + (l & 15), 32 * s + 8 * (l >> 4): 32 * s + 8 * (l >> 4) + 8]
    assert torch.equal(Ws[t, s, l], expect)


def test_fused_decode_matches_unfused():
    from theroundtaible_amd.engine import Engine, EngineConfig
    from theroundtaible_amd.models.llama import AttnMeta
    e = Engine(EngineConfig(model="tiny-llama-128", weights="random-full:5", device=DEV, num_blocks=64,
                            use_graphs=False))
    ids = e.encode_prompt("fused versus unfused decode " * 4)
    seqs = [e.kv.seq("a"), e.kv.seq("b")]
    e.prefill([(seqs[0], ids), (seqs[1], ids[:-3])])
    for s in seqs:
        e.kv.ensure_capacity(s, s.length + 1)
    pos = torch.tensor([s.length for s in seqs], device=DEV)
    slots = torch.tensor([s.blocks[p // 32] * 32 + p % 32 for s, p in zip(seqs, pos.tolist())], device=DEV)
    bt = torch.zeros(2, 8, dtype=torch.int32)
    for j, s in enumerate(seqs):
        bt[j, :len(s.blocks)] = torch.tensor(s.blocks)
    meta = AttnMeta("decode", slots, bt.to(DEV), (pos + 1).to(torch.int32), num_splits=4)
    tok = torch.tensor([5, 7], device=DEV)
    fused = e.model.forward(tok, pos, e.kv, meta).float()
    e.model.use_fused = False
    plain = e.model.forward(tok, pos, e.kv, meta).float()
    cos = torch.nn.functional.cosine_similarity(fused, plain, dim=-1)
    assert float(cos.min()) > 0.999


@pytest.mark.parametrize("B", [12, 24, 32])
def test_fused_decode_matches_unfused_serving_batch(B):
    """Serving batches up to 32 rows take the fused decode path at tp 1 (two 16-row blocks in the
    skinny GEMMs above 16 rows): logits agree with the unfused hipBLASLt path."""
    from theroundtaible_amd.engine import Engine, EngineConfig
    from theroundtaible_amd.models.llama import AttnMeta
    e = Engine(EngineConfig(model="tiny-llama-128", weights="random-full:5", device=DEV, num_blocks=256,
                            use_graphs=False))
    base = e.encode_prompt("serving batch decode " * 3)
    seqs = [e.kv.seq(f"s{i}") for i in range(B)]
    e.prefill([(s, base[: len(base) - (i % 5)]) for i, s in enumerate(seqs)])
    for s in seqs:
        e.kv.ensure_capacity(s, s.length + 1)
    pos = torch.tensor([s.length for s in seqs], device=DEV)
    slots = torch.tensor([s.blocks[p // 32] * 32 + p % 32 for s, p in zip(seqs, pos.tolist())], device=DEV)
    bt = torch.zeros(B, 8, dtype=torch.int32)
    for j, s in enumerate(seqs):
        bt[j, :len(s.blocks)] = torch.tensor(s.blocks)
    meta = AttnMeta("decode", slots, bt.to(DEV), (pos + 1).to(torch.int32), num_splits=1)
    tok = torch.arange(B, device=DEV) * 7 + 3
    assert e.model.fused_decode_ok(tok)
    fused = e.model.forward(tok, pos, e.kv, meta).float()
    e.model.use_fused = False
    plain = e.model.forward(tok, pos, e.kv, meta).float()
    cos = torch.nn.functional.cosine_similarity(fused, plain, dim=-1)
    assert float(cos.min()) > 0.999, cos


def test_fused_decode_is_deterministic():
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    sp = SamplingParams(temperature=0.0, max_new_tokens=32, ignore_eos=True, stop_on_consensus=False)
    outs = []
    for _ in range(2):
        e = Engine(EngineConfig(model="tiny-llama-128", weights="random:5", device=DEV, num_blocks=64))
        outs.append([t.ids for t in e.run_turns([Turn("a", "determinisme", sp), Turn("b", "nog een", sp)])])
    assert outs[0] == outs[1]


@pytest.mark.parametrize("M,hq,hkv,d", [(1, 32, 8, 128), (3, 32, 8, 128), (16, 12, 4, 64), (5, 8, 8, 128),
                                         (24, 32, 8, 128), (32, 12, 4, 64)])
def test_skinny_gemm_rope_epilogue(M, hq, hkv, d):
    """qkv GEMM + RMSNorm + RoPE + paged K/V scatter in one kernel == fp32 GEMM -> K2 reference."""
    K = 512
    N = (hq + 2 * hkv) * d
    x = bf(M, K, seed=61)
    W = bf(N, K, scale=0.05, seed=62)
    gam = bf(K, seed=63)
    cos_sin = ref.rope_cos_sin(4096, d, 500000.0, DEV)
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int64)
    nb = 8
    slots = torch.randperm(nb * 32, device=DEV)[:M].to(torch.int64)
    kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
    kc_r, vc_r = kc.cpu().clone(), vc.cpu().clone()
    Ws = ops.shuffle_weight(W, gam, rope_heads=hq + hkv, head_dim=d)
    q = ops.skinny_gemm_rope(x, Ws, ops.PRO_NORM, positions, cos_sin, kc, vc, slots, hq, hkv, d, 1e-5)
    Wp = ref.fold_gamma(W.cpu(), gam.cpu(), hq + hkv, d)
    q_r = ref.skinny_gemm_rope(x.cpu(), Wp, 1, positions.cpu(), cos_sin.cpu(), kc_r, vc_r, slots.cpu(), hq, hkv, d,
                               1e-5)
    close(q, q_r.to(DEV), 0.05, 0.02)
    close(kc, kc_r.to(DEV), 0.05, 0.02)
    close(vc, vc_r.to(DEV), 0.05, 0.02)
    # the permuted reference equals the plain (unpermuted) path: GEMM -> rope_and_cache
    kc2, vc2 = torch.zeros_like(kc_r), torch.zeros_like(vc_r)
    qkv = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W.cpu(), gam.cpu()), 1, eps=1e-5)
    q2 = ref.rope_and_cache(qkv, positions.cpu(), cos_sin.cpu(), kc2, vc2, slots.cpu(), hq, hkv, d)
    close(q_r, q2, 0.05, 0.02)


@pytest.mark.parametrize("M", [1, 3, 20])
@pytest.mark.parametrize("hq,hkv,K,d", [(28, 4, 3584, 128), (4, 1, 3584, 128), (14, 2, 896, 64)])
def test_skinny_gemm_rope_qkv_bias(M, hq, hkv, K, d):
    """Qwen2 q/k/v bias in the RoPE epilogue (after the norm scale, before the rotation; the
    rotate-half partner gets its own column's bias) on every launch form the shapes select —
    whole tiles, CU-balanced halves (Qwen2.5-7B: 288 tiles), split-K (a 48-tile tp shard), the
    20-row serving form — against the natural-order path: fp32 GEMM + bias -> K2 reference."""
    N = (hq + 2 * hkv) * d
    x = bf(M, K, seed=161)
    W = bf(N, K, scale=0.05, seed=162)
    gam = bf(K, seed=163)
    b = bf(N, scale=0.5, seed=164)
    cos_sin = ref.rope_cos_sin(4096, d, 1e6, DEV)
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int64)
    nb = 8
    slots = torch.randperm(nb * 32, device=DEV)[:M].to(torch.int64)
    kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
    Ws = ops.shuffle_weight(W, gam, rope_heads=hq + hkv, head_dim=d)
    q = ops.skinny_gemm_rope(x, Ws, ops.PRO_NORM, positions, cos_sin, kc, vc, slots, hq, hkv, d, 1e-6,
                             split_ws=ops.split_workspace(DEV), bias=ops.rope_bias(b, hq, hkv, d))
    kc_r, vc_r = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    qkv = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W.cpu(), gam.cpu()), 1, 3, None, 1e-6) + b.cpu().float()[None, :]
    q_r = ref.rope_and_cache(qkv, positions.cpu(), cos_sin.cpu(), kc_r, vc_r, slots.cpu(), hq, hkv, d)
    close(q, q_r.to(DEV), 0.05, 0.02)
    close(kc, kc_r.to(DEV), 0.05, 0.02)
    close(vc, vc_r.to(DEV), 0.05, 0.02)


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("hq,hkv,K", [(32, 8, 4096), (40, 8, 1024)])
def test_skinny_gemm_rope_balanced_split(M, hq, hkv, K):
    """CU-balanced qkv launch (remainder tiles as two K-halves; the rotate-half partner is read
    after the hand-off): q / K / V cache equal the fp32 reference, three calls agree bit for bit,
    counters re-arm, and the plain launch agrees up to summation order."""
    d = 128
    N = (hq + 2 * hkv) * d
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert (N // 16) > cus and (N // 16) % cus != 0
    x = bf(M, K, seed=81)
    W = bf(N, K, scale=0.05, seed=82)
    gam = bf(K, seed=83)
    cos_sin = ref.rope_cos_sin(4096, d, 500000.0, DEV)
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int64)
    nb = 8
    slots = torch.randperm(nb * 32, device=DEV)[:M].to(torch.int64)
    Ws = ops.shuffle_weight(W, gam, rope_heads=hq + hkv, head_dim=d)
    ws = ops.split_workspace(DEV)
    runs = []
    for i in range(4):
        kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
        q = ops.skinny_gemm_rope(x, Ws, ops.PRO_NORM, positions, cos_sin, kc, vc, slots, hq, hkv, d, 1e-5,
                                 split_ws=ws if i < 3 else None)
        runs.append((q, kc, vc))
    assert int(ws[:256].abs().sum()) == 0, "split counters must re-arm to zero"
    kc_r = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16)
    vc_r = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16)
    Wp = ref.fold_gamma(W.cpu(), gam.cpu(), hq + hkv, d)
    q_r = ref.skinny_gemm_rope(x.cpu(), Wp, 1, positions.cpu(), cos_sin.cpu(), kc_r, vc_r, slots.cpu(), hq, hkv, d,
                               1e-5)
    for q, kc, vc in runs[:3]:
        close(q, q_r.to(DEV), 0.05, 0.02)
        close(kc, kc_r.to(DEV), 0.05, 0.02)
        close(vc, vc_r.to(DEV), 0.05, 0.02)
        assert torch.equal(q, runs[0][0]) and torch.equal(kc, runs[0][1]) and torch.equal(vc, runs[0][2])
    for a, b in zip(runs[0], runs[3]):
        close(a, b, 0.02, 0.02)


@pytest.mark.parametrize("M", [12, 24, 32])
@pytest.mark.parametrize("hq,hkv,K", [(16, 4, 4096), (32, 8, 4096), (4, 1, 4096)])
def test_skinny_gemm_rope_serving_batches(M, hq, hkv, K):
    """qkv (+RMSNorm, RoPE, paged K/V write) at serving batch sizes: (16, 4) = 192 tiles takes the
    two-tile / two-K-half split launch (hand-off before the rotate-half partner read), (32, 8) =
    384 tiles two tiles per workgroup, (4, 1) = 48 tiles one tile; above 16 rows every one of them
    runs two row blocks. q / K / V cache equal the fp32 reference, repeats agree bit for bit, the
    split counters re-arm."""
    d = 128
    N = (hq + 2 * hkv) * d
    x = bf(M, K, seed=91)
    W = bf(N, K, scale=0.05, seed=92)
    gam = bf(K, seed=93)
    cos_sin = ref.rope_cos_sin(4096, d, 500000.0, DEV)
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int64)
    nb = 4
    slots = torch.randperm(nb * 32, device=DEV)[:M].to(torch.int64)
    Ws = ops.shuffle_weight(W, gam, rope_heads=hq + hkv, head_dim=d)
    ws = ops.split_workspace(DEV)
    runs = []
    for _ in range(2):
        kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
        q = ops.skinny_gemm_rope(x, Ws, ops.PRO_NORM, positions, cos_sin, kc, vc, slots, hq, hkv, d, 1e-5, split_ws=ws)
        runs.append((q, kc, vc))
    assert int(ws[:256].abs().sum()) == 0, "split counters must re-arm to zero"
    kc_r = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16)
    vc_r = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16)
    Wp = ref.fold_gamma(W.cpu(), gam.cpu(), hq + hkv, d)
    q_r = ref.skinny_gemm_rope(x.cpu(), Wp, 1, positions.cpu(), cos_sin.cpu(), kc_r, vc_r, slots.cpu(), hq, hkv, d,
                               1e-5)
    for q, kc, vc in runs:
        close(q, q_r.to(DEV), 0.05, 0.02)
        close(kc, kc_r.to(DEV), 0.05, 0.02)
        close(vc, vc_r.to(DEV), 0.05, 0.02)
    assert all(torch.equal(a, b) for a, b in zip(runs[0], runs[1]))


def test_norm_add_prologue():
    """TP decode prologue: normalize bf16(x + x2), workgroup 0 publishes the sum."""
    M, N, K = 3, 512, 4096
    x, x2 = bf(M, K, seed=71), bf(M, K, seed=72)
    W = bf(N, K, scale=0.05, seed=73)
    gam = bf(K, seed=74)
    xo = torch.zeros_like(x)
    got = ops.skinny_gemm(x, ops.shuffle_weight(W, gam), ops.PRO_NORM_ADD, eps=1e-5, x2=x2, xout=xo)
    xo_r = torch.zeros(M, K, dtype=torch.bfloat16)
    exp = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W.cpu(), gam.cpu()), 2, eps=1e-5, x2=x2.cpu(), xout=xo_r)
    close(got, exp.to(DEV), 0.05, 0.02)
    assert torch.equal(xo, xo_r.to(DEV))
    # SwiGLU epilogue with the same prologue
    W2 = bf(2 * N, K, scale=0.05, seed=75)
    got = ops.skinny_gemm(x, ops.shuffle_weight(W2, gam, swiglu=True), ops.PRO_NORM_ADD, ops.EPI_SWIGLU, x2=x2)
    exp = ref.skinny_gemm(x.cpu(), ref.fold_gamma(W2.cpu(), gam.cpu()), 2, 2, x2=x2.cpu())
    close(got, exp.to(DEV), 0.05, 0.03)


def test_tp_fused_decode_path_matches_tp1_fused():
    """The tensor-parallel fused forward (NORM_ADD prologues, ping-pong residual) at tp=1 equals
    the single-GPU fused forward (in-place RESID epilogues)."""
    from theroundtaible_amd.engine import Engine, EngineConfig
    from theroundtaible_amd.models.llama import AttnMeta
    e = Engine(EngineConfig(model="tiny-llama-128", weights="random-full:5", device=DEV, num_blocks=64,
                            use_graphs=False))
    ids = e.encode_prompt("tensor parallel fused decode " * 4)
    s = e.kv.seq("a")
    e.prefill([(s, ids)])
    e.kv.ensure_capacity(s, s.length + 1)
    pos = torch.tensor([s.length], device=DEV)
    slots = torch.tensor([s.blocks[s.length // 32] * 32 + s.length % 32], device=DEV)
    bt = torch.zeros(1, 8, dtype=torch.int32)
    bt[0, :len(s.blocks)] = torch.tensor(s.blocks)
    meta = AttnMeta("decode", slots, bt.to(DEV), (pos + 1).to(torch.int32), num_splits=4)
    tok = torch.tensor([9], device=DEV)
    a = e.model.forward(tok, pos, e.kv, meta).float()
    e.model.force_tp_path = True
    b = e.model.forward(tok, pos, e.kv, meta).float()
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert float(cos.min()) > 0.999



def _cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


# Llama-3-8B / 70B tensor-parallel shard shapes with fewer tiles than CUs (split-K launches):
# (N, K) of qkv / gate_up rows at tp 8 and 4, plus odd tile counts (T % 8 != 0: plain placement)
SPLITK_SHAPES = [(768, 4096), (1536, 4096), (1792, 4096), (80, 1024), (1200, 8192)]


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("N,K", SPLITK_SHAPES)
def test_skinny_gemm_splitk_every_epilogue(M, N, K):
    """Split-K (tiles < CUs, K cut into S parts, last arriver combines in index order): every
    prologue / epilogue the decode path uses equals the fp32 reference, repeated calls are bit-
    identical and the tile counters re-arm."""
    T = N // 16
    assert T < _cus() and ops.native().splitk_parts(T, K // 32, _cus(), ops.SPLIT_WS_INTS) >= 2
    ws = ops.split_workspace(DEV)
    x, x2 = bf(M, K, seed=91), bf(M, K, seed=92)
    gam = bf(K, seed=93)
    W = bf(N, K, scale=0.05, seed=94)
    Ws, Wg = ops.shuffle_weight(W), ops.shuffle_weight(W, gam)
    Wf = ref.fold_gamma(W.cpu(), gam.cpu())
    # PLAIN / NORM store
    outs = [ops.skinny_gemm(x, Ws, split_ws=ws) for _ in range(3)]
    close(outs[0], ref.skinny_gemm(x.cpu(), W.cpu()).to(DEV), 0.05, 0.02)
    assert all(torch.equal(o, outs[0]) for o in outs)
    close(ops.skinny_gemm(x, Wg, ops.PRO_NORM, eps=1e-5, split_ws=ws),
          ref.skinny_gemm(x.cpu(), Wf, 1, eps=1e-5).to(DEV), 0.05, 0.02)
    # NORM_ADD (tp residual + partial): every part of tile 0 publishes its K range of x + x2
    xo = torch.zeros_like(x)
    xo_r = torch.zeros(M, K, dtype=torch.bfloat16)
    got = ops.skinny_gemm(x, Wg, ops.PRO_NORM_ADD, eps=1e-5, x2=x2, xout=xo, split_ws=ws)
    close(got, ref.skinny_gemm(x.cpu(), Wf, 2, eps=1e-5, x2=x2.cpu(), xout=xo_r).to(DEV), 0.05, 0.02)
    assert torch.equal(xo, xo_r.to(DEV))
    # RESID in place
    res = bf(M, N, seed=95)
    res_ref = res.cpu().clone()
    ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res, split_ws=ws)
    ref.skinny_gemm(x.cpu(), W.cpu(), 0, 1, res=res_ref)
    close(res, res_ref.to(DEV), 0.06, 0.02)
    # SwiGLU over [gate; up] (N rows each) with NORM and NORM_ADD prologues
    W2 = bf(2 * N, K, scale=0.05, seed=96)
    W2s = ops.shuffle_weight(W2, gam, swiglu=True)
    W2f = ref.fold_gamma(W2.cpu(), gam.cpu())
    close(ops.skinny_gemm(x, W2s, ops.PRO_NORM, ops.EPI_SWIGLU, split_ws=ws),
          ref.skinny_gemm(x.cpu(), W2f, 1, 2).to(DEV), 0.05, 0.03)
    close(ops.skinny_gemm(x, W2s, ops.PRO_NORM_ADD, ops.EPI_SWIGLU, x2=x2, split_ws=ws),
          ref.skinny_gemm(x.cpu(), W2f, 2, 2, x2=x2.cpu()).to(DEV), 0.05, 0.03)
    assert int(ws[:256].abs().sum()) == 0, "split counters must re-arm to zero"
    # no workspace: one workgroup per tile, same result up to summation order
    close(ops.skinny_gemm(x, Ws), outs[0], 0.02, 0.02)


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("hq,hkv,K", [(4, 1, 4096), (8, 2, 4096), (16, 2, 8192), (2, 1, 1024)])
def test_skinny_gemm_rope_splitk(M, hq, hkv, K):
    """qkv shard of a tensor-parallel knight (Llama-3-8B tp 8 / 4, 70B tp 4): split-K with the
    NORM_ADD prologue and the RoPE + paged K/V epilogue equals the fp32 reference."""
    d = 128
    N = (hq + 2 * hkv) * d
    assert N // 16 < _cus()
    x, x2 = bf(M, K, seed=101), bf(M, K, seed=102)
    W = bf(N, K, scale=0.05, seed=103)
    gam = bf(K, seed=104)
    cos_sin = ref.rope_cos_sin(4096, d, 500000.0, DEV)
    positions = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int64)
    nb = 8
    slots = torch.randperm(nb * 32, device=DEV)[:M].to(torch.int64)
    Ws = ops.shuffle_weight(W, gam, rope_heads=hq + hkv, head_dim=d)
    Wp = ref.fold_gamma(W.cpu(), gam.cpu(), hq + hkv, d)
    ws = ops.split_workspace(DEV)
    for pro in (ops.PRO_NORM, ops.PRO_NORM_ADD):
        kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
        xo = torch.zeros_like(x)
        kw = dict(x2=x2, xout=xo) if pro == ops.PRO_NORM_ADD else {}
        q = ops.skinny_gemm_rope(x, Ws, pro, positions, cos_sin, kc, vc, slots, hq, hkv, d, 1e-5, split_ws=ws, **kw)
        kc_r = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16)
        vc_r = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16)
        kw_r = dict(x2=x2.cpu(), xout=torch.zeros(M, K, dtype=torch.bfloat16)) if pro == ops.PRO_NORM_ADD else {}
        q_r = ref.skinny_gemm_rope(x.cpu(), Wp, pro, positions.cpu(), cos_sin.cpu(), kc_r, vc_r, slots.cpu(), hq, hkv,
                                   d, 1e-5, **kw_r)
        close(q, q_r.to(DEV), 0.05, 0.02)
        close(kc, kc_r.to(DEV), 0.05, 0.02)
        close(vc, vc_r.to(DEV), 0.05, 0.02)
        if pro == ops.PRO_NORM_ADD:
            assert torch.equal(xo, kw_r["xout"].to(DEV))
    assert int(ws[:256].abs().sum()) == 0


@pytest.mark.parametrize("N,K,rope,swiglu", [(6 * 128, 256, 4, False), (512, 4096, 0, True), (4096, 14336, 0, False)])
def test_unshuffle_is_exact_inverse(N, K, rope, swiglu):
    W = bf(N, K, seed=3)
    Ws = ops.shuffle_weight(W, None, rope_heads=rope, head_dim=128 if rope else 0, swiglu=swiglu)
    assert torch.equal(ops.unshuffle_weight(Ws, rope_heads=rope, head_dim=128 if rope else 0, swiglu=swiglu), W)


def test_shuffled_only_residency_engine():
    """One resident weight copy (shuffled; prefill unshuffles per GEMM) vs both copies: same
    prefill logits (up to the folded-gamma rounding) and the same fused decode."""
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    kw = dict(model="llama3-8b", weights="random-full:5", device=DEV, num_blocks=256,
              model_overrides={"n_layers": 2})
    a = Engine(EngineConfig(weight_residency="dual", **kw))
    b = Engine(EngineConfig(weight_residency="shuffled", **kw))
    assert b.model.shuffled_only and not a.model.shuffled_only
    ids = a.encode_prompt("een enkele kopie van de gewichten in HBM " * 20)
    la = a.prefill([(a.kv.seq("k"), ids)]).float()
    lb = b.prefill([(b.kv.seq("k"), ids)]).float()
    assert float(torch.nn.functional.cosine_similarity(la, lb, dim=-1).min()) > 0.999
    sp = SamplingParams(temperature=0.0, max_new_tokens=6, ignore_eos=True, stop_on_consensus=False)
    oa = a.run_turns([Turn("x", "hallo tafel " * 30, sp)])[0]
    ob = b.run_turns([Turn("x", "hallo tafel " * 30, sp)])[0]
    assert oa.error is None and ob.error is None and len(ob.ids) == 6


def test_shuffled_only_load_peak_is_one_weight_copy():
    """shuffled-only residency frees each row-major linear as soon as its shuffled copy
    exists (both references), so the load peak is ONE weight copy + one tensor — not the row-major
    weights plus the full shuffled copy (a 70B knight on one GPU fits by only ~8 GB)."""
    import gc
    from theroundtaible_amd.engine import Engine, EngineConfig
    from theroundtaible_amd.models.config import get_config
    gc.collect()
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    e = Engine(EngineConfig(model="llama3-8b", weights="random:5", device=DEV, weight_residency="shuffled",
                            defer_kv=True, model_overrides={"n_layers": 4}))
    assert e.model.shuffled_only
    cfg = e.cfg
    wbytes = cfg.n_params() * 2
    biggest = cfg.vocab * cfg.hidden * 2
    peak = torch.cuda.max_memory_allocated() - base
    assert peak <= wbytes + 1.05 * biggest + (256 << 20), (peak / 2**30, wbytes / 2**30)
    del e
