"""CPU checks of the op reference semantics the HIP kernels are tested against.

The fused decode kernels (csrc/gemm_skinny.hip) work on re-laid-out weights; these tests
pin that the re-layouts are semantic no-ops, so the GPU tests' fp32 oracle is the model.
"""
import torch

from theroundtaible_amd import ops
from theroundtaible_amd.ops import reference as ref


def test_rope_row_perm_is_pair_interleave():
    p = ref.rope_row_perm(3 * 8 + 4, 3, 8)
    assert p[:8].tolist() == [0, 4, 1, 5, 2, 6, 3, 7]
    assert p[8:16].tolist() == [8, 12, 9, 13, 10, 14, 11, 15]
    assert p[24:].tolist() == [24, 25, 26, 27]
    assert sorted(p.tolist()) == list(range(28))


def test_skinny_gemm_rope_reference_matches_unfused():
    torch.manual_seed(0)
    M, hq, hkv, d, K = 3, 8, 2, 64, 128
    N = (hq + 2 * hkv) * d
    x = torch.randn(M, K).bfloat16()
    W = (torch.randn(N, K) * 0.05).bfloat16()
    g = torch.randn(K).bfloat16()
    cs = ref.rope_cos_sin(256, d, 10000.0)
    pos = torch.tensor([5, 100, 200])
    slots = torch.tensor([3, 40, 77])
    kc = torch.zeros(4, hkv, 32, d).bfloat16()
    vc = torch.zeros(4, hkv, d, 32).bfloat16()
    Wp = ops.shuffle_weight(W, g, rope_heads=hq + hkv, head_dim=d)
    q = ops.skinny_gemm_rope(x, Wp, ops.PRO_NORM, pos, cs, kc, vc, slots, hq, hkv, d)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    qkv = ref.skinny_gemm(x, ref.fold_gamma(W, g), ops.PRO_NORM)
    q2 = ref.rope_and_cache(qkv, pos, cs, kc2, vc2, slots, hq, hkv, d)
    assert (q.float() - q2.float()).abs().max() < 0.02
    assert (kc.float() - kc2.float()).abs().max() < 0.02
    assert torch.equal(vc, vc2)


def test_skinny_gemm_rope_bias_reference_matches_unfused():
    """Qwen2 q/k/v bias: permuted into the shuffled weight's column order (ops.rope_bias) and
    added before RoPE, it equals the natural-order GEMM + bias -> K2 path."""
    torch.manual_seed(2)
    M, hq, hkv, d, K = 3, 8, 2, 64, 128
    N = (hq + 2 * hkv) * d
    x = torch.randn(M, K).bfloat16()
    W = (torch.randn(N, K) * 0.05).bfloat16()
    g = torch.randn(K).bfloat16()
    b = (torch.randn(N) * 0.5).bfloat16()
    cs = ref.rope_cos_sin(256, d, 1e6)
    pos = torch.tensor([5, 100, 200])
    slots = torch.tensor([3, 40, 77])
    kc = torch.zeros(4, hkv, 32, d).bfloat16()
    vc = torch.zeros(4, hkv, d, 32).bfloat16()
    Wp = ops.shuffle_weight(W, g, rope_heads=hq + hkv, head_dim=d)
    q = ops.skinny_gemm_rope(x, Wp, ops.PRO_NORM, pos, cs, kc, vc, slots, hq, hkv, d,
                             bias=ops.rope_bias(b, hq, hkv, d))
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    qkv = ref.skinny_gemm(x, ref.fold_gamma(W, g), ops.PRO_NORM, 3) + b.float()[None, :]
    q2 = ref.rope_and_cache(qkv, pos, cs, kc2, vc2, slots, hq, hkv, d)
    assert (q.float() - q2.float()).abs().max() < 0.02
    assert (kc.float() - kc2.float()).abs().max() < 0.02
    assert (vc.float() - vc2.float()).abs().max() < 0.02
    # without the bias the result differs (the test would not see a dropped bias otherwise)
    kc3, vc3 = torch.zeros_like(kc), torch.zeros_like(vc)
    q3 = ops.skinny_gemm_rope(x, Wp, ops.PRO_NORM, pos, cs, kc3, vc3, slots, hq, hkv, d)
    assert (q3.float() - q2.float()).abs().max() > 0.1


def test_skinny_gemm_norm_prologue_equals_rmsnorm_then_linear():
    torch.manual_seed(1)
    x = torch.randn(4, 256).bfloat16()
    W = (torch.randn(64, 256) * 0.05).bfloat16()
    g = torch.randn(256).bfloat16()
    fused = ref.skinny_gemm(x, ref.fold_gamma(W, g), ops.PRO_NORM, eps=1e-5).float()
    plain = ref.rms_norm(x, g, 1e-5).float() @ W.float().t()
    assert (fused - plain).abs().max() < 0.05


def test_decode_splits_bounds():
    assert ops.decode_splits(1, 8) == 32
    assert ops.decode_splits(4, 8) == 8
    assert ops.decode_splits(16, 8) == 2
    assert ops.decode_splits(64, 8) == 1
    assert ops.decode_splits(3, 8) == 10
    assert ops.decode_splits(1, 1) == 64
    # shared-prefix groups: the whole chip, the 3-knight table included
    assert ops.decode_splits(3, 8, num_cus=256, grouped=True) == 10
    assert ops.decode_splits(8, 8, num_cus=256, grouped=True) == 4
    assert ops.decode_splits(16, 8, num_cus=256, grouped=True) == 2


def test_decode_prep_and_advance_reference():
    bt = torch.tensor([[5, 7, 9], [2, 3, 4]], dtype=torch.int32)
    pos = torch.tensor([33, 64])
    ids = torch.tensor([1, 3])
    emb = torch.arange(4 * 8, dtype=torch.float32).reshape(4, 8).bfloat16()
    slots, offs = torch.zeros(2, dtype=torch.int64), torch.zeros(2, dtype=torch.int64)
    res = torch.zeros(2, 8).bfloat16()
    ops.decode_prep(slots, offs, res, ids, pos, bt, emb, 32)
    assert slots.tolist() == [7 * 32 + 1, 4 * 32 + 0]
    assert offs.tolist() == [34, 65]
    assert torch.equal(res, emb[[1, 3]])
    out = torch.zeros(4, 2, dtype=torch.int64)
    ctx = torch.tensor([34, 65], dtype=torch.int32)
    step = torch.zeros(1, dtype=torch.int64)
    ops.decode_advance(out, ids, pos, ctx, step, torch.tensor([11, 12]))
    assert out[0].tolist() == [11, 12] and ids.tolist() == [11, 12]
    assert pos.tolist() == [34, 65] and ctx.tolist() == [35, 66] and step.item() == 1
    # fused next-step prep: same result as a separate decode_prep on the advanced state
    s2, o2, r2 = torch.zeros_like(slots), torch.zeros_like(offs), torch.zeros_like(res)
    ops.decode_advance(out, ids, pos, ctx, step, torch.tensor([2, 0]), prep=(s2, o2, r2, bt, emb, 32))
    ops.decode_prep(slots, offs, res, ids, pos, bt, emb, 32)
    assert torch.equal(s2, slots) and torch.equal(o2, offs) and torch.equal(r2, res)
    assert s2.tolist() == [7 * 32 + 3, 4 * 32 + 2] and torch.equal(r2, emb[[2, 0]])
    # a position past the block table (after a turn's last step) maps into block 0, no fault
    ops.decode_prep(slots, offs, res, ids, torch.tensor([96, 97]), bt, emb, 32)
    assert slots.tolist() == [0, 1]


def _guard_case():
    bt = torch.tensor([[3, 5, 0], [7, 1, 2]], dtype=torch.int32)
    ctx = torch.tensor([40, 33], dtype=torch.int32)
    pos = (ctx - 1).to(torch.int64)
    slots = torch.tensor([5 * 32 + 7, 1 * 32 + 0], dtype=torch.int64)
    return bt, ctx, pos, slots


def test_paging_guard_reference_codes():
    bt, ctx, pos, slots = _guard_case()
    err = torch.zeros(1, dtype=torch.int32)
    ref.paging_guard(bt, ctx, pos, slots, err, num_blocks=8, block_size=32)
    assert int(err[0]) == 0
    bad = bt.clone()
    bad[1, 1] = 8                                     # outside an 8-block pool
    ref.paging_guard(bad, ctx, pos, None, err, 8, 32)
    assert int(err[0]) == 2
    err.zero_()
    ref.paging_guard(bt, ctx, pos, slots + 1, err, 8, 32)   # wrong write slot
    assert int(err[0]) == 4
    err.zero_()
    ref.paging_guard(bt, ctx + 1, pos, None, err, 8, 32)    # ctx / position disagree
    assert int(err[0]) == 8
    err.zero_()
    ref.paging_guard(bt, torch.tensor([97, 0], dtype=torch.int32), None, None, err, 8, 32)
    assert int(err[0]) == 1
    assert "KV pool" in ops.paging_guard_message(2) and ops.paging_guard_message(0) == "ok"


def test_debug_env_mode():
    from theroundtaible_amd.utils.debug import apply_debug_env
    env = {"ROUNDTABLE_DEBUG": "1", "HIP_LAUNCH_BLOCKING": "0"}
    assert apply_debug_env(env)
    assert env["AMD_SERIALIZE_KERNEL"] == "3" and env["ROUNDTABLE_DEBUG_CHECKS"] == "1"
    assert env["HIP_LAUNCH_BLOCKING"] == "0"          # explicit settings win
    assert not apply_debug_env({})


def test_split_workspace_matches_native_layout():
    """ops.SPLIT_WS_INTS (Python allocation of the CU-balanced GEMM workspace) covers what the
    launcher needs for the largest remainder (255 split tiles); the extension imports on a CPU
    host, so the check runs here."""
    import pytest
    if not ops.native_available():
        pytest.skip("native extension not built")
    assert ops.SPLIT_WS_INTS >= ops.native().split_workspace_ints(255)
    assert ops.split_workspace("cpu").numel() == ops.SPLIT_WS_INTS


def test_prefill_split_plan_shapes():
    """The planner splits only when whole tiles leave most CUs idle, and its parts tile each key
    range exactly (host-only check of the plan the GPU test runs)."""
    cu = torch.tensor([0, 1772], dtype=torch.int32)
    st = torch.tensor([16000], dtype=torch.int32)
    assert ops.prefill_split_plan(cu, 64, st, 8, num_cus=256) is None          # tp 1: 28 x 8 tiles
    items, cmap, parts = ops.prefill_split_plan(cu, 64, st, 1, num_cus=256)    # tp 8: 28 tiles
    assert items.shape[1] == 5 and cmap.shape[1] == 4 and parts == int(cmap[:, 3].sum())
    assert len(items) >= 256                                                    # ~2 items per CU
    for s, r, p0, n in cmap.tolist():
        mine = sorted((tb, te) for s2, r2, tb, te, p in items.tolist() if (s2, r2) == (s, r))
        assert mine[0][0] == 0 and all(a[1] == b[0] for a, b in zip(mine, mine[1:]))
        assert sorted(p for s2, r2, tb, te, p in items.tolist() if (s2, r2) == (s, r)) == list(range(p0, p0 + n))


def test_k_cache_blocks_are_chunk_major():
    """The K cache layout every kernel and the oracle share (csrc/common.h kc_elem): block
    [blk, head] holds [head_dim/32][block_size][32]; write_k / k_rows / set_k_row index it."""
    hkv, d = 2, 64
    kc = torch.zeros(4, hkv, 32, d)
    k = torch.randn(3, hkv, d)
    ref.write_k(kc, torch.tensor([1, 1, 3]), torch.tensor([0, 5, 31]), k)
    rows = ref.k_rows(kc, torch.tensor([1, 3]))
    assert torch.equal(rows[0], k[0]) and torch.equal(rows[5], k[1]) and torch.equal(rows[32 + 31], k[2])
    flat = kc.view(-1)
    for (blk, h, key, dd, want) in [(1, 0, 5, 40, k[1, 0, 40]), (3, 1, 31, 7, k[2, 1, 7]), (1, 1, 0, 63, k[0, 1, 63])]:
        assert flat[(blk * hkv + h) * 32 * d + (dd // 32) * 32 * 32 + key * 32 + dd % 32] == want
    r = torch.randn(d)
    ref.set_k_row(kc, 2, 1, 9, r)
    assert torch.equal(ref.k_rows(kc, torch.tensor([2]))[9, 1], r)
