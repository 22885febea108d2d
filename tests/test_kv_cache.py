"""Paged KV cache: K8 block copies (copy-on-write tail, deep snapshot forks)."""
import pytest
import torch

from theroundtaible_amd.engine.kv_cache import PagedKVCache


def _cache(device="cpu", dtype=torch.float32):
    kv = PagedKVCache(n_layers=3, n_kv_heads=2, head_dim=16, num_blocks=12, block_size=4, device=device, dtype=dtype)
    g = torch.Generator().manual_seed(0)
    kv.k.copy_(torch.randn(kv.k.shape, generator=g).to(dtype))
    kv.v.copy_(torch.randn(kv.v.shape, generator=g).to(dtype))
    return kv


def test_copy_blocks_all_layers():
    kv = _cache()
    k0, v0 = kv.k.clone(), kv.v.clone()
    kv.copy_blocks([1, 5], [7, 9])
    assert torch.equal(kv.k[:, 7], k0[:, 1]) and torch.equal(kv.v[:, 9], v0[:, 5])
    assert torch.equal(kv.k[:, 1], k0[:, 1]) and torch.equal(kv.k[:, 3], k0[:, 3])


def test_fork_copy_is_a_deep_snapshot():
    kv = _cache()
    a = kv.seq("a")
    kv.ensure_capacity(a, 10)
    a.tokens.extend(range(10))
    b = kv.fork("a", "b", copy=True)
    assert b.tokens == a.tokens and not set(b.blocks) & set(a.blocks)
    for x, y in zip(a.blocks, b.blocks):
        assert torch.equal(kv.k[:, x], kv.k[:, y]) and torch.equal(kv.v[:, x], kv.v[:, y])
    assert all(kv.alloc.ref[blk] == 1 for blk in a.blocks + b.blocks)
    shared = kv.fork("a", "c")
    assert shared.blocks == a.blocks and all(kv.alloc.ref[blk] == 2 for blk in a.blocks)


def test_cow_tail_copies_partial_block():
    kv = _cache()
    a = kv.seq("a")
    kv.ensure_capacity(a, 6)
    a.tokens.extend(range(6))                 # 2 blocks, the second half full
    kv.fork("a", "b")
    b = kv.seqs["b"]
    tail = b.blocks[-1]
    kv.ensure_capacity(b, 7)                  # writes into the shared partial block -> COW
    assert b.blocks[-1] != tail and a.blocks[-1] == tail
    assert torch.equal(kv.k[:, b.blocks[-1]], kv.k[:, tail])


@pytest.mark.gpu
def test_kv_block_copy_kernel_matches_torch():
    kv = _cache("cuda", torch.bfloat16)
    k0, v0 = kv.k.clone(), kv.v.clone()
    src, dst = [0, 3, 4], [11, 10, 2]
    kv.copy_blocks(src, dst)
    torch.cuda.synchronize()
    for s_, d_ in zip(src, dst):
        assert torch.equal(kv.k[:, d_], k0[:, s_]) and torch.equal(kv.v[:, d_], v0[:, s_])
    untouched = [b for b in range(12) if b not in dst]
    assert torch.equal(kv.k[:, untouched], k0[:, untouched])
    with pytest.raises(RuntimeError):
        kv.copy_blocks([0], [12])              # out of range: refused before the launch
