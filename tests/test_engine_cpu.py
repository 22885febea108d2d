"""Engine plumbing on CPU (PyTorch reference ops): paged KV, prefix reuse, errors, config 1 shapes."""
import pytest
import torch

from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
from theroundtaible_amd.engine.kv_cache import BlockAllocator, KVCacheOOM, PagedKVCache
from theroundtaible_amd.errors import AdapterError
from theroundtaible_amd.prompt import Prompt

GREEDY = SamplingParams(temperature=0.0, max_new_tokens=10, ignore_eos=True, stop_on_consensus=False)


def cpu_engine(model="tiny-llama", **kw):
    cfg = dict(model=model, device="cpu", dtype="fp32", num_blocks=128, weights="random:2")
    cfg.update(kw)
    return Engine(EngineConfig(**cfg))


def test_block_allocator_refcounts():
    a = BlockAllocator(4)
    b = [a.alloc() for _ in range(4)]
    with pytest.raises(KVCacheOOM):
        a.alloc()
    a.incref(b[0])
    a.release(b[0])
    assert a.num_free == 0
    a.release(b[0])
    assert a.num_free == 1


def test_truncate_fork_cow():
    kv = PagedKVCache(1, 1, 8, 16, 4, "cpu", torch.float32)
    s = kv.seq("a")
    kv.ensure_capacity(s, 6)
    s.tokens.extend(range(6))
    kv.k[0, s.blocks[1]].fill_(7.0)
    f = kv.fork("a", "b")
    assert f.blocks == s.blocks and kv.alloc.ref[s.blocks[0]] == 2
    kv.ensure_capacity(f, 7)          # tail block shared & partial -> copy-on-write
    assert f.blocks[1] != s.blocks[1] and float(kv.k[0, f.blocks[1]].mean()) == 7.0
    kv.truncate(s, 3)
    assert len(s.blocks) == 1 and s.tokens == [0, 1, 2]
    kv.free_seq("a")
    kv.free_seq("b")
    assert kv.alloc.num_free == 16


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-llama-128", "tiny-gpt2"])
def test_prefix_reuse_is_exact(model):
    e = cpu_engine(model)
    t1 = e.run_turns([Turn("K", "Onderwerp: caching in de tafel.", GREEDY)])[0]
    p2 = Prompt().add("Onderwerp: caching in de tafel.").add(t1.text, t1.ids, e.tokenizer.family).add(" Verder.")
    t2 = e.run_turns([Turn("K", p2, GREEDY)])[0]
    assert t2.metrics["reused_tokens"] == t1.metrics["prompt_tokens"] + len(t1.ids) - 1
    fresh = cpu_engine(model).run_turns([Turn("K", p2, GREEDY)])[0]
    assert fresh.ids == t2.ids


def test_batched_equals_single():
    e = cpu_engine()
    both = e.run_turns([Turn("A", "eerste knight", GREEDY), Turn("B", "tweede knight, langer prompt", GREEDY)])
    solo = cpu_engine().run_turns([Turn("B", "tweede knight, langer prompt", GREEDY)])
    assert both[1].ids == solo[0].ids


def test_chunked_prefill_matches_unchunked():
    long = "woord " * 300
    a = cpu_engine(prefill_chunk=64).run_turns([Turn("K", long, GREEDY)])[0]
    b = cpu_engine(prefill_chunk=8192).run_turns([Turn("K", long, GREEDY)])[0]
    assert a.ids == b.ids


def test_oom_is_classified_and_recovers():
    e = cpu_engine(num_blocks=4)
    out = e.run_turns([Turn("K", "x " * 400, GREEDY)])[0]
    assert isinstance(out.error, AdapterError) and out.error.kind == "oom"
    assert e.kv.alloc.num_free == 4
    ok = e.run_turns([Turn("K", "kort", SamplingParams(temperature=0, max_new_tokens=4, ignore_eos=True,
                                                        stop_on_consensus=False))])[0]
    assert ok.error is None and len(ok.ids) == 4


def test_context_past_max_positions_fails_the_turn_on_the_host():
    """A context longer than the model's positions (RoPE table, block-table width) must fail the
    turn before any kernel indexes past those tables (Qwen2.5-7B: 32768 positions; a 40K-token
    discussion faulted the GPU before this guard) — as prefill and as decode growth."""
    from dataclasses import replace as dc_replace
    e = cpu_engine(num_blocks=256)
    assert e.kv.max_tokens == e.cfg.max_pos
    e.kv.max_tokens = 128                    # a short-context model without building one
    out = e.run_turns([Turn("K", "woord " * 200, GREEDY)])[0]
    assert isinstance(out.error, AdapterError) and out.error.kind == "oom" and "positions" in str(out.error)
    # a prompt that fits but whose reply would cross the limit fails the same way
    n = len(e.encode_prompt("woord " * 40))
    assert n + 2 < 128
    sp = dc_replace(GREEDY, max_new_tokens=128 - n + 8)
    out = e.run_turns([Turn("K2", "woord " * 40, sp)])[0]
    assert out.error is not None and out.error.kind == "oom"
    ok = e.run_turns([Turn("K3", "kort", GREEDY)])[0]
    assert ok.error is None and len(ok.ids) == 10


def test_timeout():
    e = cpu_engine(sync_every=1)
    out = e.run_turns([Turn("K", "hallo", SamplingParams(temperature=0, max_new_tokens=50, ignore_eos=True,
                                                         stop_on_consensus=False), timeout_s=0.0)])[0]
    assert out.error is not None and out.error.kind == "timeout"


def test_stop_on_consensus_cuts_generation(monkeypatch):
    from theroundtaible_amd.engine import engine as eng_mod
    e = cpu_engine()
    tok = e.tokenizer
    block = tok.encode('```json\n{"consensus_score": 9}\n```')
    ids = block + tok.encode(" trailing junk")
    assert eng_mod._cut_at_consensus(tok, ids) == block or len(eng_mod._cut_at_consensus(tok, ids)) <= len(block)


def test_gpt2_small_shapes_cpu():
    """Config 1's model builds and runs on CPU with the real GPT-2-small shapes."""
    e = Engine(EngineConfig(model="gpt2-small", device="cpu", dtype="fp32", num_blocks=64, weights="random:0"))
    assert e.cfg.n_layers == 12 and e.cfg.hidden == 768 and e.cfg.vocab == 50257
    out = e.run_turns([Turn("K", "GPT-2 knight", SamplingParams(temperature=0.7, max_new_tokens=4, ignore_eos=True,
                                                                 stop_on_consensus=False))])[0]
    assert len(out.ids) == 4 and all(0 <= i < 50257 for i in out.ids)


def test_engine_fault_injection_and_health():
    """injected faults surface as classified per-turn errors; a device fault marks
    the engine unhealthy so later turns are refused (the orchestrator then skips / falls back)."""
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    sp = SamplingParams(temperature=0.0, max_new_tokens=3, ignore_eos=True, stop_on_consensus=False)
    e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=64,
                            faults={0: "oom", 1: "timeout", 3: "device"}))
    r0 = e.run_turns([Turn("a", "x", sp)])[0]
    assert r0.error is not None and r0.error.kind == "oom"
    r1 = e.run_turns([Turn("a", "x", sp)])[0]
    assert r1.error is not None and r1.error.kind == "timeout"
    r2 = e.run_turns([Turn("a", "x", sp)])[0]
    assert r2.error is None and len(r2.ids) == 3
    r3 = e.run_turns([Turn("a", "x", sp)])[0]
    assert r3.error.kind == "device" and not e.healthy
    # the next call probes the device, drops the (possibly stale) resident KV and serves again
    r4 = e.run_turns([Turn("a", "x", sp)])[0]
    assert r4.error is None and e.healthy and len(r4.ids) == 3 and r4.metrics["reused_tokens"] == 0


def test_engine_unrecoverable_device_and_flag_faults():
    """A device the recovery probe cannot clear stays unhealthy; a device-side poll expiry (K9 /
    persistent-kernel error flag) fails only that turn and drops its KV."""
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    sp = SamplingParams(temperature=0.0, max_new_tokens=3, ignore_eos=True, stop_on_consensus=False)
    e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=64,
                            faults={1: "flag", 3: "device-dead"}))
    assert e.run_turns([Turn("a", "hello", sp)])[0].error is None
    r1 = e.run_turns([Turn("a", "hello", sp)])[0]
    assert r1.error.kind == "device" and "poll expiry" in str(r1.error) and e.healthy
    assert "a" not in e.kv.seqs                      # its KV was dropped, not trusted
    assert e.run_turns([Turn("a", "hello", sp)])[0].error is None
    r3 = e.run_turns([Turn("a", "hello", sp)])[0]
    assert r3.error.kind == "device" and not e.healthy
    assert e.run_turns([Turn("a", "hello", sp)])[0].error.kind == "device"


def test_engine_reads_device_flags_after_decode(monkeypatch):
    """The error flags of bounded device waits are read at the end-of-turn sync; a raised flag
    fails the turn with kind 'device'."""
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    sp = SamplingParams(temperature=0.0, max_new_tokens=3, ignore_eos=True, stop_on_consensus=False)
    e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=64))
    monkeypatch.setattr(e, "device_flag_errors", lambda: ["K9 one-shot all-reduce: a peer's flag never arrived"])
    r = e.run_turns([Turn("a", "hello", sp)])[0]
    assert r.error.kind == "device" and "K9" in str(r.error)


def test_debug_paging_checks():
    import pytest as _pt
    from theroundtaible_amd.engine import Engine, EngineConfig
    e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=16, debug_checks=True))
    e.check_paging(torch.tensor([[0, 15]], dtype=torch.int32), [0, 16 * 32 - 1])
    with _pt.raises(AssertionError):
        e.check_paging(torch.tensor([[16]], dtype=torch.int32), [])
    with _pt.raises(AssertionError):
        e.check_paging(torch.tensor([[0]], dtype=torch.int32), [16 * 32])


def test_shuffled_only_residency_matches_dual():
    """Dropping the row-major linears after shuffling (one weight copy resident) leaves the
    unfused/prefill path numerically equal: it rebuilds each gamma-folded operand by the exact
    inverse permutation (ops.unshuffle_weight) and normalizes with unit weights."""
    from theroundtaible_amd.engine import Engine, EngineConfig
    from theroundtaible_amd import ops
    a = Engine(EngineConfig(model="tiny-llama-128", device="cpu", dtype="fp32", num_blocks=64, weights="random-full:5"))
    b = Engine(EngineConfig(model="tiny-llama-128", device="cpu", dtype="fp32", num_blocks=64, weights="random-full:5"))
    b.model.decode_weights(drop_originals=True)
    assert b.model.shuffled_only and b.model.layers[0]["wqkv"] is None and b.model.w["lm_head"] is None
    ids = a.encode_prompt("Een gedeelde sleutel voor de ronde tafel, graag. " * 4)
    la = a.prefill([(a.kv.seq("k"), ids)])
    lb = b.prefill([(b.kv.seq("k"), ids)])
    assert torch.allclose(la, lb, atol=1e-4, rtol=1e-4)
    # the inverse permutation is exact, rope-permuted qkv rows included
    W = torch.randn(3 * 2 * 128, 64)
    Ws = ops.shuffle_weight(W, None, rope_heads=4, head_dim=128)
    assert torch.equal(ops.unshuffle_weight(Ws, rope_heads=4, head_dim=128), W)
