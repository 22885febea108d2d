"""Engine on the GPU: HIP path vs CPU reference, hipGraph decode vs eager, resident-KV reuse."""
import pytest
import torch

from theroundtaible_amd import ops
from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
from theroundtaible_amd.prompt import Prompt

pytestmark = pytest.mark.gpu

GREEDY = SamplingParams(temperature=0.0, max_new_tokens=24, ignore_eos=True, stop_on_consensus=False)


def eng(model="tiny-llama-128", **kw):
    cfg = dict(model=model, weights="random-full:3", device="cuda:0", num_blocks=512)
    cfg.update(kw)
    return Engine(EngineConfig(**cfg))


@pytest.mark.parametrize("model", ["tiny-llama-128", "tiny-llama", "tiny-gpt2"])
def test_prefill_logits_match_cpu(model):
    g = eng(model, use_graphs=False)
    c = Engine(EngineConfig(model=model, weights="random-full:3", device="cpu", dtype="fp32", num_blocks=512))
    ids = g.encode_prompt("De ridders van de ronde tafel bespreken de architectuur van de cache-laag. " * 3)
    lg = g.prefill([(g.kv.seq("a"), ids)]).float().cpu()
    lc = c.prefill([(c.kv.seq("a"), ids)]).float()
    cos = torch.nn.functional.cosine_similarity(lg, lc, dim=-1)
    assert float(cos.min()) > 0.99


def test_graph_decode_equals_eager():
    a = eng(use_graphs=True)
    b = eng(use_graphs=False)
    p = "Hallo tafel, wat is het plan voor vandaag?"
    ta = a.run_turns([Turn("K1", p, GREEDY), Turn("K2", p + " Anders.", GREEDY)])
    tb = b.run_turns([Turn("K1", p, GREEDY), Turn("K2", p + " Anders.", GREEDY)])
    assert [t.ids for t in ta] == [t.ids for t in tb]
    assert ops.native_available()


def test_graph_decode_pipelined_stop(monkeypatch):
    """graphs.DecodeGraph.run checks stops one chunk behind the replays (pinned async copies):
    a stop condition met at 40 tokens ends the turn at the first checked chunk past it (49
    tokens with sync_every 32), with the same tokens as an uninterrupted decode."""
    import theroundtaible_amd.engine.engine as em
    monkeypatch.setattr(em, "_finished", lambda out, params, eos, tok: len(out) >= 40)
    sp = SamplingParams(temperature=0.0, max_new_tokens=200, ignore_eos=False, stop_on_consensus=False)
    a = eng(use_graphs=True)
    p = "Hallo tafel, wat is het plan voor vandaag?"
    ta = a.run_turns([Turn("K1", p, sp), Turn("K2", p + " Anders.", sp)])
    monkeypatch.setattr(em, "_finished", lambda out, params, eos, tok: False)
    tb = eng(use_graphs=True).run_turns([Turn("K1", p, sp), Turn("K2", p + " Anders.", sp)])
    for x, y in zip(ta, tb):
        assert x.error is None and len(x.ids) <= 49
        assert x.ids == y.ids[:len(x.ids)]
    assert max(len(x.ids) for x in ta) == 49 or any(len(y.ids) < 49 for y in tb)
    # the engine keeps serving after the discarded extra replays
    tc = a.run_turns([Turn("K1", p, GREEDY)])
    assert tc[0].error is None


def test_resident_kv_reuse_matches_fresh():
    a = eng()
    p = "Onderwerp: caching."
    t1 = a.run_turns([Turn("K", p, GREEDY)])[0]
    p2 = Prompt().add(p).add(t1.text, t1.ids, a.tokenizer.family).add(" Reactie van de andere knight.")
    t2 = a.run_turns([Turn("K", p2, GREEDY)])[0]
    assert t2.metrics["reused_tokens"] >= len(a.encode_prompt(p))
    fresh = eng().run_turns([Turn("K", p2, GREEDY)])[0]
    # The resident path computed the response's K/V with the decode kernels (fused MFMA GEMMs),
    # the fresh path with the prefill kernels (hipBLASLt + K1/K4): equal math, different bf16
    # rounding order, so greedy streams agree for a while and may then diverge on a near-tie.
    assert fresh.ids[:4] == t2.ids[:4]


def test_sampling_deterministic_per_knight_position():
    sp = SamplingParams(temperature=0.8, top_p=0.9, max_new_tokens=16, ignore_eos=True, stop_on_consensus=False,
                        seed=5)
    a = eng().run_turns([Turn("K1", "abc", sp), Turn("K2", "abc", sp)])
    b = eng().run_turns([Turn("K2", "abc", sp)])
    assert a[1].ids == b[0].ids      # batching does not change a knight's stream
    assert a[0].ids != a[1].ids      # different knights differ


def test_long_context_split_decode():
    a = eng(num_blocks=1024)
    long = "token " * 3000
    out = a.run_turns([Turn("K", long, GREEDY)])[0]
    assert len(out.ids) == GREEDY.max_new_tokens
    b = eng(num_blocks=1024, use_graphs=False)
    out2 = b.run_turns([Turn("K", long, GREEDY)])[0]
    assert out.ids == out2.ids


def test_serve_on_gpu_batches_requests():
    import json
    import threading
    import urllib.request
    from theroundtaible_amd.serve import build_server
    srv = build_server("tiny-llama-128", weights="random:2", device="cuda:0", port=0, max_batch=4, max_tokens=8,
                       num_blocks=512).start()
    try:
        codes = []

        def go(i):
            req = urllib.request.Request(srv.url + "/v1/chat/completions", method="POST",
                                         headers={"Content-Type": "application/json"},
                                         data=json.dumps({"messages": [{"role": "user", "content": f"q{i}"}],
                                                          "max_tokens": 8}).encode())
            with urllib.request.urlopen(req, timeout=120) as r:
                codes.append((r.status, json.loads(r.read())["usage"]["completion_tokens"]))
        ts = [threading.Thread(target=go, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert codes == [(200, 8)] * 4
        assert srv.engine.graphs   # decode ran through captured hipGraphs
    finally:
        srv.close()


def test_serve_on_gpu_shared_system_prompt_grouped_decode():
    """Concurrent clients with one system prompt: its KV is resident once, and their batched
    decode runs the grouped (shared-prefix) hipGraph."""
    import json
    import threading
    import urllib.request
    from theroundtaible_amd.serve import build_server
    srv = build_server("tiny-llama-128", weights="random:2", device="cuda:0", port=0, max_batch=4, max_tokens=8,
                       num_blocks=512).start()
    sys_prompt = "Een lange gedeelde systeemprompt voor alle clients. " * 30
    try:
        codes = []

        def go(i):
            req = urllib.request.Request(srv.url + "/v1/chat/completions", method="POST",
                                         headers={"Content-Type": "application/json"},
                                         data=json.dumps({"messages": [{"role": "system", "content": sys_prompt},
                                                                       {"role": "user", "content": f"q{i}"}],
                                                          "max_tokens": 8, "user": f"u{i}"}).encode())
            with urllib.request.urlopen(req, timeout=120) as r:
                codes.append(r.status)
        ts = [threading.Thread(target=go, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert codes == [200] * 4
        assert any(k.startswith("@shared:sys:") for k in srv.engine.kv.seqs)
        assert any(key[2] for key in srv.engine.graphs)          # a grouped decode graph was used
    finally:
        srv.close()


def test_debug_paging_guard_in_decode_graph():
    """ROUNDTABLE_DEBUG_CHECKS: the captured step validates its own paging metadata on the device.
    Normal decoding never trips it; corrupted graph state does, at the next host sync point."""
    e = eng(use_graphs=True, debug_checks=True)
    p = "Hallo tafel, wat is het plan voor vandaag?"
    out = e.run_turns([Turn("K1", p, GREEDY), Turn("K2", p + " Anders.", GREEDY)])
    assert all(len(t.ids) == GREEDY.max_new_tokens for t in out)
    g = next(iter(e.graphs.values()))
    assert int(g.guard_err.item()) == 0
    # a length one past the position: every kernel still reads valid (allocated or scratch)
    # blocks, so the replay is safe, but the guard must flag the inconsistency (code 8)
    g.ctx_lens.add_(1)
    g.graph.replay()
    with pytest.raises(AssertionError, match="position"):
        g.check_guard()
    assert int(g.guard_err.item()) == 0           # cleared after reporting


def _shared_turns(transcript, rnd, keyed=True, n_new=16):
    from theroundtaible_amd.prompt import TurnContext, build_turn_prompt_shared
    from theroundtaible_amd.types import KnightConfig
    ks = [KnightConfig(name=n, adapter="local-llm", capabilities=["x"], priority=i) for i, n in
          enumerate(["Claude", "Gemini", "GPT"])]
    ctx = TurnContext(topic="Gedeelde KV-blokken voor alle knights van een tafel. " * 40)
    out = []
    for k in ks:
        p = build_turn_prompt_shared(k, ks, ctx, transcript, rnd, shared_key="t@table")
        if not keyed:
            p.shared_key = None
        out.append(Turn(k.name, p, SamplingParams(temperature=0.0, max_new_tokens=n_new, ignore_eos=True,
                                                  stop_on_consensus=False)))
    return ks, out


@pytest.mark.parametrize("model", ["tiny-llama-128", "llama3-8b-2l"])
def test_shared_prefix_grouped_decode_matches_private(model):
    """One decode step over resident KV whose prefix blocks are shared by 3 knights: grouped K3
    (shared blocks read once for the group) vs every sequence alone — same logits."""
    from theroundtaible_amd.models.llama import AttnMeta
    from theroundtaible_amd.prompt import Segment
    kw = {"model_overrides": {"n_layers": 2}} if model == "llama3-8b-2l" else {}
    e = eng("llama3-8b" if model == "llama3-8b-2l" else model, num_blocks=2048, **kw)
    ks, turns = _shared_turns([], 1)
    outs = e.run_turns(turns)
    tr = []
    for k, o in zip(ks, outs):
        assert o.error is None and o.metrics["shared_tokens"] > 0
        tr += [Segment(f"\n\n### {k.name} (Ronde 1):\n"), Segment(o.text, o.ids, e.tokenizer.family)]
    ks, turns = _shared_turns(tr, 2)
    outs = e.run_turns(turns)
    assert all(o.error is None for o in outs)
    seqs = [e.kv.seqs[k.name] for k in ks]
    sq = e.kv.seqs[e.shared_seq_key("t@table")]
    from theroundtaible_amd.engine.engine import common_blocks
    nsh = min(common_blocks(s, sq) for s in seqs)
    assert nsh >= 4
    B = len(seqs)
    dev = e.device
    bt = torch.zeros(B, max(len(s.blocks) for s in seqs) + 1, dtype=torch.int32)
    for j, s in enumerate(seqs):
        e.kv.ensure_capacity(s, s.length + 1)
        bt[j, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
    pos = [s.length for s in seqs]
    slots = [s.blocks[p // 32] * 32 + p % 32 for s, p in zip(seqs, pos)]
    splits = ops.decode_splits(3, e.model.n_kv_heads)
    G = e.model.n_heads // e.model.n_kv_heads
    ids = torch.tensor([o.ids[-1] for o in outs], dtype=torch.int64, device=dev)
    res = []
    for grouped in (False, True):
        gt = e.group_table((["t"] * B, [nsh] * B), B).to(dev) if grouped else None
        ws = ops.DecodeWorkspace(B, e.model.n_heads, e.cfg.head_dim, splits, dev,
                                 max_group=16 // G if grouped else 1)
        meta = AttnMeta(kind="decode", slot_mapping=torch.tensor(slots, dtype=torch.int64, device=dev),
                        block_tables=bt.to(dev), ctx_lens=torch.tensor([p + 1 for p in pos], dtype=torch.int32,
                                                                      device=dev),
                        num_splits=splits, workspace=ws, groups=gt)
        res.append(e.model.forward(ids, torch.tensor(pos, dtype=torch.int64, device=dev), e.kv, meta).float())
    cos = torch.nn.functional.cosine_similarity(res[0], res[1], dim=-1)
    assert float(cos.min()) > 0.999, cos


def test_shared_layout_graph_equals_eager():
    """Grouped decode in the captured hipGraph and eagerly: identical greedy tokens."""
    a = eng(use_graphs=True)
    b = eng(use_graphs=False)
    _, ta = _shared_turns([], 1)
    _, tb = _shared_turns([], 1)
    oa, ob = a.run_turns(ta), b.run_turns(tb)
    assert [o.ids for o in oa] == [o.ids for o in ob]
    assert all(o.metrics["shared_tokens"] > 0 for o in oa)


def test_heterogeneous_engines_share_gpu_concurrently():
    """Two different models on one GPU: the pool splits the free HBM between their KV pools
    after both loaded, and each engine runs on its own HIP stream from its own host thread —
    same greedy tokens as running them one after the other."""
    from concurrent.futures import ThreadPoolExecutor
    from theroundtaible_amd.knights.engine_backend import EnginePool
    pool = EnginePool()
    cfgs = [EngineConfig(model=m, weights="random-full:3", device="cuda:0", max_kv_tokens=1 << 20)
            for m in ("tiny-llama-128", "tiny-llama")]
    engines = [pool.get(c, defer_kv=True)[0] for c in cfgs]
    assert not any(e.kv_allocated for e in engines)
    caps = pool.finalize()["cuda:0"]
    assert len(caps) == 2 and all(c > 0 for c in caps)
    assert engines[0].stream is not None and engines[0].stream != engines[1].stream
    p = "Twee modellen, een GPU, twee streams. " * 6
    solo = [e.run_turns([Turn("k", p, GREEDY)])[0].ids for e in engines]
    for e in engines:
        e.release("k")
    with ThreadPoolExecutor(2) as ex:
        both = list(ex.map(lambda e: e.run_turns([Turn("k", p, GREEDY)])[0].ids, engines))
    assert both == solo


def test_simulated_tp_device_collectives_cost_their_latency_in_a_graph():
    """``bench.py --simulate-tp N --sim-k9-us X`` (round 5): every simulated collective is a kernel
    holding the K9 launch's CUs for X µs INSIDE the captured graph (csrc/oneshot_ar.hip
    sim_comm_spin), calibrated so a call costs X µs there. 20 all-reduces at 20 µs must add
    ~400 µs to a replay; with the stand-in off they cost nothing; values pass through unchanged."""
    from theroundtaible_amd.parallel.tp import SimulatedTP
    x = torch.randn(3, 4096, device="cuda").to(torch.bfloat16)
    ref = x.clone()

    def replay_us(tp, calls=20):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(calls):
                tp.all_reduce(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(calls):
                tp.all_reduce(x)
        g.replay()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b) * 1e3)
        return best

    on = SimulatedTP(8, comm_us=20.0)
    on.calibrate_stand_in()
    t_on = replay_us(on)
    assert 0.85 * 400 < t_on < 1.25 * 400, t_on
    off = SimulatedTP(8)
    for _ in range(5):
        off.all_reduce(x)                 # the identity: no stand-in launch at all
    assert getattr(off, "sim_comm_calls", 0) == 0 and getattr(on, "sim_comm_calls", 0) > 0
    assert torch.equal(x, ref)
    g = on.all_gather_last(x[:, :512].contiguous())
    assert g.shape == (3, 4096) and torch.equal(g[:, 512:1024], x[:, :512])
