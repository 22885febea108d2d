"""``shared`` prompt layout: a table's common prefix (header + context + transcript) is
prefilled once into a shared sequence whose KV blocks every knight references (refcounted),
and grouped decode reads them once. Same tokens as private per-knight caches, fewer blocks."""
import torch

from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
from theroundtaible_amd.engine.engine import group_order
from theroundtaible_amd.prompt import Prompt, Segment, build_turn_prompt_shared, TurnContext
from theroundtaible_amd.types import KnightConfig

KNIGHTS = [KnightConfig(name=n, adapter=f"local-llm-{n.lower()}", capabilities=["x"], priority=i + 1)
           for i, n in enumerate(["Claude", "Gemini", "GPT"])]


def _engine():
    return Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=512, weights="random:3"))


def _turns(transcript, rnd, key):
    ctx = TurnContext(topic="Gedeelde KV voor de ronde tafel " * 8)
    out = []
    for k in KNIGHTS:
        p = build_turn_prompt_shared(k, KNIGHTS, ctx, transcript, rnd, shared_key="t0@table")
        if key is None:
            p.shared_key = None
        out.append(Turn(k.name, p, SamplingParams(temperature=0.0, max_new_tokens=12, ignore_eos=True,
                                                  stop_on_consensus=False)))
    return out


def test_shared_layout_same_tokens_fewer_blocks():
    shared, private = _engine(), _engine()
    tr_s, tr_p = [], []
    fwd = shared.model.forward
    calls = []

    def counted(*a, **k):
        calls.append(a[3].kind)
        return fwd(*a, **k)
    shared.model.forward = counted
    for rnd in (1, 2, 3):
        calls.clear()
        a = shared.run_turns(_turns(tr_s, rnd, "t0"))
        # the shared span and the knights' own deltas are prefilled in ONE forward
        assert calls.count("prefill") == 1, calls
        b = private.run_turns(_turns(tr_p, rnd, None))
        for x, y in zip(a, b):
            assert x.error is None and y.error is None
            assert x.ids == y.ids
        for k, x in zip(KNIGHTS, a):
            tr_s += [Segment(f"\n\n### {k.name} (Ronde {rnd}):\n"), Segment(x.text, x.ids, shared.tokenizer.family)]
        for k, y in zip(KNIGHTS, b):
            tr_p += [Segment(f"\n\n### {k.name} (Ronde {rnd}):\n"), Segment(y.text, y.ids, private.tokenizer.family)]
        assert a[0].metrics["shared_tokens"] > 0 and b[0].metrics["shared_tokens"] == 0
    used_s = shared.kv.num_blocks - shared.kv.alloc.num_free
    used_p = private.kv.num_blocks - private.kv.alloc.num_free
    assert used_s < 0.6 * used_p, (used_s, used_p)
    # per round, the shared prefill is the new transcript once plus three short suffixes
    assert sum(x.metrics["prefill_tokens"] for x in a) < sum(y.metrics["prefill_tokens"] for y in b)


def test_attach_keeps_blocks_refcounted():
    e = _engine()
    e.run_turns(_turns([], 1, "t0"))
    sq = e.kv.seqs[e.shared_seq_key("t0@table")]
    full = sq.length // e.kv.block_size
    assert full > 0
    for k in KNIGHTS:
        s = e.kv.seqs[k.name]
        assert s.blocks[:full] == sq.blocks[:full]
    for b in sq.blocks[:full]:
        assert e.kv.alloc.ref[b] == 1 + len(KNIGHTS)
    # releasing the knights leaves the shared sequence intact
    for k in KNIGHTS:
        e.release(k.name)
    assert all(e.kv.alloc.ref[b] == 1 for b in sq.blocks[:full])


def test_group_order_makes_members_adjacent():
    assert group_order(["a", None, "b", "a", "b", None]) == [0, 3, 1, 2, 4, 5]
    assert group_order([None, None]) == [0, 1]


def test_lcp_matches_elementwise_scan():
    import random
    from theroundtaible_amd.engine.engine import lcp
    rng = random.Random(5)
    for _ in range(300):
        n = rng.randrange(0, 10000)
        a = [rng.randrange(3) for _ in range(n)]
        b = a[:rng.randrange(0, n + 1)] + [rng.randrange(3) for _ in range(rng.randrange(0, 40))]
        lim = rng.choice([None, rng.randrange(0, n + 2)])
        m, end = 0, min(len(a), len(b)) if lim is None else min(lim, len(a), len(b))
        while m < end and a[m] == b[m]:
            m += 1
        assert lcp(a, b, lim) == m and lcp(tuple(a), b, lim) == m


def test_encode_prompt_split_head_length():
    """The shared head's length is the sum of its segments' ids (pinned ids used as given),
    the same as encoding the head on its own."""
    e = _engine()
    for t in _turns([], 1, "t0") + _turns([], 2, "t0"):
        p = t.prompt
        p.segments.append(Segment("vastgezet", ids=[5, 6, 7], tokenizer=e.tokenizer.family))
        ids, n = e.encode_prompt_split(p)
        head = Prompt(list(p.segments[:p.shared_segments]), templated=True)
        want = len(e.encode_prompt(head)) + (len(e.tokenizer.chat_prefix or []) if not p.templated else 0)
        assert n == min(want, len(ids) - 1) and ids == e.encode_prompt(p)
        assert ids[-3:] == [5, 6, 7] or e.tokenizer.chat_suffix


def test_flag_fault_drops_the_shared_prefix_too():
    """an expired device wait ('flag' fault) during a shared-layout turn fails the
    turn AND frees the table's shared sequence (its all-reduced KV may be stale); the next turn
    prefills the shared prefix again instead of handing it to every member by LCP."""
    e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", num_blocks=512, weights="random:3",
                            faults={1: "flag"}))
    a = e.run_turns(_turns([], 1, "t0"))
    assert all(x.error is None for x in a)
    sk = e.shared_seq_key("t0@table")
    assert sk in e.kv.seqs and e.kv.seqs[sk].length > 0
    b = e.run_turns(_turns([], 1, "t0"))                      # call 1: injected poll expiry
    assert all(x.error is not None and x.error.kind == "device" for x in b)
    assert sk not in e.kv.seqs and sk not in e._shared_lru
    c = e.run_turns(_turns([], 1, "t0"))
    assert all(x.error is None for x in c)
    assert c[0].metrics["prefill_tokens"] >= e.kv.seqs[sk].length   # shared prefix prefilled again
    assert [x.ids for x in c] == [x.ids for x in a]


def test_lru_never_evicts_a_shared_key_of_the_current_batch():
    """with more distinct shared keys in one batch than MAX_SHARED_SEQS, the LRU
    must not free a shared sequence the same batch reserved before its members attached."""
    e = _engine()
    e.MAX_SHARED_SEQS = 2
    ctx = TurnContext(topic="LRU van gedeelde prefixen " * 6)
    turns = []
    for t in range(4):
        p = build_turn_prompt_shared(KNIGHTS[0], KNIGHTS, ctx, [], 1, shared_key=f"tafel{t}")
        turns.append(Turn(f"k{t}", p, SamplingParams(temperature=0.0, max_new_tokens=4, ignore_eos=True,
                                                     stop_on_consensus=False)))
    out = e.run_turns(turns)
    assert all(o.error is None for o in out)
    for t in range(4):          # every member still references live (allocated) blocks
        for blk in e.kv.seqs[f"k{t}"].blocks:
            assert e.kv.alloc.ref[blk] > 0


def test_warm_shared_reused_by_next_turn_and_fault_drops_it():
    """Engine.warm_shared (the C1-overlap speculative prefill): a predicted shared prefix is
    prefilled ahead of the turn and the turn keeps it by LCP (same tokens as without the warm-up,
    fewer turn-time prefill tokens); a device fault during the warm-up drops the shared sequence
    and flags the engine for recovery instead of leaving half-written KV for the LCP to reuse."""
    from theroundtaible_amd.prompt import Segment
    a, b = _engine(), _engine()
    tr = [Segment("\n\n### Claude (Ronde 1):\n"), Segment("Een eerste antwoord over gedeelde KV " * 4)]
    turns_a, turns_b = _turns(tr, 2, "t0"), _turns(tr, 2, "t0")
    n = a.warm_shared(turns_a[0].prompt)
    assert n > 0 and a.stats["speculative_tokens"] == n
    out_a = a.run_turns(turns_a)
    out_b = b.run_turns(turns_b)
    assert [o.ids for o in out_a] == [o.ids for o in out_b]
    assert a.stats["speculative_kept"] == n
    pre_a = sum(o.metrics["prefill_tokens"] for o in out_a)
    pre_b = sum(o.metrics["prefill_tokens"] for o in out_b)
    assert pre_a == pre_b - n
    # fault during a warm-up
    c = _engine()

    def boom(*args, **kw):
        raise RuntimeError("HIP error: injected fault in the speculative prefill")
    c.prefill_reserved = boom
    assert c.warm_shared(_turns(tr, 2, "t0")[0].prompt) == 0
    assert c.shared_seq_key("t0@table") not in c.kv.seqs and not c.healthy
