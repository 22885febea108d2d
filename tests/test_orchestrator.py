"""Round engine behaviour with scripted knights (the mock adapter the reference never had)."""
import json
import os

import pytest

from theroundtaible_amd import store
from theroundtaible_amd.knights.fake import FakeBackend, consensus_reply
from theroundtaible_amd.orchestrator import (Orchestrator, RunOptions, compute_allowed_files,
                                             run_tables_parallel, run_tables_sequential, select_lead_knight)
from theroundtaible_amd.types import ConsensusBlock, ContinueOptions, KnightConfig, RoundtableConfig


def config(n=3, max_rounds=3, threshold=9, mode="sequential", layout="reference", fallback=None):
    names = ["Claude", "Gemini", "GPT"][:n]
    knights = [{"name": k, "adapter": f"fake-{k.lower()}", "capabilities": ["x"], "priority": i + 1}
               for i, k in enumerate(names)]
    if fallback:
        knights[0]["fallback"] = fallback
    return RoundtableConfig.from_dict({
        "version": "1.0", "project": "p", "language": "nl", "knights": knights,
        "rules": {"max_rounds": max_rounds, "consensus_threshold": threshold, "timeout_per_turn_seconds": 5,
                  "escalate_to_user_after": 2, "auto_execute": False, "ignore": [".git"],
                  "round_mode": mode, "prompt_layout": layout},
        "chronicle": ".roundtable/chronicle.md", "adapter_config": {}})


def backends(scripts, faults=None, **kw):
    return {f"fake-{k.lower()}": FakeBackend(name=k, script={k: v}, faults=(faults or {}).get(k), **kw)
            for k, v in scripts.items()}


@pytest.fixture(autouse=True)
def _cwd(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)


def test_consensus_round_one(tmp_path):
    cfg = config()
    sc = {k: [consensus_reply(9 + (k == "GPT"), f"{k} is akkoord.", proposal=f"plan van {k}",
                              files_to_modify=["src/a.ts", f"NEW:src/{k}.ts"])] for k in ("Claude", "Gemini", "GPT")}
    res = Orchestrator(cfg, backends(sc), str(tmp_path), options=RunOptions(shuffle_seed=1)).run("Onderwerp")
    assert res.consensus and res.rounds == 1 and not res.unanimous_rejection
    assert res.decision == "plan van GPT"          # latest proposal
    assert res.lead_knight == "GPT"                # top scorer of the last round
    st = store.read_status(res.session_path)
    assert st["phase"] == "consensus_reached" and st["consensus_reached"] and st["round"] == 1
    assert st["allowed_files"] == ["src/a.ts", "NEW:src/Claude.ts", "NEW:src/Gemini.ts", "NEW:src/GPT.ts"]
    chron = open(tmp_path / ".roundtable" / "chronicle.md").read()
    assert "Consensus in 1 round(s). Lead Knight: GPT." in chron
    assert open(os.path.join(res.session_path, "decisions.md")).read().endswith("plan van GPT\n")
    # knight default in blocks is the backend name
    assert [b.knight for b in res.blocks] == ["Claude", "Gemini", "GPT"]
    assert len(store.load_round_entries(res.session_path)) == 3


def test_negative_consensus(tmp_path):
    sc = {k: [consensus_reply(2, f"{k}: slecht idee")] for k in ("Claude", "Gemini", "GPT")}
    res = Orchestrator(config(), backends(sc), str(tmp_path)).run("Slecht")
    assert res.consensus and res.unanimous_rejection and res.rounds == 1
    assert res.decision.startswith("## Claude\n\nClaude: slecht idee")
    assert "Unanimous rejection in 1 round(s)." in open(tmp_path / ".roundtable" / "chronicle.md").read()


def test_escalation_then_send_back(tmp_path):
    sc = {"Claude": [consensus_reply(9)] * 10, "Gemini": [consensus_reply(5)] * 2 + [consensus_reply(9)] * 5}
    cfg = config(n=2, max_rounds=2)
    orch = Orchestrator(cfg, backends(sc), str(tmp_path), options=RunOptions(shuffle_seed=3))
    res = orch.run("T")
    assert not res.consensus and res.rounds == 2
    assert store.read_status(res.session_path)["phase"] == "escalated"
    cont = ContinueOptions(res.session_path, res.all_rounds, res.rounds + 1)
    res2 = orch.run("T", cont)
    assert res2.consensus and res2.rounds == 3 and res2.session_path == res.session_path
    prompts = orch.backends["fake-gemini"].prompts
    assert "THE KING HAS SENT YOU BACK" in prompts[-1][1]


def test_latest_blocks_persist_across_crash(tmp_path):
    sc = {"Claude": [consensus_reply(9), consensus_reply(9)], "Gemini": [consensus_reply(9), "x"]}
    faults = {"Gemini": {("Gemini", 1): "raise:boom"}}
    res = Orchestrator(config(n=2, max_rounds=2, threshold=10), backends(sc, faults), str(tmp_path)).run("T")
    # Gemini crashed in round 2 but keeps its round-1 block
    assert {b.knight: b.round for b in res.blocks} == {"Claude": 2, "Gemini": 1}
    assert [e.knight for e in res.all_rounds] == ["Claude", "Gemini", "Claude"] or len(res.all_rounds) == 3


def test_visibility_sequential_vs_parallel(tmp_path):
    sc = {k: [consensus_reply(5, f"TOKEN_{k}_R{r}") for r in (1, 2)] for k in ("Claude", "Gemini")}
    b = backends(sc)
    Orchestrator(config(n=2, max_rounds=1), b, str(tmp_path)).run("T")
    # sequential: Gemini (priority 2) sees Claude's round-1 turn
    assert "TOKEN_Claude_R1" in b["fake-gemini"].prompts[0][1]
    b2 = backends(sc)
    Orchestrator(config(n=2, max_rounds=1, mode="parallel"), b2, str(tmp_path)).run("T")
    assert "TOKEN_Claude_R1" not in b2["fake-gemini"].prompts[0][1]


def test_tools_feed_later_prompts(tmp_path):
    (tmp_path / "src").mkdir()
    (tmp_path / "src" / "a.py").write_text("print('hi')\n")
    sc = {"Claude": [consensus_reply(5, file_requests=["src/a.py"], verify_commands=["ls src"])] * 2,
          "Gemini": [consensus_reply(5)] * 2}
    b = backends(sc)
    res = Orchestrator(config(n=2, max_rounds=1), b, str(tmp_path)).run("T")
    g = b["fake-gemini"].prompts[0][1]
    assert "OPGEVRAAGDE BESTANDEN" in g and "print('hi')" in g
    assert "VERIFICATIE RESULTATEN" in g and "### VERIFY: ls src\n```\na.py\n```" in g
    assert res.resolved_files.startswith("### src/a.py")


def test_runtime_fallback_and_missing_adapter(tmp_path):
    cfg = config(n=3, max_rounds=1, fallback="fake-backup")
    sc = {"Claude": [consensus_reply(9)], "Gemini": [consensus_reply(9)]}
    b = backends(sc, faults={"Claude": {("Claude", 0): "raise:usage limit 429"}})
    created = []

    def factory(aid):
        fb = FakeBackend(name="Backup", script={"Claude": [consensus_reply(9, "backup spreekt")]})
        created.append(fb)
        return fb

    res = Orchestrator(cfg, b, str(tmp_path), backend_factory=factory).run("T")
    assert created and "backup spreekt" in res.all_rounds[0].response
    assert "__fallback_Claude" in b
    assert [e.knight for e in res.all_rounds] == ["Claude", "Gemini"]   # GPT has no backend: "didn't show up"


def test_timeout_is_skipped(tmp_path):
    sc = {"Claude": [consensus_reply(9)], "Gemini": [consensus_reply(9)]}
    b = backends(sc, faults={"Gemini": {("Gemini", 0): "hang"}})
    res = Orchestrator(config(n=2, max_rounds=1), b, str(tmp_path)).run("T")
    assert [e.knight for e in res.all_rounds] == ["Claude"]
    assert res.consensus  # Claude's block alone satisfies "every latest block >= threshold"


def test_seeded_shuffle_is_deterministic(tmp_path):
    sc = {k: [consensus_reply(5)] * 5 for k in ("Claude", "Gemini", "GPT")}
    orders = []
    for _ in range(2):
        res = Orchestrator(config(max_rounds=4), backends(sc), str(tmp_path), options=RunOptions(shuffle_seed=42)).run("T")
        orders.append([e.knight for e in res.all_rounds])
    assert orders[0] == orders[1]
    assert orders[0][:3] == ["Claude", "Gemini", "GPT"]   # round 1: priority order


def test_append_layout_prompts_grow_append_only(tmp_path):
    sc = {k: [consensus_reply(5, f"{k} ronde {r}") for r in (1, 2, 3)] for k in ("Claude", "Gemini")}
    b = backends(sc)
    Orchestrator(config(n=2, max_rounds=3, layout="append", mode="parallel"), b, str(tmp_path),
                 options=RunOptions(shuffle_seed=0)).run("T")
    ps = [p for k, p in b["fake-claude"].prompts]
    for prev, nxt in zip(ps, ps[1:]):
        assert nxt.startswith(prev[: prev.rindex("### Claude (Ronde")])


def test_lead_knight_and_allowed_files():
    ks = [KnightConfig("A", "a", [], 2), KnightConfig("B", "b", [], 1)]
    blocks = [ConsensusBlock("A", 2, 10), ConsensusBlock("B", 2, 10), ConsensusBlock("B", 1, 3)]
    assert select_lead_knight(ks, blocks).name == "B"
    assert select_lead_knight(ks, []).name == "B"
    assert compute_allowed_files([ConsensusBlock("A", 1, 9, files_to_modify=["x", "y"]),
                                  ConsensusBlock("B", 1, 9, files_to_modify=["y", "NEW:z"])]) == ["x", "y", "NEW:z"]


def test_run_tables_lockstep(tmp_path):
    tabs = []
    for t in range(2):
        sc = {k: [consensus_reply(9 if t == 0 else 4)] * 3 for k in ("Claude", "Gemini")}
        tabs.append(Orchestrator(config(n=2, max_rounds=3, mode="parallel"), backends(sc), str(tmp_path),
                                 options=RunOptions(shuffle_seed=t)))
    res = run_tables_parallel(tabs, ["A", "B"])
    assert res[0].consensus and res[0].rounds == 1
    assert not res[1].consensus and res[1].rounds == 3


def test_run_tables_sequential_lockstep_matches_single_table_runs(tmp_path):
    """Lockstep sequential tables == each table run alone (same visibility, same decisions)."""
    def make(t):
        sc = {k: [consensus_reply(9 if t == 0 else 4)] * 3 for k in ("Claude", "Gemini", "GPT")}
        return Orchestrator(config(n=3, max_rounds=3, mode="sequential"), backends(sc), str(tmp_path),
                            options=RunOptions(shuffle_seed=t))
    res = run_tables_sequential([make(0), make(1)], ["A", "B"])
    assert res[0].consensus and res[0].rounds == 1
    assert not res[1].consensus and res[1].rounds == 3
    alone = make(1).run("B")
    assert alone.rounds == res[1].rounds and alone.consensus == res[1].consensus


def test_sequential_visibility_within_round(tmp_path):
    """Sequential mode: the second speaker's prompt contains the first speaker's reply."""
    seen = {}

    class Spy(FakeBackend):
        def _run(self, req, timeout_s):
            seen[self.name] = str(req.prompt)
            return super()._run(req, timeout_s)
    sc = {"Claude": ["EERSTE-ANTWOORD-XYZ"], "Gemini": ["tweede"]}
    bk = {f"fake-{k.lower()}": Spy(name=k, script={k: v}) for k, v in sc.items()}
    o = Orchestrator(config(n=2, max_rounds=1, mode="sequential"), bk, str(tmp_path))
    run_tables_sequential([o], ["T"])
    assert "EERSTE-ANTWOORD-XYZ" in seen["Gemini"] and "EERSTE-ANTWOORD-XYZ" not in seen["Claude"]


@pytest.mark.parametrize("mode", ["parallel", "sequential"])
def test_shared_layout_prompts_share_a_growing_prefix(tmp_path, mode):
    """`shared` layout: every knight's prompt of a round starts with the same shared segments
    (header + context + transcript), each ends in a one-line suffix naming the speaker, and the
    shared prefix only grows across rounds (pure append for the engine's shared sequence)."""
    sc = {k: [consensus_reply(5, f"{k} ronde {r}") for r in (1, 2, 3)] for k in ("Claude", "Gemini", "GPT")}
    b = backends(sc)
    Orchestrator(config(n=3, max_rounds=3, layout="shared", mode=mode), b, str(tmp_path),
                 options=RunOptions(shuffle_seed=0)).run("T")
    shared = []
    for k in ("Claude", "Gemini", "GPT"):
        for req_prompt in [p for _, p in b[f"fake-{k.lower()}"].prompt_objs]:
            assert req_prompt.shared_key and req_prompt.shared_segments > 0
            head = "".join(s.text for s in req_prompt.segments[:req_prompt.shared_segments])
            tail = "".join(s.text for s in req_prompt.segments[req_prompt.shared_segments:])
            assert f"jij bent {k}" in tail and len(tail) < 200
            shared.append(head)
    by_len = sorted(set(shared), key=len)
    for a, c in zip(by_len, by_len[1:]):
        assert c.startswith(a)                     # one growing prefix for the whole table
    if mode == "parallel":                         # a round's three prompts share the same prefix
        assert len(set(shared)) == 3


def test_shared_layout_continuation_keeps_prefix(tmp_path):
    """King's send-back with the shared layout: the continuation's prompts extend the first
    session's shared prefix (transcript + KING demand), so the engine re-prefills only the delta."""
    sc = {k: [consensus_reply(4)] * 4 for k in ("Claude", "Gemini")}
    b = backends(sc)
    o = Orchestrator(config(n=2, max_rounds=1, layout="shared", mode="parallel"), b, str(tmp_path),
                     options=RunOptions(shuffle_seed=0))
    res = o.run("T")
    first = [p for _, p in b["fake-claude"].prompt_objs][-1]
    cont = ContinueOptions(res.session_path, res.all_rounds, res.rounds + 1)
    o.run("T", continue_from=cont)
    nxt = [p for _, p in b["fake-claude"].prompt_objs][-1]
    h1 = "".join(s.text for s in first.segments[:first.shared_segments])
    h2 = "".join(s.text for s in nxt.segments[:nxt.shared_segments])
    assert h2.startswith(h1) and "THE KING HAS SENT YOU BACK" in h2[len(h1):]


def test_mirror_orchestrator_writes_nothing_and_decides_the_same(tmp_path):
    """RunOptions(persist=False): an SPMD rank's mirror of a table another rank persists drops
    every session / chronicle write but reaches the same decision from the same replies."""
    sc = {k: [consensus_reply(6, f"{k} twijfelt."), consensus_reply(9, f"{k} is akkoord.", proposal=f"plan {k}")]
          for k in ("Claude", "Gemini", "GPT")}
    a = Orchestrator(config(), backends(sc), str(tmp_path / "a"), options=RunOptions(shuffle_seed=3)).run("Spiegel")
    os.makedirs(tmp_path / "b")
    b = Orchestrator(config(), backends(sc), str(tmp_path / "b"),
                     options=RunOptions(shuffle_seed=3, persist=False)).run("Spiegel")
    assert (a.consensus, a.rounds, a.decision, a.lead_knight) == (b.consensus, b.rounds, b.decision, b.lead_knight)
    assert os.path.isdir(a.session_path) and b.session_path == "<mirror>"
    assert os.listdir(tmp_path / "b") == []
