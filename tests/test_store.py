"""On-disk formats: sessions, discussion/decisions, chronicle, manifest, decrees, keys."""
import json
import os

import pytest

from theroundtaible_amd import store
from theroundtaible_amd.store import chronicle as chron
from theroundtaible_amd.store import keys
from theroundtaible_amd.types import UNDEFINED, ConsensusBlock, RoundEntry
from theroundtaible_amd.utils.atomic import SessionLock

NOW = "2026-10-15T21:07:03.456Z"


@pytest.fixture(autouse=True)
def fixed_now(monkeypatch):
    monkeypatch.setenv("ROUNDTABLE_FAKE_NOW", NOW)


def test_slug_and_session_layout(tmp_path):
    assert store.slugify("  Hoe moeten we -- de DB schema's bouwen?! ") == "hoe-moeten-we-de-db-schema-s-bouwen"
    assert len(store.slugify("x" * 80)) == 50
    p = store.create_session(str(tmp_path), "DB schema?")
    assert os.path.basename(p) == "2026-10-15-2107-db-schema"
    assert open(os.path.join(p, "topic.md")).read() == "# Topic\n\nDB schema?\n"
    st = json.load(open(os.path.join(p, "status.json")))
    assert list(st) == ["phase", "current_knight", "round", "consensus_reached", "started_at", "updated_at"]
    assert st["phase"] == "discussing" and st["current_knight"] is None and st["started_at"] == NOW


def test_status_merge_and_undefined(tmp_path):
    p = store.create_session(str(tmp_path), "t")
    store.update_status(p, phase="consensus_reached", allowed_files=["a"], round=2)
    st = store.read_status(p)
    assert st["allowed_files"] == ["a"] and st["round"] == 2
    store.update_status(p, allowed_files=UNDEFINED)
    assert "allowed_files" not in store.read_status(p)
    raw = open(os.path.join(p, "status.json")).read()
    assert raw.startswith('{\n  "phase": "consensus_reached"')


def entries():
    return [RoundEntry("Claude", 1, "Eerste.", ConsensusBlock("Claude", 1, 8, ["plan"], ["risico"]), NOW),
            RoundEntry("GPT", 1, "Tweede.", None, NOW)]


def test_discussion_golden():
    expected = ("# Discussion\n\n## Round 1 — Claude\n*" + NOW + "*\n\nEerste.\n\n**Consensus:**\n- Score: 8/10\n"
                "- Agrees with: plan\n- Pending: risico\n\n---\n\n## Round 1 — GPT\n*" + NOW + "*\n\nTweede.\n\n\n---\n")
    assert store.render_discussion(entries()) == expected


def test_decisions_golden():
    got = store.render_decisions("Topic X", "Doe het zo.", entries())
    assert got == ("# Decision\n\n**Topic:** Topic X\n**Knights:** Claude, GPT\n**Rounds:** 2\n"
                   "**Date:** 2026-10-15\n\n---\n\nDoe het zo.\n")


def test_chronicle_headers_and_entry(tmp_path):
    root = str(tmp_path)
    store.append_to_chronicle(root, ".roundtable/chronicle.md", topic="T", outcome="Consensus in 1 round(s).",
                              knights=["A", "B"], date="2026-10-15")
    c = store.read_chronicle(root, ".roundtable/chronicle.md")
    assert c == chron.APPEND_HEADER + "## 2026-10-15 — T\n\n**Knights:** A, B\n\nConsensus in 1 round(s).\n\n---\n"
    assert store.read_chronicle(root, "nope.md") == ""


def test_manifest(tmp_path):
    root = str(tmp_path)
    assert store.manifest_summary(store.read_manifest(root)) == "No implementation history yet."
    (tmp_path / "a.ts").write_text("x")
    store.add_manifest_entry(root, {"id": "f1", "session": "s", "status": "implemented",
                                    "files": ["a.ts", "b.ts", "c.ts", "d.ts"], "summary": "S1",
                                    "applied_at": NOW, "lead_knight": "Claude"})
    store.add_manifest_entry(root, {"id": "f2", "session": "s", "status": "partial", "files": ["a.ts"],
                                    "files_skipped": ["z.ts"], "summary": "S2", "applied_at": NOW, "lead_knight": "GPT"})
    summ = store.manifest_summary(store.read_manifest(root))
    assert summ.split("\n") == ["- [~] f2 — S2 (a.ts)", "- [+] f1 — S1 (a.ts, b.ts, c.ts +1 more)"]
    assert store.check_manifest(root) == ['f1: "b.ts" no longer exists on disk (stale entry)',
                                          'f1: "c.ts" no longer exists on disk (stale entry)',
                                          'f1: "d.ts" no longer exists on disk (stale entry)']
    assert store.deprecate_feature(root, "f1", "f2")
    assert not store.deprecate_feature(root, "nope")
    m = store.read_manifest(root)
    assert m["features"][0]["status"] == "deprecated" and m["features"][0]["replaced_by"] == "f2"
    assert store.check_manifest(root) == []
    assert store.topic_to_feature_id("Add JWT auth! (v2)  now") == "add-jwt-auth-v2-now"


def test_decree_log(tmp_path):
    root = str(tmp_path)
    assert store.format_decrees_for_prompt([]) == ""
    for i in range(7):
        store.add_decree_entry(root, "deferred" if i % 2 else "rejected_no_apply", f"s{i}", "T" * (60 if i == 6 else 5),
                               "" if i == 0 else f"r{i}")
    log = store.read_decree_log(root)
    assert [e["id"] for e in log["entries"]] == [f"decree-{i:03d}" for i in range(1, 8)]
    assert log["entries"][0]["reason"] == "No reason provided"
    act = store.active_decrees(log)
    assert len(act) == 5 and act[0]["id"] == "decree-003"
    txt = store.format_decrees_for_prompt(act)
    assert txt.startswith("KING'S DECREES")
    assert '- [decree-007] REJECTED_NO_APPLY — "' + "T" * 47 + '...": "r6" (2026-10-15)' in txt
    raw = open(os.path.join(root, ".roundtable", "decree-log.json")).read()
    assert raw.endswith("}\n")


def test_list_and_latest(tmp_path):
    root = str(tmp_path)
    a = store.create_session(root, "older")
    os.rename(a, a.replace("2026-10-15-2107", "2026-01-01-0000"))
    store.create_session(root, "newer")
    ss = store.list_sessions(root)
    assert [s.topic for s in ss] == ["newer", "older"]
    assert store.find_latest_session(root).topic == "newer"


def test_rounds_jsonl_resume_roundtrip(tmp_path):
    p = store.create_session(str(tmp_path), "t")
    for e in entries():
        store.append_round_entry(p, e)
    with open(os.path.join(p, "rounds.jsonl"), "a") as f:
        f.write('{"torn": ')   # crash mid-write
    back = store.load_round_entries(p)
    assert [(e.knight, e.round, e.response) for e in back] == [("Claude", 1, "Eerste."), ("GPT", 1, "Tweede.")]
    assert back[0].consensus.consensus_score == 8


def test_keys(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.delenv("X_KEY", raising=False)
    assert keys.get_key("X_KEY") is None
    keys.save_key("X_KEY", "abc")
    assert keys.get_key("X_KEY") == "abc"
    assert oct(os.stat(keys.keys_path()).st_mode & 0o777) == "0o600"
    monkeypatch.setenv("X_KEY", "env")
    assert keys.get_key("X_KEY") == "env"


def test_session_lock(tmp_path):
    a, b = SessionLock(str(tmp_path)), SessionLock(str(tmp_path))
    assert a.acquire()
    assert b.acquire()  # same pid: re-entrant takeover
    a.release()
