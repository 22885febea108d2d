"""CLI end-to-end on CPU, incl. BASELINE config 1: 2-knight GPT-2-small discuss, max_rounds=1."""
import json
import os
import subprocess

import pytest

from theroundtaible_amd.cli import main
from theroundtaible_amd.errors import ExitCode


def run(args, capsys=None):
    rc = main(["--quiet"] + args)
    return rc


def _init(project, model="gpt2-small", knights=2, max_new=8):
    assert main(["--quiet", "init", "--yes", "--model", model, "--knights", str(knights),
                 "--max-new-tokens", str(max_new)]) == 0
    cfg = json.load(open(project / ".roundtable" / "config.json"))
    return cfg


def test_init_writes_reference_schema(project):
    cfg = _init(project, knights=3)
    assert cfg["version"] == "1.0" and cfg["language"] == "nl"
    assert [k["name"] for k in cfg["knights"]] == ["Claude", "Gemini", "GPT"]
    assert [k["priority"] for k in cfg["knights"]] == [1, 2, 3]
    assert cfg["rules"]["max_rounds"] == 5 and cfg["rules"]["consensus_threshold"] == 9
    assert cfg["adapter_config"]["claude-cli"]["engine"]["model"] == "gpt2-small"
    assert open(project / ".roundtable" / "chronicle.md").read().startswith("# Chronicle — TheRoundtAIble")
    assert json.load(open(project / ".roundtable" / "manifest.json"))["features"] == []
    assert (project / ".roundtable" / "sessions").is_dir()


def test_missing_config_exit_code(project):
    assert main(["--quiet", "discuss", "x", "--no-read-codebase"]) == ExitCode.CONFIG_ERROR


def test_config1_gpt2_two_knight_discuss_cpu(project):
    """BASELINE config 1 (plumbing, no GPU): 2 knights on GPT-2-small via the local engine."""
    cfg = _init(project, "gpt2-small", knights=2, max_new=8)
    cfg["rules"]["max_rounds"] = 1
    cfg["engine"]["dtype"] = "fp32"
    json.dump(cfg, open(project / ".roundtable" / "config.json", "w"), indent=2)
    rc = main(["--quiet", "discuss", "Hoe testen we de tafel?", "--no-read-codebase", "--choice", "0",
               "--device", "cpu", "--seed", "1"])
    assert rc == 0
    sess = os.listdir(project / ".roundtable" / "sessions")
    assert len(sess) == 1
    sp = project / ".roundtable" / "sessions" / sess[0]
    st = json.load(open(sp / "status.json"))
    assert st["phase"] == "escalated" and st["round"] == 1
    disc = open(sp / "discussion.md").read()
    assert disc.startswith("# Discussion\n") and "## Round 1 — Claude" in disc and "## Round 1 — Gemini" in disc
    metrics = [json.loads(l) for l in open(sp / "metrics.jsonl")]
    assert any(m.get("decode_tokens") == 8 for m in metrics)
    # read-only commands on the result
    for cmd in (["status"], ["list"], ["chronicle"], ["decrees"], ["manifest", "list"], ["manifest", "check"]):
        assert main(["--quiet"] + cmd) == 0


def test_king_chooses_knight(project):
    cfg = _init(project, "tiny-llama", knights=2, max_new=4)
    cfg["rules"]["max_rounds"] = 1
    json.dump(cfg, open(project / ".roundtable" / "config.json", "w"))
    assert main(["--quiet", "discuss", "Kies", "--no-read-codebase", "--choice", "2", "--device", "cpu"]) == 0
    sp = project / ".roundtable" / "sessions" / os.listdir(project / ".roundtable" / "sessions")[0]
    st = json.load(open(sp / "status.json"))
    assert st["phase"] == "consensus_reached" and st["lead_knight"] == "Gemini"
    assert (sp / "decisions.md").exists()


def test_resume_from_rounds_jsonl(project):
    cfg = _init(project, "tiny-llama", knights=2, max_new=4)
    cfg["rules"]["max_rounds"] = 1
    json.dump(cfg, open(project / ".roundtable" / "config.json", "w"))
    assert main(["--quiet", "discuss", "Hervat", "--no-read-codebase", "--choice", "0", "--device", "cpu"]) == 0
    assert main(["--quiet", "discuss", "Hervat", "--no-read-codebase", "--choice", "0", "--device", "cpu",
                 "--resume", "latest"]) == 0
    sp = project / ".roundtable" / "sessions" / os.listdir(project / ".roundtable" / "sessions")[0]
    rounds = [json.loads(l)["round"] for l in open(sp / "rounds.jsonl")]
    assert rounds == [1, 1, 2, 2]


def test_summon_without_diff(project):
    _init(project, "tiny-llama", knights=1)
    assert main(["--quiet", "summon", "--no-read-codebase", "--device", "cpu"]) == 0
    assert os.listdir(project / ".roundtable" / "sessions") == []


def test_manifest_commands(project):
    _init(project, "tiny-llama", knights=1)
    (project / "a.py").write_text("x")
    assert main(["--quiet", "manifest", "add", "feat-1", "--files", "a.py", "b.py", "--summary", "Eerste"]) == 0
    assert main(["--quiet", "manifest", "deprecate", "feat-1", "--replaced-by", "feat-2"]) == 0
    m = json.load(open(project / ".roundtable" / "manifest.json"))
    assert m["features"][0]["status"] == "deprecated" and m["features"][0]["lead_knight"] == "manual"


def _scripted(project, **script):
    cfg = _init(project, model="tiny-llama", knights=3, max_new=64)
    cfg["rules"]["max_rounds"] = 4
    cfg["rules"]["round_mode"] = "parallel"
    cfg["rules"]["prompt_layout"] = "shared"
    cfg["engine"]["scripted_consensus"] = {"free_tokens": 6, "files": ["NEW:docs/besluit.md"], **script}
    json.dump(cfg, open(project / ".roundtable" / "config.json", "w"), indent=2)
    return cfg


def _session(project):
    sess = os.listdir(project / ".roundtable" / "sessions")
    assert len(sess) == 1
    return project / ".roundtable" / "sessions" / sess[0]


def test_scripted_consensus_discuss_then_apply_dry_run(project):
    """Engine knights with the forced consensus tail (knights/script.py): round 1 scores 6, round 2
    scores 9 -> consensus after round 2 (early exit, scope, lead knight, chronicle); then
    `apply --dry-run` parses the lead's forced RTDIFF/1 block and plans one in-scope NEW file."""
    _scripted(project, scores=[6, 9])
    assert run(["discuss", "Gedeelde KV per tafel", "--no-read-codebase", "--seed", "1"]) == 0
    sp = _session(project)
    st = json.load(open(sp / "status.json"))
    assert st["consensus_reached"] is True and st["phase"] == "consensus_reached" and st["round"] == 2
    assert st["allowed_files"] == ["NEW:docs/besluit.md"] and st["lead_knight"] in ("Claude", "Gemini", "GPT")
    rounds = [json.loads(l) for l in open(sp / "rounds.jsonl")]
    assert len(rounds) == 6 and all(r["consensus"] is not None for r in rounds)      # stopped after round 2
    assert "Consensus in 2 round(s)" in open(project / ".roundtable" / "chronicle.md").read()
    assert run(["apply", "--dry-run", "--yes"]) == 0
    plan = json.load(open(sp / "apply-plan.json"))
    assert [p["path"] for p in plan["planned"]] == ["docs/besluit.md"] and plan["planned"][0]["new_file"]
    assert "+# Besluit van de ronde tafel" in plan["planned"][0]["diff"] and plan["skipped"] == []
    assert not (project / "docs" / "besluit.md").exists()                            # dry run never writes
    assert run(["apply", "--noparley", "--yes"]) == 0
    assert (project / "docs" / "besluit.md").read_text().startswith("# Besluit van de ronde tafel")
    man = json.load(open(project / ".roundtable" / "manifest.json"))
    assert man["features"][-1]["status"] == "implemented" and man["features"][-1]["files"] == ["docs/besluit.md"]


def test_scripted_unanimous_rejection(project):
    _scripted(project, reject=True, reject_round=1)
    assert run(["discuss", "Alles in een kernel", "--no-read-codebase", "--seed", "1"]) == 0
    st = json.load(open(_session(project) / "status.json"))
    assert st["consensus_reached"] is True and st["round"] == 1
    assert "Unanimous rejection in 1 round(s)" in open(project / ".roundtable" / "chronicle.md").read()


def test_resume_missing_session_is_session_error(project):
    """--resume <typo> must raise SessionError (exit 3) before reading any rounds file."""
    _init(project, "tiny-llama", knights=1, max_new=4)
    from theroundtaible_amd.errors import ExitCode
    rc = main(["--quiet", "discuss", "x", "--no-read-codebase", "--choice", "0", "--device", "cpu",
               "--resume", "no-such-session"])
    assert rc == ExitCode.SESSION_ERROR == 3


@pytest.mark.parametrize("raw,want", [("2", 2), ("2 ", 2), (" 2", 2), ("2abc", 2), ("+3", 3), ("-1", -1),
                                      ("0x2", 2), ("abc", None), ("", None), (" ", None), ("0xg", None),
                                      ("1.9", 1), ("07", 7)])
def test_king_choice_parses_like_js_parseint(raw, want):
    from theroundtaible_amd.cli import js_parse_int
    assert js_parse_int(raw) == want
