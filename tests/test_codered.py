"""code-red diagnostic mode (README.md:159-175) with scripted doctors."""
import json

from theroundtaible_amd import codered
from theroundtaible_amd.cli import main


def verdict(key, conf):
    return f"Analyse.\n```json\n{json.dumps({'confidence_score': conf, 'root_cause_key': key, 'evidence': ['log']})}\n```"


def test_parse_and_convergence():
    d = codered.parse_diagnosis(verdict("null-session-token", 9), "A", 2)
    assert d.root_cause_key == "null-session-token" and d.evidence == ["log"]
    assert codered.parse_diagnosis("no json", "A", 1) is None
    lat = {"A": d, "B": codered.Diagnosis("B", 2, 8, "Null Session Token"), "C": codered.Diagnosis("C", 2, 9, "x")}
    assert codered.check_convergence(lat) == "null-session-token"
    lat["B"].confidence_score = 7
    assert codered.check_convergence(lat) is None
    assert codered.keys_match("db-timeout", "db-timeout-on-login")


def test_code_red_command_with_fake_doctors(project):
    assert main(["--quiet", "init", "--yes", "--model", "tiny-llama", "--knights", "2"]) == 0
    cfg = json.load(open(project / ".roundtable" / "config.json"))
    for a in ("claude-cli", "gemini-cli"):
        cfg["adapter_config"][a]["engine"]["backend"] = "fake"
    json.dump(cfg, open(project / ".roundtable" / "config.json", "w"))
    from theroundtaible_amd.knights import fake
    orig = fake.FakeBackend.__init__

    def init(self, *a, **kw):
        orig(self, *a, **kw)
        self.script = lambda key, prompt, idx: verdict("race-in-cache", 9 if idx >= 1 else 5)

    fake.FakeBackend.__init__ = init
    try:
        assert main(["--quiet", "code-red", "login crasht", "--device", "cpu"]) == 0
    finally:
        fake.FakeBackend.__init__ = orig
    log = open(project / ".roundtable" / "error-log.md").read()
    assert "## CR-001 [OPEN] — login crasht" in log and "**Root cause:** race-in-cache" in log


def test_code_red_on_engine_doctors_with_scripted_verdicts(project):
    """code-red with engine-hosted doctors: the scripted tail gives every doctor the same
    root_cause_key at confidence 6 in triage and 9 from round 2 -> convergence after the
    blind round, logged OPEN as CR-001 in error-log.md."""
    import json
    from theroundtaible_amd.cli import main
    assert main(["--quiet", "init", "--yes", "--model", "tiny-llama", "--knights", "3", "--max-new-tokens", "16"]) == 0
    p = project / ".roundtable" / "config.json"
    cfg = json.load(open(p))
    cfg["engine"]["scripted_consensus"] = {"free_tokens": 4}
    json.dump(cfg, open(p, "w"), indent=2)
    assert main(["--quiet", "code-red", "decode hangt na 40K tokens", "--no-read-codebase"]) == 0
    log = (project / ".roundtable" / "error-log.md").read_text()
    assert "CR-001" in log and "OPEN" in log and "kv-cache-exhausted" in log
