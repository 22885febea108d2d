"""tools/manual_knight_test.py (parity: reference tests/manual-adapter-test.mjs)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("manual_knight_test", os.path.join(ROOT, "tools", "manual_knight_test.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_fake_knight_echoes_score_9_strict(capsys):
    assert _tool().main(["--adapters", "fake", "--device", "cpu", "--strict"]) == 0
    assert "consensus_score=9 [PASS]" in capsys.readouterr().out


def test_engine_knight_answers_on_cpu(capsys):
    rc = _tool().main(["--adapters", "claude-cli", "--device", "cpu", "--max-new-tokens", "4"])
    out = capsys.readouterr().out
    assert rc == 0 and "claude-cli (Claude)" in out and "4 decode tokens" in out
    # random weights cannot follow the instruction: strict mode reports the failure
    assert _tool().main(["--adapters", "claude-cli", "--device", "cpu", "--max-new-tokens", "4", "--strict"]) == 1


def test_unknown_adapter_fails(capsys):
    assert _tool().main(["--adapters", "nope-llm", "--device", "cpu"]) == 1
    assert "unknown adapter" in capsys.readouterr().out
