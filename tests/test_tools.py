"""verify_commands sandbox (src/utils/verify.ts) and file_requests (src/orchestrator.ts:164-222)."""
import os

import pytest

from theroundtaible_amd.tools import resolve_file_requests
from theroundtaible_amd.verify import resolve_verify_commands, validate_command


@pytest.mark.parametrize("cmd", ["ls", "ls -la src | grep ts", "grep -rn 'a\\|b' src", "cat x 2>/dev/null",
                                 "find . -name '*.py' 2>&1 | wc -l", "head -5 README.md | tail -2",
                                 "grep -rn fprint src", "ls my-execdir-notes"])
def test_allowed(cmd):
    assert validate_command(cmd) is None


@pytest.mark.parametrize("cmd,why", [
    ("", "empty command"), ("ls; rm -rf /", "forbidden pattern: ;"), ("echo `id`", "forbidden pattern: `"),
    ("ls $(pwd)", "forbidden pattern: \\$\\("), ("ls ${HOME}", "forbidden pattern: \\$\\{"),
    ("ls && ls", "forbidden pattern: &&"), ("ls || ls", "forbidden pattern: \\|\\|"),
    ("find . -exec rm {} +", "forbidden pattern: -exec\\b"), ("find . -delete", "forbidden pattern: -delete\\b"),
    ("cat a > b", "forbidden pattern: output redirect (>)"), ("cat a >> b", "forbidden pattern: append redirect (>>)"),
    ("cat < a", "forbidden pattern: input redirect (<)"), ("rm x", "forbidden command: rm"),
    ("echo hi", "command not whitelisted: echo"), ("ls | ", "empty pipe segment"),
    ("ls | python3 -c 1", "forbidden command: python3"),
    # deliberate fixes over the reference: other bash command separators
    ("ls\nrm -rf x", "forbidden pattern: newline (command separator)"),
    ("ls\r\nrm x", "forbidden pattern: newline (command separator)"),
    ("ls & rm x", "forbidden pattern: & (background / separator)"),
    ("cat a &", "forbidden pattern: & (background / separator)"),
    ("find . -execdir rm {} +", "forbidden pattern: -exec*/-ok*"),
    ("find . -okdir rm {} +", "forbidden pattern: -exec*/-ok*"),
    ("find . -fprint out.txt", "forbidden pattern: -fprint*/-fls"),
    ("find . -fprintf out.txt %p", "forbidden pattern: -fprint*/-fls"),
    ("find . -fprint0 out", "forbidden pattern: -fprint*/-fls"),
    ("find . -fls out.txt", "forbidden pattern: -fprint*/-fls"),
])
def test_denied(cmd, why):
    assert validate_command(cmd) == why


def test_apply_paths_stay_inside_project(tmp_path):
    from theroundtaible_amd.apply.apply import inside_project
    (tmp_path / "src").mkdir()
    os.symlink("/etc", tmp_path / "escape")
    assert inside_project(str(tmp_path), "src/a.py") and inside_project(str(tmp_path), "new/dir/b.py")
    for bad in ("../x.py", "src/../../x.py", "/etc/passwd", "~/x", "escape/passwd", "", "."):
        assert not inside_project(str(tmp_path), bad), bad


def test_execute(tmp_path, monkeypatch):
    (tmp_path / "a.txt").write_text("hello\nworld\n")
    monkeypatch.setenv("OPENAI_API_KEY", "secret")
    out = resolve_verify_commands(["cat a.txt", "grep nomatch a.txt", "rm a.txt", "cat a.txt | wc -l"], str(tmp_path))
    parts = out.split("\n\n")
    assert parts[0] == "### VERIFY: cat a.txt\n```\nhello\nworld\n```"
    assert "exit code 1" in parts[1]
    assert "[DENIED] forbidden command: rm" in parts[2]
    assert parts[3].endswith("```\n2\n```")
    assert (tmp_path / "a.txt").exists()


def test_env_scrubbed(tmp_path, monkeypatch):
    monkeypatch.setenv("ANTHROPIC_API_KEY", "leak")
    out = resolve_verify_commands(["grep -c leak /proc/self/environ"], str(tmp_path))
    assert "\n0\n" in out or "exit code" in out


def test_file_requests(tmp_path):
    (tmp_path / "src").mkdir()
    (tmp_path / "src" / "a.ts").write_text("\n".join(f"line{i}" for i in range(1, 251)))
    (tmp_path / "node_modules").mkdir()
    (tmp_path / "node_modules" / "x.js").write_text("x")
    out = resolve_file_requests(["src/a.ts:2-3", "src/a.ts", "../etc/passwd", "/etc/passwd",
                                 "node_modules/x.js", "missing.ts"], str(tmp_path), ["node_modules"])
    parts = out.split("\n\n")
    assert parts[0] == "### src/a.ts:2-3\n```\nline2\nline3\n```"
    assert parts[1].endswith("line200\n...(50 more lines)\n```")
    assert len(parts) == 4  # capped at 4 requests
    assert parts[2] == "[DENIED] ../etc/passwd — path traversal not allowed"
    assert parts[3] == "[DENIED] /etc/passwd — path traversal not allowed"
    out2 = resolve_file_requests(["node_modules/x.js", "missing.ts", "src/../src/a.ts:1-1"], str(tmp_path),
                                 ["node_modules"])
    assert out2.split("\n\n") == ["[DENIED] node_modules/x.js — matches ignore pattern", "[NOT FOUND] missing.ts",
                                  "### src/../src/a.ts:1-1\n```\nline1\n```"]
