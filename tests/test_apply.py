"""`roundtable apply` from its spec: RTDIFF/1, block scanner, scope, dry-run, backups, manifest."""
import json
import os

import pytest

from theroundtaible_amd import store
from theroundtaible_amd.apply import rtdiff
from theroundtaible_amd.apply.blocks import block_map, resolve, scan
from theroundtaible_amd.cli import main
from theroundtaible_amd.errors import ExitCode, ValidationError

PY = '''import os


def helper(x):
    return x + 1


class Cache:
    def get(self, k):
        return k

    @staticmethod
    def put(k, v):
        pass
'''

TS = '''import x from "y";

export function handle(req: Request): Response {
  if (req) { return new Response("{"); }
  return null;
}

export class Store {
  private items = {};
  get(key: string): string {
    return this.items[key];
  }
}

const arrow = (a: number) => {
  return a * 2;
};
'''


def test_scan_python():
    ids = {b.id: (b.start, b.end) for b in scan("m.py", PY)}
    assert ids["def:helper"] == (4, 5)
    assert ids["class:Cache"] == (8, 14)
    assert ids["def:Cache.get"] == (9, 10)
    assert ids["def:Cache.put"] == (12, 14)   # decorator included


def test_scan_typescript():
    ids = {b.id: (b.start, b.end) for b in scan("m.ts", TS)}
    assert ids["function:handle"] == (3, 6)     # brace inside a string is ignored
    assert ids["class:Store"] == (8, 13)
    assert ids["method:Store.get"] == (10, 12)
    assert ids["const:arrow"] == (15, 17)
    assert "BLOCK_MAP m.ts:" in block_map("m.ts", TS)
    assert resolve("lines:2-3", [], 10) == (2, 3) and resolve("lines:9-11", [], 10) is None


def test_rtdiff_roundtrip():
    out = """Hier is mijn diff:
```
RTDIFF/1
FILE: m.py
BLOCK_REPLACE def:helper
<<<
def helper(x):
    return x + 2
>>>
BLOCK_INSERT_AFTER def:Cache.get
<<<

    def size(self):
        return 0
>>>
BLOCK_DELETE: def:Cache.put
FILE: NEW:pkg/new.py
CREATE
<<<
VALUE = 1
>>>
END
```"""
    edits, warns = rtdiff.parse(out)
    assert not warns and [e.path for e in edits] == ["m.py", "pkg/new.py"] and edits[1].is_new
    new = rtdiff.apply_edit(edits[0], PY)
    assert "return x + 2" in new and "def size(self)" in new and "def put" not in new and "@staticmethod" not in new
    assert rtdiff.validate_syntax("m.py", new) is None
    assert rtdiff.apply_edit(edits[1], None) == "VALUE = 1\n"


def test_rtdiff_errors():
    with pytest.raises(ValidationError):
        rtdiff.parse("nothing here")
    e, _ = rtdiff.parse("RTDIFF/1\nFILE: m.py\nBLOCK_REPLACE def:nope\n<<<\nx\n>>>\n")
    with pytest.raises(ValidationError, match="unknown block"):
        rtdiff.apply_edit(e[0], PY)
    e, _ = rtdiff.parse("RTDIFF/1\nFILE: m.py\nBLOCK_DELETE class:Cache\nBLOCK_DELETE def:Cache.get\n")
    with pytest.raises(ValidationError, match="overlap"):
        rtdiff.apply_edit(e[0], PY)
    assert "syntax error" in rtdiff.validate_syntax("m.py", "def (:\n")
    assert "unbalanced" in rtdiff.validate_syntax("m.ts", "function f() {")
    assert rtdiff.validate_syntax("m.ts", TS) is None


def test_legacy_edit_format_warns():
    out = "EDIT: m.py\n<<<<<<< SEARCH\n    return x + 1\n=======\n    return x - 1\n>>>>>>> REPLACE\n"
    edits, warns = rtdiff.parse(out)
    assert warns and "deprecated" in warns[0]
    assert "return x - 1" in rtdiff.apply_edit(edits[0], PY)


def _consensus_session(project, allowed):
    assert main(["--quiet", "init", "--yes", "--model", "tiny-llama", "--knights", "2"]) == 0
    p = store.create_session(str(project), "Verbeter de helper")
    store.write_decisions(p, "Verbeter de helper", "helper moet +2 doen", [])
    store.update_status(p, phase="consensus_reached", consensus_reached=True, allowed_files=allowed,
                        lead_knight="Claude")
    return p


def test_apply_dry_run_writes_nothing(project):
    (project / "m.py").write_text(PY)
    p = _consensus_session(project, ["m.py"])
    resp = project / "resp.txt"
    resp.write_text("RTDIFF/1\nFILE: m.py\nBLOCK_REPLACE def:helper\n<<<\ndef helper(x):\n    return x + 2\n>>>\nEND\n")
    assert main(["--quiet", "apply", "--dry-run", "--response-file", str(resp)]) == 0
    assert (project / "m.py").read_text() == PY
    assert store.read_status(p)["phase"] == "consensus_reached"


def test_apply_noparley_scope_backup_manifest(project):
    (project / "m.py").write_text(PY)
    (project / "other.py").write_text("x = 1\n")
    p = _consensus_session(project, ["m.py", "NEW:pkg/n.py"])
    resp = project / "resp.txt"
    resp.write_text("RTDIFF/1\nFILE: m.py\nBLOCK_REPLACE def:helper\n<<<\ndef helper(x):\n    return x + 2\n>>>\n"
                    "FILE: other.py\nBLOCK_REPLACE lines:1-1\n<<<\nx = 2\n>>>\n"
                    "FILE: NEW:pkg/n.py\nCREATE\n<<<\nN = 1\n>>>\nEND\n")
    assert main(["--quiet", "apply", "--noparley", "--response-file", str(resp)]) == 0
    assert "return x + 2" in (project / "m.py").read_text()
    assert (project / "other.py").read_text() == "x = 1\n"          # out of scope: blocked
    assert (project / "pkg" / "n.py").read_text() == "N = 1\n"
    bak = project / ".roundtable" / "backups" / os.path.basename(p) / "m.py.bak"
    assert bak.read_text() == PY
    m = store.read_manifest(str(project))["features"][0]
    assert m["status"] == "partial" and m["files_skipped"] == ["other.py"] and m["lead_knight"] == "Claude"
    assert store.read_status(p)["phase"] == "completed"


def test_apply_override_scope_logs_decree(project):
    (project / "other.py").write_text("x = 1\n")
    _consensus_session(project, ["m.py"])
    resp = project / "resp.txt"
    resp.write_text("RTDIFF/1\nFILE: other.py\nBLOCK_REPLACE lines:1-1\n<<<\nx = 2\n>>>\n")
    assert main(["--quiet", "apply", "--noparley", "--override-scope", "--reason", "hotfix",
                 "--response-file", str(resp)]) == 0
    assert (project / "other.py").read_text() == "x = 2\n"
    d = store.read_decree_log(str(project))["entries"][0]
    assert d["type"] == "override_scope" and d["reason"] == "hotfix"


def test_apply_requires_consensus_and_valid_output(project):
    assert main(["--quiet", "init", "--yes", "--model", "tiny-llama", "--knights", "1"]) == 0
    store.create_session(str(project), "x")
    assert main(["--quiet", "apply", "--dry-run"]) == ExitCode.SESSION_ERROR
    (project / "m.py").write_text(PY)
    p = _consensus_session(project, ["m.py"])
    resp = project / "bad.txt"
    resp.write_text("RTDIFF/1\nFILE: m.py\nBLOCK_REPLACE def:helper\n<<<\ndef helper(x:\n>>>\n")
    assert main(["--quiet", "apply", "--noparley", "--session", os.path.basename(p),
                 "--response-file", str(resp)]) == ExitCode.VALIDATION_ERROR
    assert (project / "m.py").read_text() == PY
