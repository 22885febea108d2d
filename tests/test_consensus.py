"""Parity tests for the consensus engine (reference src/consensus.ts)."""
from theroundtaible_amd.consensus import (ConsensusStopDetector, balanced_objects, check_consensus,
                                          check_negative_consensus, missing_scope_warning, parse_consensus,
                                          repair_json, strip_consensus_json, summarize_consensus,
                                          validate_files_to_modify)
from theroundtaible_amd.types import ConsensusBlock


def test_fenced_json():
    r = 'Blah\n```json\n{"consensus_score": 8, "agrees_with": ["a"], "pending_issues": ["x"]}\n```\n'
    b = parse_consensus(r, "Claude", 2)
    assert b.consensus_score == 8 and b.agrees_with == ["a"] and b.pending_issues == ["x"]
    assert b.knight == "Claude" and b.round == 2


def test_any_fence_then_bare_nested():
    r = 'text ```\n{"consensus_score": 5}\n``` more'
    assert parse_consensus(r, "K", 1).consensus_score == 5
    r2 = 'I think {"x": 1} and {"consensus_score": 7, "meta": {"nested": {"a": "}"}}, "agrees_with": []} end'
    b = parse_consensus(r2, "K", 1)
    assert b.consensus_score == 7


def test_fence_without_score_falls_through_to_bare():
    r = '```python\nprint(1)\n```\nfinal: {"consensus_score": 9, "files_to_modify": ["src/a.ts"]}'
    b = parse_consensus(r, "K", 3)
    assert b.consensus_score == 9 and b.files_to_modify == ["src/a.ts"]


def test_repair_comments_trailing_commas_single_quotes():
    r = "```json\n{\n  'consensus_score': 6, // local models love comments\n  'agrees_with': ['plan',],\n}\n```"
    b = parse_consensus(r, "K", 1)
    assert b is not None and b.consensus_score == 6 and b.agrees_with == ["plan"]
    assert repair_json('{"a": 1,}') == '{"a": 1}'


def test_pending_issues_sanitized_and_caps():
    r = ('{"consensus_score": 10, "pending_issues": ["none", " N/A ", "geen", "real issue", 3], '
         '"file_requests": ["a","b","c","d","e"], "verify_commands": ["ls","ls","ls","ls","ls","ls"]}')
    b = parse_consensus(r, "K", 1)
    assert b.pending_issues == ["real issue"]
    assert len(b.file_requests) == 4 and len(b.verify_commands) == 4


def test_non_numeric_score_and_garbage():
    assert parse_consensus('{"consensus_score": "9"}', "K", 1) is None
    assert parse_consensus('{"consensus_score": true}', "K", 1) is None
    assert parse_consensus("no json here", "K", 1) is None
    assert parse_consensus('{"consensus_score": NaN}', "K", 1) is None


def test_knight_and_round_override_js_truthiness():
    b = parse_consensus('{"consensus_score": 4, "knight": "Gemini", "round": 7}', "K", 1)
    assert b.knight == "Gemini" and b.round == 7
    b = parse_consensus('{"consensus_score": 4, "knight": "", "round": 0}', "K", 3)
    assert b.knight == "K" and b.round == 3


def test_validate_files_to_modify():
    raw = ["src/a.ts", "./src/a.ts", "NEW: src/new.ts", "new:src\\win.ts", "../etc/passwd", "/abs.ts",
           "", 5, "src/a.ts", "NEW:src/new.ts"]
    assert validate_files_to_modify(raw) == ["src/a.ts", "NEW:src/new.ts", "NEW:src/win.ts"]
    assert validate_files_to_modify("nope") == []


def test_check_consensus_and_negative():
    mk = lambda s: ConsensusBlock("k", 1, s)  # noqa: E731
    assert check_consensus([mk(9), mk(10)], 9)
    assert not check_consensus([mk(9), mk(8)], 9)
    assert not check_consensus([], 9)
    assert check_negative_consensus([mk(3), mk(0)])
    assert not check_negative_consensus([mk(3)])
    assert not check_negative_consensus([mk(3), mk(4)])


def test_summarize_format():
    blocks = [ConsensusBlock("Claude", 2, 9, ["x"], ["p"], files_to_modify=["a"]), ConsensusBlock("GPT", 2, 4)]
    s = summarize_consensus(blocks)
    assert "- **Claude** (Round 2): Score 9/10 [AGREES]" in s
    assert "  Agrees with: x" in s and "  Pending: p" in s and "  Scope: a" in s
    assert "- **GPT** (Round 2): Score 4/10 [DISAGREES]" in s
    assert s.endswith("Average score: 6.5/10")
    assert summarize_consensus([]) == "No consensus data yet."


def test_missing_scope_warning():
    assert missing_scope_warning(ConsensusBlock("K", 1, 9)) is not None
    assert missing_scope_warning(ConsensusBlock("K", 1, 9, files_to_modify=["a"])) is None
    assert missing_scope_warning(ConsensusBlock("K", 1, 8)) is None


def test_balanced_and_strip():
    t = 'a {"consensus_score": 1, "s": "{"} b {"other": 2}'
    assert balanced_objects(t, "consensus_score") == ['{"consensus_score": 1, "s": "{"}']
    assert strip_consensus_json('Hi ```json\n{"consensus_score": 1}\n``` there').strip() == "Hi  there"
    assert strip_consensus_json('Hi {"consensus_score": 2, "x": {"y": 1}} bye') == "Hi  bye"


def test_stop_detector():
    d = ConsensusStopDetector()
    assert not d.feed("Mijn mening is ")
    assert not d.feed('```json\n{"consensus_score": 8,')
    assert d.feed(' "agrees_with": []}\n```')
