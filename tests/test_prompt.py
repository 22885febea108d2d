"""Prompt assembly (src/utils/prompt.ts + orchestrator.ts:397-425) in both layouts."""
from theroundtaible_amd.engine.tokenizer import get_tokenizer
from theroundtaible_amd.prompt import (EMPTY_HISTORY, KING_DEMAND, Prompt, TurnContext, build_system_prompt,
                                       build_turn_prompt_append, build_turn_prompt_reference,
                                       format_previous_rounds, transcript_entry_segments)
from theroundtaible_amd.types import ConsensusBlock, KnightConfig, RoundEntry

K = [KnightConfig("Claude", "claude-cli", ["architecture", "testing"], 1),
     KnightConfig("Gemini", "gemini-cli", ["docs"], 2), KnightConfig("Zed", "local-llm-zed", ["code"], 3)]


def test_system_prompt_placeholders_all_replaced():
    s = build_system_prompt(K[0], K, "Topic $& $1", "", [], "", "")
    assert "{{" not in s
    assert s.count("Topic $& $1") == 2  # both {{topic}} occurrences, literal (no JS $-patterns)
    assert "Naam: Claude" in s and "architecture, testing" in s and "- Gemini: docs\n- Zed: code" in s
    assert "(Geen eerdere beslissingen.)" in s and "No implementation history yet." in s
    assert EMPTY_HISTORY in s
    z = build_system_prompt(K[2], K, "t", "chron", [], "m", "d")
    assert "nuchtere knight" in z and "chron" in z


def test_previous_rounds_format():
    r = [RoundEntry("Claude", 1, "A", ConsensusBlock("Claude", 1, 7, pending_issues=["x", "y"]), ""),
         RoundEntry("Gemini", 1, "B", None, "")]
    assert format_previous_rounds(r) == ("### Claude (Ronde 1):\nA\n\nConsensus score: 7/10\nOpen punten: x, y"
                                         "\n\n---\n\n### Gemini (Ronde 1):\nB")


def test_reference_layout_order_and_filtering():
    ctx = TurnContext(topic="T", git_branch="main", git_diff="d" * 5000, recent_commits="abc fix",
                      key_file_contents="### README.md", source_file_contents="")
    p = build_turn_prompt_reference(K[0], K, ctx, [], king_demand=True, resolved_files="F", resolved_commands="C")
    t = p.text
    i = [t.index(s) for s in ["\n---\nOnderwerp: T", KING_DEMAND.strip(), "Git branch: main", "Git diff",
                              "Recente commits:\nabc fix", "Project bestanden:", "OPGEVRAAGDE BESTANDEN", "VERIFICATIE"]]
    assert i == sorted(i)
    assert "d" * 3000 + "\n```" in t and "d" * 3001 not in t
    assert "BRONCODE" not in t


def test_append_layout_is_pure_append_on_tokens():
    """Turn t+1's token ids start with turn t's ids + the knight's own response ids (resident KV reuse)."""
    tok = get_tokenizer(32000)
    ctx = TurnContext(topic="Caching")
    transcript = []
    p1 = build_turn_prompt_append(K[0], K, ctx, transcript, 1)

    def ids(p: Prompt):
        out = []
        for s in p.segments:
            out += list(s.ids) if s.ids is not None else tok.encode(s.text)
        return out

    resp_ids = tok.encode(" Mijn antwoord, met een JSON blok.")
    e1 = RoundEntry("Claude", 1, tok.decode(resp_ids), ConsensusBlock("Claude", 1, 6), "")
    transcript += transcript_entry_segments(e1, resp_ids, tok.family)
    e2 = RoundEntry("Gemini", 1, "Ander standpunt.", None, "")
    transcript += transcript_entry_segments(e2)
    p2 = build_turn_prompt_append(K[0], K, ctx, transcript, 2)
    a, b = ids(p1), ids(p2)
    assert b[:len(a) + len(resp_ids)] == a + resp_ids
    assert p2.text.endswith("### Claude (Ronde 2):\n")
