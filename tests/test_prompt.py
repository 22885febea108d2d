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


# ---- rules.placeholder_semantics = "reference": JS String.prototype.replace with a string pattern
# (src/utils/prompt.ts:95-104). Expected strings are hand-derived from ECMA-262 GetSubstitution.
import pytest  # noqa: E402

from theroundtaible_amd.prompt import fill_template, js_replace_first  # noqa: E402

JS_CASES = [
    # (string, pattern, replacement, what JS returns)
    ("A {{topic}} B {{topic}}", "{{topic}}", "X", "A X B {{topic}}"),        # first occurrence only
    ("T={{topic}}.", "{{topic}}", "<$&>", "T=<{{topic}}>."),                  # $& = the match
    ("ab{{topic}}cd", "{{topic}}", "[$`]", "ab[ab]cd"),                       # $` = text before
    ("ab{{topic}}cd", "{{topic}}", "[$']", "ab[cd]cd"),                       # $' = text after
    ("ab{{topic}}cd", "{{topic}}", "$$5", "ab$5cd"),                          # $$ = $
    ("ab{{topic}}cd", "{{topic}}", "$$&", "ab$&cd"),                          # $$ first, then '&'
    ("ab{{topic}}cd", "{{topic}}", "$1 $< $", "ab$1 $< $cd"),                 # no captures: literal
    ("ab{{topic}}cd", "{{topic}}", "$", "ab$cd"),                             # lone trailing $
    ("x{{a}}y{{a}}z", "{{a}}", "$'$`", "xy{{a}}zxy{{a}}z"),                   # after + before
    ("no placeholder", "{{topic}}", "$&", "no placeholder"),                  # not found: unchanged
]


@pytest.mark.parametrize("s,pat,rep,want", JS_CASES)
def test_js_replace_first_matches_hand_derived_js(s, pat, rep, want):
    assert js_replace_first(s, pat, rep) == want


def test_fill_template_reference_chain_order():
    # each .replace runs on the string built so far: a value holding a later placeholder is
    # where that placeholder gets filled, and the template's own occurrence stays literal
    tpl = "{{knight_name}} / {{topic}}"
    got = fill_template(tpl, {"knight_name": "K {{topic}}", "topic": "T"}, "reference")
    assert got == "K T / {{topic}}"
    assert fill_template(tpl, {"knight_name": "K {{topic}}", "topic": "T"}, "literal") == "K T / T"
    with pytest.raises(ValueError):
        fill_template(tpl, {}, "js")


def test_system_prompt_reference_semantics_second_topic_stays_literal():
    s = build_system_prompt(K[0], K, "Topic $& $1 $$", "", [], "", "", semantics="reference")
    # the template holds {{topic}} twice: the reference fills the first one only, and $& puts
    # the matched placeholder text back into the filled value
    assert "Topic {{topic}} $1 $" in s
    assert s.count("{{topic}}") == 2
    s2 = build_system_prompt(K[0], K, "plain", "", [], "", "", semantics="reference")
    assert s2.count("{{topic}}") == 1 and s2.count("plain") == 1
    lit = build_system_prompt(K[0], K, "Topic $& $1 $$", "", [], "", "")
    assert "{{topic}}" not in lit and lit.count("Topic $& $1 $$") == 2


def test_placeholder_semantics_config_and_orchestrator():
    from theroundtaible_amd.config import validate_config
    from theroundtaible_amd.errors import ConfigError
    from theroundtaible_amd.types import RulesConfig
    base = {"version": "1", "knights": [{"name": "A", "adapter": "x", "capabilities": [], "priority": 1}],
            "rules": {"max_rounds": 1, "consensus_threshold": 9, "timeout_per_turn_seconds": 10},
            "adapter_config": {}}
    validate_config(base)
    base["rules"]["placeholder_semantics"] = "reference"
    validate_config(base)
    assert RulesConfig.from_dict(base["rules"]).placeholder_semantics == "reference"
    base["rules"]["placeholder_semantics"] = "js"
    with pytest.raises(ConfigError):
        validate_config(base)
