"""Opt-in reference transports (knights/external.py): local-llm HTTP, vendor APIs, vendor CLIs.

The local-llm seat is exercised end to end against ``roundtable serve`` on a tiny CPU engine
(both the Ollama and OpenAI dialects), which is also the multi-node story: a knight on one
node talking to a serve endpoint on another. Vendor APIs/CLIs are driven by injected HTTP
callables and stub executables; no network is touched.
"""
import json
import os
import stat

import pytest

from theroundtaible_amd.errors import AdapterError
from theroundtaible_amd.knights.external import (ApiBackend, CliBackend, HttpResponse, LocalLlmHttpBackend,
                                                 create_external, extract_agent_message, is_context_window_error,
                                                 wants_external)
from theroundtaible_amd.serve import build_server


@pytest.fixture(scope="module")
def server():
    srv = build_server("tiny-llama", weights="random:3", device="cpu", port=0, max_batch=2, max_tokens=6,
                       num_blocks=128).start()
    yield srv
    srv.close()


@pytest.mark.parametrize("source", ["Ollama", None])
def test_local_llm_against_serve(server, source):
    b = LocalLlmHttpBackend("Local", "local-llm", server.url, "tiny-llama", source)
    assert b.is_available()
    ctx = b.detect_context_window()
    if source == "Ollama":
        assert ctx and ctx > 0 and b.max_source_chars() == max(ctx - 7096, 2000) * 4
    else:
        assert ctx is None and b.max_source_chars() is None
    res = b.execute("Onderwerp: caching", 60.0)
    assert isinstance(res.text, str) and res.text and res.metrics["backend"] == "local-llm-http"


def test_local_llm_unavailable_and_errors():
    b = LocalLlmHttpBackend("Local", "local-llm", "http://127.0.0.1:9", "m", None)
    assert not b.is_available()
    calls = []

    def http(method, url, body, headers, timeout):
        calls.append((url, body))
        if len(calls) == 1:
            return HttpResponse(500, "Model reloaded, try again")
        return HttpResponse(200, json.dumps({"choices": [{"message": {"content": "ok"}}]}))

    b = LocalLlmHttpBackend("Local", "local-llm", "http://x", "m", "LM Studio", http=http, retry_delay_s=0)
    assert b.execute("p", 5.0).text == "ok" and len(calls) == 2
    assert "max_tokens" not in calls[0][1]                       # local-llm.ts:157-160
    assert b.max_source_chars() == (16384 - 7096) * 4            # LM Studio assumed window

    b = LocalLlmHttpBackend("Local", "local-llm", "http://x", "m", "LM Studio",
                            http=lambda *a: HttpResponse(400, "n_keep: 9000 >= n_ctx: 4096"))
    with pytest.raises(AdapterError) as ei:
        b.execute("p", 5.0)
    assert "context window too small" in str(ei.value)
    assert is_context_window_error("This model's maximum context length is 8192")


def test_ollama_num_ctx_clamped():
    seen = {}

    def http(method, url, body, headers, timeout):
        if url.endswith("/api/show"):
            return HttpResponse(200, json.dumps({"model_info": {"llama.context_length": 8192}}))
        seen.update(body)
        return HttpResponse(200, json.dumps({"message": {"content": "antwoord"}}))

    b = LocalLlmHttpBackend("L", "local-llm", "http://x", "m", "Ollama", http=http)
    assert b.detect_context_window() == 8192
    assert b.execute("x" * 100, 5.0).text == "antwoord" and seen["options"]["num_ctx"] == 25 + 4096 + 512
    b.execute("x" * 40000, 5.0)
    assert seen["options"]["num_ctx"] == 8192


@pytest.mark.parametrize("aid,needle,payload", [
    ("claude-api", "/v1/messages", {"content": [{"type": "text", "text": "hi"}]}),
    ("openai-api", "/v1/chat/completions", {"choices": [{"message": {"content": "hi"}}]}),
    ("gemini-api", ":generateContent?key=K", {"candidates": [{"content": {"parts": [{"text": "hi"}]}}]}),
])
def test_api_backends(monkeypatch, aid, needle, payload):
    env = {"claude-api": "ANTHROPIC_API_KEY", "openai-api": "OPENAI_API_KEY", "gemini-api": "GEMINI_API_KEY"}[aid]
    monkeypatch.setenv("HOME", "/nonexistent-home")
    monkeypatch.delenv(env, raising=False)
    seen = {}

    def http(method, url, body, headers, timeout):
        seen.update(url=url, body=body, headers=headers)
        return HttpResponse(200, json.dumps(payload))

    b = ApiBackend("V", aid, base_url="http://api", http=http)
    assert not b.is_available()
    with pytest.raises(AdapterError):
        b.execute("p", 5.0)
    monkeypatch.setenv(env, "K")
    assert b.is_available() and b.execute("p", 5.0).text == "hi" and needle in seen["url"]
    assert "16384" in json.dumps(seen["body"])                   # MAX_OUTPUT_TOKENS per vendor
    b2 = ApiBackend("V", aid, base_url="http://api", http=lambda *a: HttpResponse(401, "invalid api key"))
    with pytest.raises(AdapterError) as ei:
        b2.execute("p", 5.0)
    assert ei.value.kind == "auth"


def _stub(tmp_path, name, script):
    p = tmp_path / name
    p.write_text("#!/bin/sh\n" + script)
    p.chmod(p.stat().st_mode | stat.S_IEXEC)
    return str(p)


def test_cli_backends(tmp_path):
    claude = _stub(tmp_path, "claude", 'if [ "$1" = "--version" ]; then echo 1.0; exit 0; fi\n'
                                       'cat > /dev/null; echo "args:$*"; [ -z "$CLAUDECODE" ] && echo clean\n')
    b = CliBackend("Claude", "claude-cli", command=claude, cwd=str(tmp_path))
    assert b.is_available()
    out = CliBackend("Claude", "claude-cli", command=claude).execute("prompt", 10.0).text
    assert "--disallowedTools" in out and "clean" in out

    gem = _stub(tmp_path, "gemini", 'case "$*" in *approval-mode*) echo "unknown approval-mode" >&2; exit 2;; esac\n'
                                    'cat > /dev/null; echo short; exit 0\n')
    assert CliBackend("Gemini", "gemini-cli", command=gem).execute("p", 10.0).text.strip() == "short"

    codex_lines = [json.dumps({"type": "thread.started"}),
                   json.dumps({"type": "item.completed", "item": {"type": "agent_message", "text": "eerste"}}),
                   "not json", json.dumps({"type": "item.completed", "item": {"type": "reasoning", "text": "x"}}),
                   json.dumps({"type": "item.completed", "item": {"type": "agent_message", "text": "tweede"}})]
    jsonl = "\n".join(codex_lines)
    assert extract_agent_message(jsonl) == "eerste\ntweede"
    (tmp_path / "events.jsonl").write_text(jsonl)
    codex = _stub(tmp_path, "codex", f'cat > /dev/null; cat "{tmp_path}/events.jsonl"\n')
    assert CliBackend("GPT", "openai-cli", command=codex, cwd=str(tmp_path)).execute("p", 10.0).text == "eerste\ntweede"

    missing = CliBackend("Claude", "claude-cli", command=str(tmp_path / "nope"))
    assert not missing.is_available()
    with pytest.raises(AdapterError) as ei:
        missing.execute("p", 5.0)
    assert ei.value.kind == "not_installed"


def test_factory_routing(server):
    assert wants_external("local-llm-x", {"endpoint": "http://h:1"})
    assert not wants_external("local-llm-x", {"endpoint": "http://h:1", "engine": {}})
    assert wants_external("claude-api", {"backend": "external"}) and not wants_external("claude-api", {})
    assert isinstance(create_external("openai-cli", {}, "GPT"), CliBackend)
    assert isinstance(create_external("gemini-api", {}, "G"), ApiBackend)

    from theroundtaible_amd.knights.registry import initialize_backends
    from theroundtaible_amd.types import RoundtableConfig
    cfg = RoundtableConfig.from_dict({
        "version": "1.0", "project": "t", "knights": [{"name": "Remote", "adapter": "local-llm-remote",
                                                       "capabilities": [], "priority": 1}],
        "rules": {}, "chronicle": ".roundtable/chronicle.md",
        "adapter_config": {"local-llm-remote": {"endpoint": server.url, "model": "tiny-llama", "source": "Ollama"}}})
    backends = initialize_backends(cfg)
    assert isinstance(backends["local-llm-remote"], LocalLlmHttpBackend)
    assert backends["local-llm-remote"].detected_ctx
