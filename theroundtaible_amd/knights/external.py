"""External knight backends: the reference's own transports, kept as opt-in seats.

Every adapter id resolves to an engine-hosted model by default (BASELINE north star). A
config can still seat a knight on the reference's transports by setting
``adapter_config[<id>].backend = "external"`` (or, for ``local-llm*`` ids, by giving an
``endpoint`` without an ``engine`` section). This is what lets a user of the reference switch
over without losing a seat, and what lets a table span nodes: a ``local-llm`` knight can point
at ``roundtable serve`` running on another MI355X node (same Ollama/OpenAI dialects).

Transports and the reference behaviour they keep:

* :class:`LocalLlmHttpBackend` — `src/adapters/local-llm.ts:6-249`: ``GET /v1/models`` probe
  (3 s), Ollama ``/api/show`` context detection (``*.context_length``), the source budget
  ``(ctx - 4096 - 3000, min 2000) * 4`` chars (LM Studio assumed 16384), Ollama ``/api/chat``
  with ``num_ctx = ceil(len/4) + 4096 + 512`` clamped to the detected window, OpenAI-compat
  ``/v1/chat/completions`` without ``max_tokens``, one retry after 3 s on "Model reloaded",
  LM Studio context-overflow hint, empty-response errors.
* :class:`ApiBackend` — `src/adapters/claude-api.ts:5-74`, `openai-api.ts:5-73`,
  `gemini-api.ts:5-70`: key from env then ``~/.theroundtaible/keys.json``, 16384 output
  tokens, vendor default models. ``base_url`` may be overridden (proxies, tests).
* :class:`CliBackend` — `src/adapters/claude-cli.ts:5-58`, `gemini-cli.ts:5-77`,
  `openai-cli.ts:5-94`: prompt on stdin, ``<cmd> --version`` availability probe, vendor flags
  (claude read-only tool deny-list and ``CLAUDECODE`` removed from the env; gemini plan mode
  with a retry without it and >50-char stdout tolerance; codex ``exec -`` JSONL
  ``agent_message`` extraction and ``--skip-git-repo-check`` outside a repository).

All failures are mapped through :func:`classify_error` (`src/utils/errors.ts:86-126`), so
the orchestrator's fallback/skip logic treats them exactly like engine failures.
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import time
import urllib.error
import urllib.request
from typing import Any, Callable, Dict, List, Optional

from ..errors import classify_error
from ..prompt import prompt_text
from ..store.keys import get_key
from .base import KnightBackend, TurnRequest, TurnResult

DEFAULT_TIMEOUT_S = 120.0
MAX_OUTPUT_TOKENS = 16384                      # claude-api.ts:47, openai-api.ts:47, gemini-api.ts:44
RESPONSE_RESERVE_TOKENS = 4096                 # local-llm.ts:63-66
OVERHEAD_RESERVE_TOKENS = 3000
LM_STUDIO_ASSUMED_CTX = 16384                  # local-llm.ts:60-61

HttpFn = Callable[[str, str, Optional[Dict[str, Any]], Dict[str, str], float], "HttpResponse"]


class HttpResponse:
    def __init__(self, status: int, body: str):
        self.status = status
        self.body = body

    @property
    def ok(self) -> bool:
        return 200 <= self.status < 300

    def json(self) -> Any:
        return json.loads(self.body)


def http_request(method: str, url: str, body: Optional[Dict[str, Any]] = None,
                 headers: Optional[Dict[str, str]] = None, timeout_s: float = DEFAULT_TIMEOUT_S) -> HttpResponse:
    """Blocking JSON HTTP call; HTTP error statuses are returned, transport failures raise."""
    data = json.dumps(body).encode() if body is not None else None
    hdrs = {"Content-Type": "application/json"} if data is not None else {}
    hdrs.update(headers or {})
    req = urllib.request.Request(url, data=data, method=method, headers=hdrs)
    try:
        with urllib.request.urlopen(req, timeout=timeout_s) as r:
            return HttpResponse(r.status, r.read().decode("utf-8", "replace"))
    except urllib.error.HTTPError as e:
        return HttpResponse(e.code, e.read().decode("utf-8", "replace"))
    except (TimeoutError, OSError) as e:
        if "timed out" in str(e).lower() or isinstance(e, TimeoutError):
            raise TimeoutError(f"request to {url} timed out after {timeout_s}s") from e
        raise


class LocalLlmHttpBackend(KnightBackend):
    """A knight served by an Ollama / LM Studio / ``roundtable serve`` endpoint."""

    def __init__(self, name: str, adapter_id: str, endpoint: str, model: str, source: Optional[str] = None,
                 http: Optional[Callable[..., HttpResponse]] = None, retry_delay_s: float = 3.0):
        self.name = name
        self.adapter_id = adapter_id
        self.endpoint = endpoint.rstrip("/")
        self.model = model
        self.source = source                       # "Ollama" | "LM Studio" | None
        self.http = http or http_request
        self.retry_delay_s = retry_delay_s
        self.detected_ctx: Optional[int] = None

    def is_available(self) -> bool:
        try:
            return self.http("GET", f"{self.endpoint}/v1/models", None, {}, 3.0).ok
        except Exception:  # noqa: BLE001 - probe failure == unavailable
            return False

    def detect_context_window(self) -> Optional[int]:
        if self.source == "Ollama":
            self.detected_ctx = self._ollama_context()
        return self.detected_ctx

    def _ollama_context(self) -> Optional[int]:
        try:
            r = self.http("POST", f"{self.endpoint}/api/show", {"name": self.model}, {}, 5.0)
            if not r.ok:
                return None
            info = r.json().get("model_info") or {}
            for k, v in info.items():
                if k.endswith(".context_length") and isinstance(v, (int, float)) and not isinstance(v, bool):
                    return int(v)
        except Exception:  # noqa: BLE001
            return None
        return None

    def max_source_chars(self) -> Optional[int]:
        ctx = self.detected_ctx or (LM_STUDIO_ASSUMED_CTX if self.source == "LM Studio" else None)
        if not ctx:
            return None
        return max(ctx - RESPONSE_RESERVE_TOKENS - OVERHEAD_RESERVE_TOKENS, 2000) * 4

    def _run(self, req: TurnRequest, timeout_s: float) -> TurnResult:
        prompt = prompt_text(req.prompt)
        t0 = time.perf_counter()
        try:
            try:
                text = self._once(prompt, timeout_s)
            except Exception as e:  # noqa: BLE001
                if "Model reloaded" not in str(e):
                    raise
                time.sleep(self.retry_delay_s)
                text = self._once(prompt, timeout_s)
        except Exception as e:  # noqa: BLE001
            raise classify_error(e, self.name) from e
        return TurnResult(text=text, metrics={"backend": "local-llm-http", "turn_ms": 1e3 * (time.perf_counter() - t0),
                                              "prompt_chars": len(prompt)})

    def _once(self, prompt: str, timeout_s: float) -> str:
        return self._ollama(prompt, timeout_s) if self.source == "Ollama" else self._openai(prompt, timeout_s)

    def _ollama(self, prompt: str, timeout_s: float) -> str:
        num_ctx = math.ceil(len(prompt) / 4) + RESPONSE_RESERVE_TOKENS + 512
        if self.detected_ctx:
            num_ctx = min(num_ctx, self.detected_ctx)
        r = self.http("POST", f"{self.endpoint}/api/chat",
                      {"model": self.model, "messages": [{"role": "user", "content": prompt}], "stream": False,
                       "options": {"num_ctx": num_ctx}}, {}, timeout_s)
        if not r.ok:
            raise RuntimeError(f"Ollama error ({r.status}): {r.body}")
        content = ((r.json() or {}).get("message") or {}).get("content")
        if not content:
            raise RuntimeError("Ollama returned empty response")
        return content

    def _openai(self, prompt: str, timeout_s: float) -> str:
        # No max_tokens: prompt + max_tokens > n_ctx is rejected by LM Studio (local-llm.ts:157-160).
        r = self.http("POST", f"{self.endpoint}/v1/chat/completions",
                      {"model": self.model, "messages": [{"role": "user", "content": prompt}]}, {}, timeout_s)
        if not r.ok:
            if self.source == "LM Studio" and is_context_window_error(r.body):
                est = math.ceil(len(prompt) / 4)
                raise RuntimeError(
                    f"LM Studio context window too small (prompt needs ~{est} tokens).\n"
                    "  Fix: In LM Studio → Developer → Model Settings → increase Context Length.\n"
                    "  Also uncheck the Response Limit, or set it higher.\n"
                    "  Note: higher context = more VRAM. Find the sweet spot for your GPU.")
            raise RuntimeError(f"Local LLM error ({r.status}): {r.body}")
        choices = (r.json() or {}).get("choices") or []
        content = ((choices[0] if choices else {}).get("message") or {}).get("content")
        if not content:
            raise RuntimeError("Local LLM returned empty response")
        return content


def is_context_window_error(body: str) -> bool:
    low = body.lower()
    return (("n_keep" in low and "n_ctx" in low) or "context length exceeded" in low
            or "maximum context length" in low or "too many tokens" in low)


API_VENDORS: Dict[str, Dict[str, str]] = {
    "claude-api": {"display": "Claude", "model": "claude-sonnet-4-6", "env_key": "ANTHROPIC_API_KEY",
                   "base_url": "https://api.anthropic.com", "label": "Anthropic"},
    "openai-api": {"display": "GPT", "model": "gpt-5.2", "env_key": "OPENAI_API_KEY",
                   "base_url": "https://api.openai.com", "label": "OpenAI"},
    "gemini-api": {"display": "Gemini", "model": "gemini-2.5-flash", "env_key": "GEMINI_API_KEY",
                   "base_url": "https://generativelanguage.googleapis.com", "label": "Gemini"},
}


class ApiBackend(KnightBackend):
    """Hosted vendor API seat (Anthropic messages / OpenAI chat completions / Gemini generateContent)."""

    def __init__(self, name: str, adapter_id: str, model: Optional[str] = None, env_key: Optional[str] = None,
                 base_url: Optional[str] = None, http: Optional[Callable[..., HttpResponse]] = None):
        v = API_VENDORS[adapter_id]
        self.name = name
        self.adapter_id = adapter_id
        self.model = model or v["model"]
        self.env_key = env_key or v["env_key"]
        self.base_url = (base_url or v["base_url"]).rstrip("/")
        self.label = v["label"]
        self.http = http or http_request

    def is_available(self) -> bool:
        return bool(get_key(self.env_key))

    def _run(self, req: TurnRequest, timeout_s: float) -> TurnResult:
        prompt = prompt_text(req.prompt)
        t0 = time.perf_counter()
        try:
            key = get_key(self.env_key)
            if not key:
                raise RuntimeError(f"{self.label} API key not set. Set {self.env_key} or run 'roundtable init'.")
            text = self._call(prompt, key, timeout_s)
        except Exception as e:  # noqa: BLE001
            raise classify_error(e, self.name) from e
        return TurnResult(text=text, metrics={"backend": self.adapter_id, "turn_ms": 1e3 * (time.perf_counter() - t0)})

    def _call(self, prompt: str, key: str, timeout_s: float) -> str:
        if self.adapter_id == "claude-api":
            r = self.http("POST", f"{self.base_url}/v1/messages",
                          {"model": self.model, "max_tokens": MAX_OUTPUT_TOKENS,
                           "messages": [{"role": "user", "content": prompt}]},
                          {"x-api-key": key, "anthropic-version": "2023-06-01"}, timeout_s)
            self._check(r)
            text = next((c.get("text") for c in (r.json().get("content") or []) if c.get("type") == "text"), None)
        elif self.adapter_id == "openai-api":
            r = self.http("POST", f"{self.base_url}/v1/chat/completions",
                          {"model": self.model, "max_completion_tokens": MAX_OUTPUT_TOKENS,
                           "messages": [{"role": "user", "content": prompt}]},
                          {"Authorization": f"Bearer {key}"}, timeout_s)
            self._check(r)
            choices = r.json().get("choices") or []
            text = ((choices[0] if choices else {}).get("message") or {}).get("content")
        else:
            r = self.http("POST", f"{self.base_url}/v1beta/models/{self.model}:generateContent?key={key}",
                          {"contents": [{"parts": [{"text": prompt}]}],
                           "generationConfig": {"maxOutputTokens": MAX_OUTPUT_TOKENS}}, {}, timeout_s)
            self._check(r)
            cands = r.json().get("candidates") or []
            parts = (((cands[0] if cands else {}).get("content") or {}).get("parts") or [{}])
            text = parts[0].get("text") if parts else None
        if not text:
            raise RuntimeError(f"{self.label} API returned empty response")
        return text

    def _check(self, r: HttpResponse) -> None:
        if not r.ok:
            raise RuntimeError(f"{self.label} API error ({r.status}): {r.body}")


CLAUDE_DENIED_TOOLS = "Edit,Write,Bash,Read,Glob,Grep,NotebookEdit,WebFetch,WebSearch,Task"
CLI_VENDORS: Dict[str, Dict[str, str]] = {
    "claude-cli": {"display": "Claude", "command": "claude", "label": "Claude CLI"},
    "gemini-cli": {"display": "Gemini", "command": "gemini", "label": "Gemini CLI", "model": "gemini-2.5-pro"},
    "openai-cli": {"display": "GPT", "command": "codex", "label": "Codex CLI"},
}


class CliBackend(KnightBackend):
    """Vendor CLI seat: prompt on stdin, response on stdout (no shell, explicit argv)."""

    def __init__(self, name: str, adapter_id: str, command: Optional[str] = None, model: Optional[str] = None,
                 cwd: Optional[str] = None):
        v = CLI_VENDORS[adapter_id]
        self.name = name
        self.adapter_id = adapter_id
        self.command = command or v["command"]
        self.model = model or v.get("model")
        self.label = v["label"]
        self.cwd = cwd

    def is_available(self) -> bool:
        try:
            return subprocess.run([self.command, "--version"], capture_output=True, timeout=10,
                                  cwd=self.cwd).returncode == 0
        except (OSError, subprocess.SubprocessError):
            return False

    def _exec(self, args: List[str], prompt: str, timeout_s: float,
              env: Optional[Dict[str, str]] = None) -> subprocess.CompletedProcess:
        try:
            return subprocess.run([self.command] + args, input=prompt, capture_output=True, text=True,
                                  timeout=timeout_s, env=env, cwd=self.cwd)
        except subprocess.TimeoutExpired as e:
            raise TimeoutError(f"{self.label} timed out after {timeout_s}s") from e
        except FileNotFoundError as e:
            raise RuntimeError(f"ENOENT: {self.command} not found") from e

    def _fail(self, r: subprocess.CompletedProcess) -> RuntimeError:
        return RuntimeError(f"{self.label} failed (exit {r.returncode}): {r.stderr or r.stdout or 'Unknown error'}")

    def _run(self, req: TurnRequest, timeout_s: float) -> TurnResult:
        prompt = prompt_text(req.prompt)
        t0 = time.perf_counter()
        try:
            text = getattr(self, "_" + self.adapter_id.split("-")[0])(prompt, timeout_s)
        except Exception as e:  # noqa: BLE001
            raise classify_error(e, self.name) from e
        return TurnResult(text=text, metrics={"backend": self.adapter_id, "turn_ms": 1e3 * (time.perf_counter() - t0)})

    def _claude(self, prompt: str, timeout_s: float) -> str:
        env = dict(os.environ)
        env.pop("CLAUDECODE", None)
        r = self._exec(["--print", "--output-format", "text", "--disallowedTools", CLAUDE_DENIED_TOOLS],
                       prompt, timeout_s, env)
        if r.returncode != 0:
            raise self._fail(r)
        return r.stdout

    def _gemini(self, prompt: str, timeout_s: float) -> str:
        r = self._exec(["-p", "", "--approval-mode", "plan", "-o", "text", "-m", self.model], prompt, timeout_s)
        if r.returncode != 0 and "approval-mode" in (r.stderr or ""):
            r = self._exec(["-p", "", "-o", "text", "-m", self.model], prompt, timeout_s)
        if r.stdout and len(r.stdout.strip()) > 50:      # useful output despite a non-zero exit
            return r.stdout
        if r.returncode != 0:
            raise self._fail(r)
        return r.stdout

    def _openai(self, prompt: str, timeout_s: float) -> str:
        args = ["exec", "-", "--sandbox", "read-only", "--json", "--color", "never"]
        inside = subprocess.run(["git", "rev-parse", "--is-inside-work-tree"], capture_output=True,
                                cwd=self.cwd).returncode == 0
        if not inside:
            args.append("--skip-git-repo-check")
        r = self._exec(args, prompt, timeout_s)
        if r.returncode != 0:
            raise self._fail(r)
        msg = extract_agent_message(r.stdout)
        if not msg:
            raise RuntimeError("Codex CLI returned no agent_message events")
        return msg


def extract_agent_message(jsonl: str) -> str:
    """Join the ``item.completed``/``agent_message`` texts of a Codex JSONL stream."""
    parts = []
    for line in jsonl.splitlines():
        s = line.strip()
        if not s.startswith("{"):
            continue
        try:
            evt = json.loads(s)
        except ValueError:
            continue
        item = evt.get("item") if isinstance(evt, dict) else None
        if (evt.get("type") == "item.completed" and isinstance(item, dict) and item.get("type") == "agent_message"
                and isinstance(item.get("text"), str)):
            parts.append(item["text"])
    return "\n".join(parts).strip()


def wants_external(adapter_id: str, ac: Dict[str, Any]) -> bool:
    """True when a config seats this adapter id on its reference transport instead of the engine."""
    backend = ac.get("backend")
    if backend is not None:
        return backend == "external"
    # A reference-shaped local-llm entry (endpoint, no engine section) keeps talking HTTP.
    return adapter_id.startswith("local-llm") and bool(ac.get("endpoint")) and "engine" not in ac


def create_external(adapter_id: str, ac: Dict[str, Any], name: str) -> KnightBackend:
    if adapter_id.startswith("local-llm"):
        b = LocalLlmHttpBackend(name, adapter_id, str(ac.get("endpoint", "http://localhost:11434")),
                                str(ac.get("model", "")), ac.get("source"))
        b.detect_context_window()                  # adapters.ts:78-83
        return b
    if adapter_id in API_VENDORS:
        return ApiBackend(name, adapter_id, ac.get("model"), ac.get("env_key"), ac.get("base_url"))
    if adapter_id in CLI_VENDORS:
        # adapter_config.args is ignored, as in the reference (commands are hard-coded per vendor).
        return CliBackend(name, adapter_id, ac.get("command"), ac.get("model"))
    raise ValueError(f'adapter "{adapter_id}" has no external transport')
