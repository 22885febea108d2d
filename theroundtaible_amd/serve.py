"""``roundtable serve``: host a knight model on this GPU behind an OpenAI-/Ollama-compatible
HTTP endpoint (bound to 127.0.0.1 by default).

Why: the reference's only self-hosted path is its ``local-llm`` adapter talking to an
Ollama / LM Studio server (`src/adapters/local-llm.ts:6-249`, discovery in
`src/utils/local-detect.ts:103-134`). This module is that *server side*, built on the
MI355X engine instead of a third-party runtime, so any client that speaks those two
dialects (including another roundtable's knights, scripts, IDE plugins) can use a
resident-KV, hipGraph-decoding MI355X knight.

Serving model:

* one :class:`~theroundtaible_amd.engine.Engine` per process (one process per GPU; run
  several ``serve`` processes for several GPUs);
* a model too large or too slow for one GPU is served **tensor-parallel** (``serve --tp N``:
  N ranks, one per GPU, the Megatron split of parallel/tp.py with K9 / RCCL collectives): rank 0
  runs the HTTP front end and the scheduler on a :class:`MirroredEngine`, which broadcasts every
  engine operation (admit = prefill + first token, decode chunk, release) over the gloo control
  plane before running it; ranks 1..N-1 execute the same operations in the same order
  (:func:`serve_follower`), so every collective inside them lines up. Sampling is a counter RNG
  keyed by (seed, sequence, position) over all-gathered logits, so every rank draws the same
  tokens; rank 0's are the ones returned;
* continuous batching (:class:`Scheduler`): between decode chunks finished requests leave
  and waiting ones are prefilled and join, so concurrent clients share one hipGraph replay
  per token (up to ``max_batch``) — the batching the round table uses for parallel knights;
* conversation KV reuse: a request carrying ``"user"`` (OpenAI) or ``"session"`` keeps
  its KV sequence resident under that key, so the next request of the conversation
  prefills only its new tokens (longest-common-prefix reuse, engine.sync_prefix);
  anonymous requests get a fresh sequence that is released afterwards;
* endpoints: ``GET /v1/models``, ``POST /v1/chat/completions`` (``stream`` answered as one
  SSE delta + ``[DONE]``), ``POST /v1/completions``, ``POST /api/chat`` and
  ``POST /api/show`` (Ollama), ``GET /health``, ``GET /metrics`` (Prometheus text).
"""
from __future__ import annotations

import itertools
import json
import os
import queue
import sys
import threading
import time
import uuid
from dataclasses import dataclass, field
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, Tuple

from .engine import Engine, EngineConfig, SamplingParams, Turn
from .engine.engine import cut_at_stop
from .utils import failsafe

ROLE_TAGS = {"system": "Systeem", "user": "Gebruiker", "assistant": "Assistent"}


def _content_text(content: Any) -> str:
    if isinstance(content, list):  # OpenAI content parts
        return "".join(p.get("text", "") for p in content if isinstance(p, dict))
    return str(content)


def render_chat(messages: List[Dict[str, Any]]) -> str:
    """Plain role-tagged transcript ending in an open assistant turn (the bundled models
    have no chat special tokens; the tags match the roundtable's own prompt style)."""
    return "".join(s.text for s in chat_segments(messages)[0])


def cut_at_stop_strings(text: str, stops) -> Tuple[str, bool]:
    """``text`` up to the earliest occurrence of any stop string (OpenAI ``stop``: the stop string
    itself is not returned), and whether one occurred."""
    cut = -1
    for st in stops:
        i = text.find(st) if st else -1
        if i >= 0 and (cut < 0 or i < cut):
            cut = i
    return (text[:cut], True) if cut >= 0 else (text, False)


def stop_prefix_hold(text: str, stops) -> int:
    """Characters at the end of ``text`` that may still grow into a stop string (a streamed piece
    holds them back until the next piece decides)."""
    hold = 0
    for st in stops:
        for k in range(min(len(st) - 1, len(text)), hold, -1):
            if text.endswith(st[:k]):
                hold = k
                break
    return hold


def parse_stops(v) -> Tuple[str, ...]:
    if v is None:
        return ()
    if isinstance(v, str):
        v = [v]
    if not isinstance(v, list) or not all(isinstance(x, str) for x in v) or len(v) > 16:
        raise ValueError("'stop' must be a string or a list of at most 16 strings")
    return tuple(x for x in v if x)


def chat_segments(messages: List[Dict[str, Any]]):
    """The :func:`render_chat` transcript as prompt segments, plus how many leading segments
    are the conversation's system message(s) — the part many clients send identically."""
    from .prompt import Segment
    parts, n_sys, leading = [], 0, True
    for m in messages:
        role = str(m.get("role", "user"))
        content = _content_text(m.get("content", ""))
        sep = "\n" if parts else ""
        parts.append(Segment(f"{sep}### {ROLE_TAGS.get(role, role)}:\n{content}\n"))
        if leading and role == "system":
            n_sys = len(parts)
        else:
            leading = False
    parts.append(Segment(("\n" if parts else "") + f"### {ROLE_TAGS['assistant']}:\n"))
    return parts, n_sys


class ContextLengthError(ValueError):
    """A prompt longer than the model's positions (HTTP 400, OpenAI's error code)."""
    code = "context_length_exceeded"


@dataclass
class _Request:
    key: str
    prompt: str
    params: SamplingParams
    persistent: bool
    done: threading.Event = field(default_factory=threading.Event)
    result: Any = None
    error: Optional[BaseException] = None
    # streaming: the scheduler puts the generated ids so far after every host readback (the first
    # token after prefill, then every decode chunk), then None when the request is complete
    stream_q: Optional["queue.Queue"] = None
    cancelled: bool = False        # the streaming client went away: stop decoding it
    stops: Tuple[str, ...] = ()    # OpenAI "stop" / Ollama options.stop strings

    def publish(self, gen: List[int]) -> None:
        if self.stream_q is not None:
            self.stream_q.put(list(gen))


@dataclass
class _Active:
    req: _Request
    seq: Any
    turn: Turn
    gen: List[int]
    metrics: Dict[str, Any]
    t0: float
    checked: int = 0     # tokens of gen already scanned for stop strings


class Scheduler:
    """Continuous batching over one engine.

    Between decode chunks (``chunk`` tokens, one hipGraph replay per token for the whole
    batch) finished requests leave and waiting ones join: a newcomer is prefilled (delta only,
    LCP reuse) and its first token sampled, then it decodes in the same batch as everyone
    else — so a long generation never blocks a short one behind it for more than a chunk.
    """

    def __init__(self, engine: Engine, max_batch: int = 16, timeout_s: float = 600.0, chunk: int = 16):
        self.engine = engine
        self.max_batch = max(1, int(max_batch))
        self.timeout_s = timeout_s
        self.chunk = max(1, int(chunk))
        self.q: "queue.Queue[_Request]" = queue.Queue()
        self.stats = {"requests": 0, "batches": 0, "prompt_tokens": 0, "completion_tokens": 0,
                      "reused_tokens": 0, "busy_s": 0.0, "errors": 0, "admitted_midflight": 0,
                      "decode_steps": 0, "decode_rows": 0, "prefill_s": 0.0}
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self.thread = threading.Thread(target=self._loop, name="roundtable-serve", daemon=True)
        self.thread.start()

    def submit(self, req: _Request) -> _Request:
        self.q.put(req)
        return req

    def close(self) -> None:
        self._stop.set()
        self.q.put(None)  # type: ignore[arg-type]
        self.thread.join(timeout=5)

    # ---- queue --------------------------------------------------------------------------------
    def _take(self, room: int, busy_keys: set, block: bool) -> List[_Request]:
        out: List[_Request] = []
        later: List[_Request] = []
        keys = set(busy_keys)
        while len(out) < room:
            try:
                r = self.q.get(timeout=0.5) if (block and not out) else self.q.get_nowait()
            except queue.Empty:
                break
            if r is None:
                self._stop.set()
                break
            if r.key in keys:          # one in-flight turn per sequence
                later.append(r)
                continue
            keys.add(r.key)
            out.append(r)
        for r in later:
            self.q.put(r)
        return out

    # ---- completion ---------------------------------------------------------------------------
    def _finished(self, a: _Active) -> bool:
        if a.req.cancelled:
            return True
        stops = self.engine.tokenizer.stop_ids
        if len(a.gen) >= a.req.params.max_new_tokens or (not a.req.params.ignore_eos and not stops.isdisjoint(a.gen)):
            return True
        # stop strings: checked after every decode chunk on the decoded TAIL only (the tokens since
        # the last check plus enough earlier ones to hold the longest stop string), so a long reply
        # costs O(n) decoding, not O(n^2)
        if not a.req.stops:
            return False
        k = (len(a.gen) - a.checked) + max(len(st) for st in a.req.stops) + 8
        a.checked = len(a.gen)
        return cut_at_stop_strings(self.engine.tokenizer.decode(a.gen[-k:]), a.req.stops)[1]

    def _complete(self, a: _Active, error: Optional[BaseException] = None) -> None:
        r = a.req
        if error is not None:
            r.error = error
            with self._lock:
                self.stats["errors"] += 1
        else:
            gen = a.gen[:a.req.params.max_new_tokens]
            if not a.req.params.ignore_eos:
                gen = cut_at_stop(gen, self.engine.tokenizer.stop_ids)
            m = dict(a.metrics, decode_tokens=len(gen), turn_ms=(time.perf_counter() - a.t0) * 1e3)
            text = self.engine.tokenizer.decode(gen)
            if r.stops:
                text, hit = cut_at_stop_strings(text, r.stops)
                m["stop_string"] = hit
            r.result = _Output(text, gen, m)
            with self._lock:
                self.stats["requests"] += 1
                self.stats["prompt_tokens"] += int(m.get("prompt_tokens", 0))
                self.stats["completion_tokens"] += len(gen)
                self.stats["reused_tokens"] += int(m.get("reused_tokens", 0))
        if not r.persistent:
            try:
                self.engine.release(r.key)
            except Exception:  # noqa: BLE001
                pass
        r.done.set()
        if r.stream_q is not None:
            r.stream_q.put(None)

    # ---- engine loop --------------------------------------------------------------------------
    def _loop(self) -> None:
        active: List[_Active] = []
        while not self._stop.is_set():
            new = self._take(self.max_batch - len(active), {a.req.key for a in active}, block=not active)
            t_busy = time.perf_counter()
            if new:
                turns = [Turn(r.key, r.prompt, r.params, timeout_s=self.timeout_s) for r in new]
                t_pf = time.perf_counter()
                try:
                    started = self.engine.start_turns(turns)
                except BaseException as e:  # noqa: BLE001 - reported per request
                    for r in new:
                        self._complete(_Active(r, None, None, [], {}, time.perf_counter()), e)
                    started = []
                with self._lock:
                    self.stats["prefill_s"] += time.perf_counter() - t_pf
                    if active and started:
                        self.stats["admitted_midflight"] += len(started)
                for r, t, (sq, first, m) in zip(new, turns, started):
                    a = _Active(r, sq, t, [first], dict(m, batch=0), time.perf_counter())
                    r.publish(a.gen)
                    if self._finished(a):
                        self._complete(a)
                    else:
                        active.append(a)
            if not active:
                continue
            steps = min(self.chunk, min(a.req.params.max_new_tokens - len(a.gen) for a in active))
            try:
                outs = self.engine.continue_decode([a.seq for a in active], [a.turn for a in active],
                                                   [a.gen[-1] for a in active], max(1, steps))
            except BaseException as e:  # noqa: BLE001
                for a in active:
                    self._complete(a, e)
                active = []
                continue
            for a, toks in zip(active, outs):
                a.gen.extend(toks)
                a.metrics["batch"] = max(a.metrics.get("batch", 0), len(active))
                if not self._finished(a):          # a finished request's text comes with its result
                    a.req.publish(a.gen)
            with self._lock:
                self.stats["batches"] += 1
                self.stats["decode_steps"] += max(1, steps)
                self.stats["decode_rows"] += max(1, steps) * len(active)
                self.stats["busy_s"] += time.perf_counter() - t_busy
            still = []
            for a in active:
                (self._complete(a) if self._finished(a) else still.append(a))
            active = still


PING_INTERVAL_S = float(os.environ.get("ROUNDTABLE_SERVE_PING_S", "600"))


class MirroredEngine:
    """Rank 0's view of a tensor-parallel engine: the scheduler's engine operations are announced
    to the follower ranks (:func:`serve_follower`) over the control plane, then run locally —
    the followers run the same call with the same arguments, so the TP collectives inside
    match. Everything else (tokenizer, stats, capacity, health) reads the local engine."""

    def __init__(self, engine: Engine, cluster, op_limit_s: Optional[float] = None):
        self._engine, self._cluster = engine, cluster
        self._op_limit_s = op_limit_s
        self._lock = threading.Lock()    # one announced operation at a time, in issue order
        self.diverged: Optional[str] = None   # set when a follower's outcome differed from ours
        self._last_op = time.monotonic()
        self._stopped = False
        # an idle server pings its followers: their wait for the next operation then
        # never runs into the wait group's (7-day) timeout, however long no request comes
        self.ping_s = PING_INTERVAL_S
        threading.Thread(target=self._keepalive, name="serve-tp-keepalive", daemon=True).start()

    def _keepalive(self) -> None:
        while True:
            time.sleep(min(self.ping_s, 60.0))
            with self._lock:
                if self._stopped or self.diverged is not None:
                    return
                if time.monotonic() - self._last_op >= self.ping_s:
                    self._cluster.broadcast_object(("ping",), wait=True)
                    self._last_op = time.monotonic()

    def __getattr__(self, name):
        return getattr(self._engine, name)

    def _run(self, op: tuple, fn):
        """Announce ``op``, run it here, then agree on every rank's outcome (one gloo gather):
        equal inputs give equal outcomes on every rank (the KV pools are agreed at creation), so a
        mismatch means the group's state has diverged — the followers leave their loop, and this
        engine refuses every later operation instead of entering collectives no peer will join."""
        if self.diverged is not None:
            raise RuntimeError(f"tensor-parallel group stopped: {self.diverged}")
        # announced over the wait group (a follower idles in that broadcast between requests);
        # the operation and the outcome gather run on the containment-timeout groups and under a
        # stage limit, so a follower that stalls mid-operation ends the server with a message
        self._cluster.broadcast_object(op, wait=True)
        self._last_op = time.monotonic()
        res, err = None, None
        try:
            with failsafe.stage(f"serve {op[0]}", limit_s=self._op_limit_s):
                res = fn()
        except Exception as e:  # noqa: BLE001 - re-raised after the agreement round
            err = e
        outs = self._cluster.all_gather_object(_outcome(err))
        if any(o != outs[0] for o in outs):
            self.diverged = f"ranks disagree on {op[0]!r}: {outs}"
            self._engine.healthy = False
            raise RuntimeError(f"tensor-parallel group stopped: {self.diverged}") from err
        if err is not None:
            raise err
        return res

    def start_turns(self, turns):
        with self._lock:
            return self._run(("start", list(turns)), lambda: self._engine.start_turns(turns))

    def continue_decode(self, seqs, turns, last, steps):
        with self._lock:
            return self._run(("decode", [s.key for s in seqs], list(turns), [int(x) for x in last], int(steps)),
                             lambda: self._engine.continue_decode(seqs, turns, last, steps))

    def release(self, key: str) -> None:
        with self._lock:
            self._run(("release", key), lambda: self._engine.release(key))

    def stop_followers(self) -> None:
        with self._lock:
            if self.diverged is None and not self._stopped:
                self._cluster.broadcast_object(("stop",), wait=True)
            self._stopped = True


def _outcome(err: Optional[BaseException]) -> tuple:
    """What every rank of the group must agree on after an operation: ok, or the error's type."""
    return ("ok",) if err is None else ("err", type(err).__name__)


def serve_follower(engine: Engine, cluster, op_limit_s: Optional[float] = None) -> int:
    """Ranks 1..N-1 of ``serve --tp N``: run rank 0's engine operations in its order until it
    announces ``stop``. Returns the number of operations executed. After each operation the
    ranks gather their outcomes (MirroredEngine._run): rank 0 reports a request's error; if
    any rank's outcome differs, every rank leaves the loop (the group has diverged)."""
    n = 0
    while True:
        op = cluster.broadcast_object(None, wait=True)     # idle between requests: no timeout
        kind = op[0]
        if kind == "stop":
            return n
        if kind == "ping":                                  # rank 0's idle keepalive
            continue
        err = None
        try:
            with failsafe.stage(f"serve {kind}", limit_s=op_limit_s):
                if kind == "start":
                    engine.start_turns(op[1])
                elif kind == "decode":
                    seqs = [engine.kv.seqs[k] for k in op[1]]
                    engine.continue_decode(seqs, op[2], op[3], op[4])
                elif kind == "release":
                    engine.release(op[1])
        except Exception as e:  # noqa: BLE001 - rank 0 reports the request's error
            err = e
        outs = cluster.all_gather_object(_outcome(err))
        n += 1
        if any(o != outs[0] for o in outs):
            return n


class _HTTPServer(ThreadingHTTPServer):
    """``ThreadingHTTPServer`` with a listen backlog for bursts of clients. socketserver's default
    backlog is 5: when more connections arrive than the accept thread takes in time (it shares the
    GIL with the scheduler and every handler thread), Linux resets the overflow — 32-64 client
    bursts lost 1-9 requests (CPU repro with 128 simultaneous clients against a
    5-deep backlog: 54 of 384 requests reset, 0 with 1024). The kernel caps the value at
    ``net.core.somaxconn``."""
    request_queue_size = 1024
    daemon_threads = True
    allow_reuse_address = True


@dataclass
class _Output:
    text: str
    ids: List[int]
    metrics: Dict[str, Any]


class RoundtableServer:
    """The HTTP front end. ``start()`` serves on a background thread; ``serve_forever()`` blocks."""

    _anon = itertools.count()

    def __init__(self, engine: Engine, model_name: str, host: str = "127.0.0.1", port: int = 8000,
                 max_batch: int = 16, default_max_tokens: int = 512, timeout_s: float = 600.0,
                 share_system_prompts: bool = True):
        self.engine = engine
        self.model_name = model_name
        self.share_system_prompts = share_system_prompts
        self.default_max_tokens = default_max_tokens
        self.sched = Scheduler(engine, max_batch, timeout_s)
        self.started = time.time()
        server = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, fmt, *args):  # quiet by default (one line per request)
                pass

            def log_error(self, fmt, *args):     # errors are never silent (stderr)
                sys.stderr.write("roundtable serve: %s - %s\n" % (self.address_string(), fmt % args))

            def _send(self, code: int, obj: Any, ctype: str = "application/json") -> None:
                body = obj if isinstance(obj, bytes) else (
                    obj.encode() if isinstance(obj, str) else json.dumps(obj).encode())
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _chunk(self, data: bytes) -> None:
                """One HTTP/1.1 chunk (Transfer-Encoding: chunked), flushed at once."""
                self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
                self.wfile.flush()

            def _stream(self, prompt, body, session, first, delta, last, sse: bool = True) -> None:
                """Stream a completion as it decodes: SSE ``data:`` events (OpenAI) or NDJSON lines
                (Ollama). Text goes out after every host readback of the decode loop (the first
                token after prefill, then each decode chunk); the pieces concatenate to exactly
                the non-streamed text (Server.visible_text, the final result's cut and decode)."""
                r = server.submit(prompt, body, session, stream=True)
                self.send_response(200)
                self.send_header("Content-Type", "text/event-stream" if sse else "application/x-ndjson")
                self.send_header("Cache-Control", "no-cache")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()

                def emit(obj) -> None:
                    self._chunk((f"data: {json.dumps(obj)}\n\n" if sse else json.dumps(obj) + "\n").encode())
                try:
                    self._stream_body(r, emit, first, delta, last, sse)
                except (BrokenPipeError, ConnectionResetError):
                    # the client went away mid-stream: its request stops decoding at the next chunk
                    # (and releases its KV) instead of running to max_tokens for nobody
                    r.cancelled = True
                    self.close_connection = True

            def _stream_body(self, r, emit, first, delta, last, sse: bool) -> None:
                if first is not None:
                    emit(first)
                sent = ""
                deadline = time.monotonic() + server.sched.timeout_s + 30
                while True:
                    try:
                        ids = r.stream_q.get(timeout=max(0.1, deadline - time.monotonic()))
                    except queue.Empty:
                        r.error = r.error or TimeoutError("generation timed out")
                        break
                    if ids is None:
                        break
                    text = server.visible_text(ids, r.params, r.stops)
                    if text.startswith(sent) and len(text) > len(sent):
                        emit(delta(text[len(sent):]))
                        sent = text
                if r.error is None and r.result is not None:
                    final = r.result.text
                    if final.startswith(sent) and len(final) > len(sent):
                        emit(delta(final[len(sent):]))
                    emit(last(r.result, r))
                else:
                    emit({"error": {"message": str(r.error), "type": "server_error"}})
                if sse:
                    self._chunk(b"data: [DONE]\n\n")
                self._chunk(b"")                      # end of the chunked body

            def _json_body(self) -> Dict[str, Any]:
                n = int(self.headers.get("Content-Length") or 0)
                raw = self.rfile.read(n) if n else b"{}"
                try:
                    d = json.loads(raw or b"{}")
                except ValueError:
                    raise ValueError("request body is not valid JSON")
                if not isinstance(d, dict):
                    raise ValueError("request body must be a JSON object")
                return d

            def do_GET(self):  # noqa: N802
                if self.path.rstrip("/") == "/v1/models":
                    self._send(200, {"object": "list", "data": [
                        {"id": server.model_name, "object": "model", "created": int(server.started),
                         "owned_by": "theroundtaible-amd"}]})
                elif self.path.rstrip("/") in ("/health", ""):
                    self._send(200, {"status": "ok" if server.engine.healthy else "unhealthy",
                                     "model": server.model_name, "device": str(server.engine.device),
                                     "tp": int(server.engine.tp.size)})
                elif self.path.rstrip("/") == "/metrics":
                    self._send(200, server.metrics_text(), "text/plain; version=0.0.4")
                else:
                    self._send(404, {"error": {"message": f"no route {self.path}"}})

            def do_POST(self):  # noqa: N802
                path = self.path.rstrip("/")
                try:
                    body = self._json_body()
                    if path == "/v1/chat/completions":
                        self._chat_openai(body)
                    elif path == "/v1/completions":
                        self._completion_openai(body)
                    elif path == "/api/chat":
                        self._chat_ollama(body)
                    elif path == "/api/show":
                        self._send(200, server.show())
                    else:
                        self._send(404, {"error": {"message": f"no route {self.path}"}})
                except ValueError as e:
                    self._send(400, {"error": {"message": str(e), "type": "invalid_request_error",
                                               "code": getattr(e, "code", None)}})
                except Exception as e:  # noqa: BLE001
                    self._send(500, {"error": {"message": str(e), "type": "server_error"}})

            def _chat_openai(self, body):
                msgs = body.get("messages")
                if not isinstance(msgs, list) or not msgs:
                    raise ValueError("'messages' must be a non-empty list")
                rid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
                if body.get("stream"):
                    base = {"id": rid, "object": "chat.completion.chunk", "created": int(time.time()),
                            "model": server.model_name}

                    def piece(delta, finish=None):
                        return dict(base, choices=[{"index": 0, "delta": delta, "finish_reason": finish}])
                    include_usage = bool((body.get("stream_options") or {}).get("include_usage"))

                    def last(out, r):
                        # OpenAI stream_options.include_usage: the finishing chunk carries the usage
                        end = piece({}, server.finish(out, r))
                        if include_usage:
                            end["usage"] = server.usage(out)
                        return end
                    self._stream(server.chat_prompt(msgs), body, body.get("user") or body.get("session"),
                                 first=piece({"role": "assistant", "content": ""}),
                                 delta=lambda t: piece({"content": t}), last=last)
                    return
                out, r = server.generate(server.chat_prompt(msgs), body, body.get("user") or body.get("session"))
                usage = server.usage(out)
                self._send(200, {"id": rid, "object": "chat.completion", "created": int(time.time()),
                                 "model": server.model_name,
                                 "choices": [{"index": 0, "message": {"role": "assistant", "content": out.text},
                                              "finish_reason": server.finish(out, r)}],
                                 "usage": usage})

            def _completion_openai(self, body):
                prompt = body.get("prompt")
                if isinstance(prompt, list):
                    prompt = "".join(str(p) for p in prompt)
                if not isinstance(prompt, str):
                    raise ValueError("'prompt' must be a string")
                if body.get("stream"):
                    base = {"id": f"cmpl-{uuid.uuid4().hex[:24]}", "object": "text_completion",
                            "created": int(time.time()), "model": server.model_name}

                    def piece(text, finish=None):
                        return dict(base, choices=[{"index": 0, "text": text, "finish_reason": finish}])
                    self._stream(prompt, body, body.get("user"), first=None, delta=piece,
                                 last=lambda out, r: piece("", server.finish(out, r)))
                    return
                out, r = server.generate(prompt, body, body.get("user"))
                self._send(200, {"id": f"cmpl-{uuid.uuid4().hex[:24]}", "object": "text_completion",
                                 "created": int(time.time()), "model": server.model_name,
                                 "choices": [{"index": 0, "text": out.text, "finish_reason": server.finish(out, r)}],
                                 "usage": server.usage(out)})

            def _chat_ollama(self, body):
                msgs = body.get("messages")
                if not isinstance(msgs, list) or not msgs:
                    raise ValueError("'messages' must be a non-empty list")
                opts = body.get("options") or {}
                params = {"temperature": opts.get("temperature"), "top_p": opts.get("top_p"),
                          "top_k": opts.get("top_k"), "seed": opts.get("seed"),
                          "max_tokens": opts.get("num_predict"), "stop": opts.get("stop")}
                if body.get("stream"):
                    # Ollama's NDJSON stream: one message object per line, then a done record
                    # (a request without "stream" keeps the one-object reply of rounds 1-5)
                    def line(text):
                        return {"model": server.model_name, "created_at": time.strftime("%Y-%m-%dT%H:%M:%SZ"),
                                "message": {"role": "assistant", "content": text}, "done": False}

                    def done(out, r):
                        return {"model": server.model_name, "created_at": time.strftime("%Y-%m-%dT%H:%M:%SZ"),
                                "message": {"role": "assistant", "content": ""}, "done": True,
                                "done_reason": server.finish(out, r),
                                "prompt_eval_count": int(out.metrics.get("prompt_tokens", 0)),
                                "eval_count": len(out.ids)}
                    self._stream(server.chat_prompt(msgs), params, body.get("session"), first=None, delta=line,
                                 last=done, sse=False)
                    return
                out, _ = server.generate(server.chat_prompt(msgs), params, body.get("session"))
                self._send(200, {"model": server.model_name, "created_at": time.strftime("%Y-%m-%dT%H:%M:%SZ"),
                                 "message": {"role": "assistant", "content": out.text}, "done": True,
                                 "prompt_eval_count": int(out.metrics.get("prompt_tokens", 0)),
                                 "eval_count": len(out.ids)})

        self.httpd = _HTTPServer((host, port), Handler)
        self.host, self.port = self.httpd.server_address[:2]
        self._thread: Optional[threading.Thread] = None

    # ---- request plumbing -----------------------------------------------------------------
    def chat_prompt(self, messages: List[Dict[str, Any]]):
        """The conversation through the checkpoint's own chat template when the engine has one
        (marked templated: no extra wrap), else the plain role-tagged transcript."""
        from .prompt import Prompt, Segment
        render = getattr(self.engine.tokenizer, "render_chat", None)
        if render is not None:
            norm = [{"role": str(m.get("role", "user")), "content": _content_text(m.get("content", ""))}
                    for m in messages]
            text = render(norm)
            if text is not None:
                return Prompt([Segment(text)], templated=True)
        segs, n_sys = chat_segments(messages)
        if n_sys and self.share_system_prompts:
            # clients sending the same system prompt share ONE resident copy of its KV
            # (engine shared-prefix groups: prefilled once, attention reads it once per step)
            import hashlib
            sys_text = "".join(x.text for x in segs[:n_sys])
            key = "sys:" + hashlib.sha1(sys_text.encode("utf-8")).hexdigest()[:16]
            return Prompt(segs, shared_key=key, shared_segments=n_sys)
        return Prompt(segs)

    def sampling(self, body: Dict[str, Any]) -> SamplingParams:
        def num(key, default, cast):
            v = body.get(key)
            return default if v is None else cast(v)
        max_tokens = num("max_tokens", None, int)
        if max_tokens is None:
            max_tokens = num("max_completion_tokens", self.default_max_tokens, int)
        if max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        return SamplingParams(temperature=num("temperature", 0.7, float), top_p=num("top_p", 1.0, float),
                              top_k=num("top_k", 0, int), seed=num("seed", 0, int),
                              max_new_tokens=min(max_tokens, 8192), ignore_eos=bool(body.get("ignore_eos", False)),
                              stop_on_consensus=False)

    def submit(self, prompt, body: Dict[str, Any], session: Optional[str], stream: bool = False) -> _Request:
        params = self.sampling(body)
        # the model's positions bound prompt + reply (the engine would fail the turn past them):
        # a prompt that alone reaches them is the client's error (OpenAI's 400
        # context_length_exceeded); otherwise the reply is cut to the room left (finish "length")
        limit = int(self.engine.cfg.max_pos)
        n = len(self.engine.encode_prompt(prompt))
        if n >= limit:
            raise ContextLengthError(f"This model's maximum context length is {limit} tokens, "
                                     f"but the prompt has {n} tokens.")
        if n + params.max_new_tokens > limit:
            params = SamplingParams(**{**params.__dict__, "max_new_tokens": limit - n})
        key = f"session:{session}" if session else f"anon:{next(self._anon)}"
        stops = parse_stops(body.get("stop"))
        return self.sched.submit(_Request(key, prompt, params, persistent=bool(session),
                                          stream_q=queue.Queue() if stream else None, stops=stops))

    def visible_text(self, ids: List[int], params: SamplingParams, stops=()) -> str:
        """The text of ``ids`` so far as the final result will show it (cut at max_new_tokens and at
        a stop id, decoded, cut at a stop string), minus a trailing incomplete UTF-8 character (a
        byte-level BPE token can end mid-character) and minus a tail that may still become a stop
        string: both are held back until the next piece decides."""
        gen = ids[:params.max_new_tokens]
        if not params.ignore_eos:
            gen = cut_at_stop(gen, self.engine.tokenizer.stop_ids)
        text = self.engine.tokenizer.decode(gen).rstrip("\ufffd")
        if stops:
            text, hit = cut_at_stop_strings(text, stops)
            if not hit:
                text = text[:len(text) - stop_prefix_hold(text, stops)]
        return text

    def generate(self, prompt: str, body: Dict[str, Any], session: Optional[str]) -> Tuple[Any, _Request]:
        r = self.submit(prompt, body, session)
        if not r.done.wait(self.sched.timeout_s + 30):
            raise TimeoutError("generation timed out")
        if r.error is not None:
            raise RuntimeError(str(r.error))
        return r.result, r

    @staticmethod
    def finish(out, r: _Request) -> str:
        if out.metrics.get("stop_string"):
            return "stop"
        return "length" if len(out.ids) >= r.params.max_new_tokens else "stop"

    @staticmethod
    def usage(out) -> Dict[str, int]:
        p = int(out.metrics.get("prompt_tokens", 0))
        return {"prompt_tokens": p, "completion_tokens": len(out.ids), "total_tokens": p + len(out.ids)}

    def show(self) -> Dict[str, Any]:
        cfg = self.engine.cfg
        arch = "llama" if cfg.arch == "llama" else cfg.arch
        return {"modelfile": "", "details": {"family": arch, "parameter_size": cfg.name},
                "model_info": {f"{arch}.context_length": int(min(cfg.max_pos, self.engine.kv_capacity_tokens)),
                               f"{arch}.embedding_length": cfg.hidden, f"{arch}.block_count": cfg.n_layers}}

    def metrics_text(self) -> str:
        st = dict(self.sched.stats)
        e = self.engine.stats
        lines = [
            "# TYPE roundtable_requests_total counter", f"roundtable_requests_total {st['requests']}",
            "# TYPE roundtable_request_errors_total counter", f"roundtable_request_errors_total {st['errors']}",
            "# TYPE roundtable_batches_total counter", f"roundtable_batches_total {st['batches']}",
            "# TYPE roundtable_prompt_tokens_total counter", f"roundtable_prompt_tokens_total {st['prompt_tokens']}",
            "# TYPE roundtable_completion_tokens_total counter",
            f"roundtable_completion_tokens_total {st['completion_tokens']}",
            "# TYPE roundtable_reused_kv_tokens_total counter", f"roundtable_reused_kv_tokens_total {st['reused_tokens']}",
            "# TYPE roundtable_engine_busy_seconds_total counter", f"roundtable_engine_busy_seconds_total {st['busy_s']:.6f}",
            "# TYPE roundtable_decode_steps_total counter", f"roundtable_decode_steps_total {st['decode_steps']}",
            "# TYPE roundtable_decode_rows_total counter", f"roundtable_decode_rows_total {st['decode_rows']}",
            "# TYPE roundtable_decode_tokens_total counter", f"roundtable_decode_tokens_total {e['decode_tokens']}",
            "# TYPE roundtable_kv_capacity_tokens gauge", f"roundtable_kv_capacity_tokens {self.engine.kv_capacity_tokens}",
            "# TYPE roundtable_engine_healthy gauge", f"roundtable_engine_healthy {int(bool(self.engine.healthy))}",
        ]
        return "\n".join(lines) + "\n"

    # ---- lifecycle ----------------------------------------------------------------------------
    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def start(self) -> "RoundtableServer":
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="roundtable-http", daemon=True)
        self._thread.start()
        return self

    def serve_forever(self) -> None:
        self.httpd.serve_forever()

    def close(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
        self.sched.close()
        if isinstance(self.engine, MirroredEngine):
            self.engine.stop_followers()


def build_server(model: str, weights: str = "random:0", device: str = "cuda:0", dtype: str = "bf16",
                 host: str = "127.0.0.1", port: int = 8000, max_batch: int = 16, max_tokens: int = 512,
                 use_graphs: bool = True, num_blocks: Optional[int] = None,
                 tp: int = 1, op_limit_s: float = 660.0) -> Optional[RoundtableServer]:
    """The server (rank 0), or — on a follower rank of a ``tp > 1`` launch — None after that
    rank has served rank 0's operations until shutdown."""
    # a checkpoint directory defines the architecture: preset + shape overrides from config.json
    from .utils.local_detect import resolve_model
    model, overrides = resolve_model(model, weights)
    cluster, tpi = None, None
    if tp > 1:
        import torch.distributed as dist
        from .parallel.cluster import init_cluster
        from .parallel.tp import TPInfo
        # containment: collectives fail after the request timeout + a minute, and
        # every engine operation runs under a stage limit (a stalled rank ends the server with a
        # message naming it, utils/failsafe.py); idle waits for the next request use the
        # cluster's long-timeout wait group
        cluster = init_cluster(prefer_gpu=device != "cpu", timeout_s=int(op_limit_s + 60))
        if cluster.world != tp:
            raise ValueError(f"serve --tp {tp} needs {tp} ranks, {cluster.world} joined")
        failsafe.RunGuard(cluster.rank, cluster.world,
                          lambda rec: sys.stderr.write(failsafe.describe(rec, "roundtable serve") + "\n"),
                          default_s=float("inf"), exit_code=2,
                          limits={"engine_load": 900.0, "k9_create": 900.0, "capture": op_limit_s}).start()
        # the engine meets on the load-timeout group after loading (a slower follower is waited for)
        tpi = TPInfo(size=tp, rank=cluster.rank, group=dist.group.WORLD, load_group=cluster.load_group)
        if device != "cpu":
            device = cluster.device
    ecfg = EngineConfig(model=model, weights=weights, device=device, dtype=dtype, use_graphs=use_graphs,
                        max_batch=max_batch, num_blocks=num_blocks, model_overrides=overrides)
    if ecfg.device == "cpu":
        ecfg.dtype = "fp32" if dtype == "bf16" else dtype
        ecfg.use_graphs = False
    if tpi is not None:
        with failsafe.stage("engine_load"):
            engine = Engine(ecfg, tpi)
        if cluster.rank != 0:
            serve_follower(engine, cluster, op_limit_s)
            return None
        return RoundtableServer(MirroredEngine(engine, cluster, op_limit_s), model, host, port, max_batch, max_tokens)
    return RoundtableServer(Engine(ecfg), model, host, port, max_batch, max_tokens)
