"""`roundtable serve` on a CPU engine: OpenAI + Ollama dialects, batching, session KV reuse."""
import json
import threading
import time
import urllib.error
import urllib.request

import pytest

from theroundtaible_amd.serve import build_server, render_chat


def _post(url, body):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=120) as r:
        return r.status, r.read().decode()


def _get(url):
    with urllib.request.urlopen(url, timeout=30) as r:
        return r.status, r.read().decode()


@pytest.fixture(scope="module")
def server():
    srv = build_server("tiny-llama", weights="random:1", device="cpu", port=0, max_batch=4, max_tokens=8,
                       num_blocks=256).start()
    yield srv
    srv.close()


def test_models_health_metrics(server):
    code, body = _get(server.url + "/v1/models")
    assert code == 200 and json.loads(body)["data"][0]["id"] == "tiny-llama"
    assert json.loads(_get(server.url + "/health")[1])["status"] == "ok"
    assert "roundtable_requests_total" in _get(server.url + "/metrics")[1]


def test_chat_completion_openai(server):
    code, body = _post(server.url + "/v1/chat/completions",
                       {"model": "tiny-llama", "messages": [{"role": "user", "content": "Hallo ridders"}],
                        "max_tokens": 6, "temperature": 0})
    d = json.loads(body)
    assert code == 200 and d["object"] == "chat.completion"
    assert d["choices"][0]["message"]["role"] == "assistant"
    assert d["usage"]["completion_tokens"] == 6 and d["choices"][0]["finish_reason"] == "length"


def test_stream_and_completions_and_ollama(server):
    code, body = _post(server.url + "/v1/chat/completions",
                       {"messages": [{"role": "user", "content": "x"}], "max_tokens": 3, "stream": True})
    assert code == 200 and body.rstrip().endswith("data: [DONE]")
    code, body = _post(server.url + "/v1/completions", {"prompt": "Onderwerp:", "max_tokens": 4})
    assert json.loads(body)["object"] == "text_completion"
    code, body = _post(server.url + "/api/chat", {"model": "tiny-llama", "messages": [{"role": "user", "content": "q"}],
                                                  "options": {"num_predict": 5}, "stream": False})
    d = json.loads(body)
    assert d["done"] is True and d["eval_count"] == 5
    ctx = json.loads(_post(server.url + "/api/show", {"name": "tiny-llama"})[1])["model_info"]
    assert any(k.endswith(".context_length") for k in ctx)


def test_greedy_is_deterministic_and_session_reuses_kv(server):
    body = {"messages": [{"role": "user", "content": "Wat is het plan?"}], "max_tokens": 5, "temperature": 0}
    a = json.loads(_post(server.url + "/v1/chat/completions", body)[1])["choices"][0]["message"]["content"]
    b = json.loads(_post(server.url + "/v1/chat/completions", body)[1])["choices"][0]["message"]["content"]
    assert a == b
    conv = [{"role": "user", "content": "Eerste vraag over caching."}]
    s1 = dict(body, messages=conv, user="knight-7")
    r1 = json.loads(_post(server.url + "/v1/chat/completions", s1)[1])
    conv2 = conv + [{"role": "assistant", "content": r1["choices"][0]["message"]["content"]},
                    {"role": "user", "content": "En nu?"}]
    before = server.sched.stats["reused_tokens"]
    _post(server.url + "/v1/chat/completions", dict(body, messages=conv2, user="knight-7"))
    assert server.sched.stats["reused_tokens"] - before > 10   # the first exchange stayed resident


def test_session_with_system_message_keeps_conversation_kv(server):
    """with a system message (shared system-prompt prefix, on by default) the session's
    next turn must still reuse the whole first exchange — attaching the shared system blocks may
    not truncate a conversation that already holds them."""
    body = {"max_tokens": 5, "temperature": 0, "user": "knight-sys"}
    sys_msg = {"role": "system", "content": "Je bent een ridder van de ronde tafel. " * 12}
    conv = [sys_msg, {"role": "user", "content": "Eerste vraag over de gedeelde systeemprompt."}]
    r1 = json.loads(_post(server.url + "/v1/chat/completions", dict(body, messages=conv))[1])
    conv2 = conv + [{"role": "assistant", "content": r1["choices"][0]["message"]["content"]},
                    {"role": "user", "content": "En de tweede?"}]
    prompt1 = r1["usage"]["prompt_tokens"]
    before = server.sched.stats["reused_tokens"]
    _post(server.url + "/v1/chat/completions", dict(body, messages=conv2))
    # the first request's prompt (system + first question) was reused, not just the system blocks
    assert server.sched.stats["reused_tokens"] - before >= prompt1 - 1


def test_concurrent_requests_are_batched(server):
    results, errs = [], []

    def go(i):
        try:
            results.append(_post(server.url + "/v1/chat/completions",
                                 {"messages": [{"role": "user", "content": f"vraag {i}"}], "max_tokens": 4})[0])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    b0 = server.sched.stats["batches"]
    ts = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and results == [200] * 6
    assert server.sched.stats["batches"] - b0 < 6   # at least two requests shared a batch


def test_bad_requests(server):
    import urllib.error
    with pytest.raises(urllib.error.HTTPError) as ei:
        _post(server.url + "/v1/chat/completions", {"messages": []})
    assert ei.value.code == 400


def test_render_chat():
    s = render_chat([{"role": "system", "content": "S"}, {"role": "user", "content": [{"type": "text", "text": "U"}]}])
    assert s.endswith("### Assistent:\n") and "### Systeem:\nS" in s and "### Gebruiker:\nU" in s


def test_continuous_batching_admits_midflight(server):
    """A short request that arrives while a long generation runs joins the running batch at
    the next chunk boundary and finishes first."""
    done = {}

    def go(name, n, delay):
        time.sleep(delay)
        _post(server.url + "/v1/chat/completions",
              {"messages": [{"role": "user", "content": name}], "max_tokens": n, "temperature": 0})
        done[name] = time.perf_counter()
    before = server.sched.stats["admitted_midflight"]
    server.sched.chunk = 4
    ts = [threading.Thread(target=go, args=("lang", 160, 0.0)), threading.Thread(target=go, args=("kort", 4, 0.15))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert server.sched.stats["admitted_midflight"] > before
    assert done["kort"] < done["lang"]


def test_shared_system_prompt_kv(server):
    """Clients sending the same system prompt share one resident copy of its KV: the shared
    sequence holds it, each request's sequence references its full blocks, and greedy answers
    equal those of a server that does not share."""
    sys_prompt = "Je bent een knight van de ronde tafel. " * 30
    body = lambda u: {"messages": [{"role": "system", "content": sys_prompt}, {"role": "user", "content": u}],
                      "max_tokens": 6, "temperature": 0, "user": f"deel-{u}"}
    outs = [json.loads(_post(server.url + "/v1/chat/completions", body(u))[1]) for u in ("een", "twee")]
    e = server.engine
    shared = [e.kv.seqs[k] for k in e.kv.seqs if k.startswith("@shared:sys:")]
    assert shared, "no shared system-prompt sequence"
    first = e.kv.seqs["session:deel-een"].blocks[:1]
    sq = next(q for q in shared if q.blocks[:1] == first)    # (other tests' system prompts live too)
    full = sq.length // e.kv.block_size
    assert full >= 2
    for u in ("een", "twee"):
        s = e.kv.seqs[f"session:deel-{u}"]
        assert s.blocks[:full] == sq.blocks[:full]
    plain = build_server("tiny-llama", weights="random:1", device="cpu", port=0, max_batch=4, max_tokens=8,
                         num_blocks=256)
    plain.share_system_prompts = False
    plain.start()
    try:
        ref = [json.loads(_post(plain.url + "/v1/chat/completions", body(u))[1]) for u in ("een", "twee")]
    finally:
        plain.close()
    assert [o["choices"][0]["message"]["content"] for o in outs] == \
        [o["choices"][0]["message"]["content"] for o in ref]


def test_shared_system_prompt_concurrent_batch(server):
    sys_prompt = "Gedeelde systeemprompt voor iedereen. " * 25
    res, errs = [], []

    def go(i):
        try:
            res.append(_post(server.url + "/v1/chat/completions",
                             {"messages": [{"role": "system", "content": sys_prompt},
                                           {"role": "user", "content": f"vraag {i}"}], "max_tokens": 5})[0])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=go, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and res == [200] * 4


def _stream_events(url, body):
    """POST with stream=true; (list of parsed SSE data objects, arrival times relative to the POST)."""
    req = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    t0 = time.perf_counter()
    events, times = [], []
    with urllib.request.urlopen(req, timeout=120) as r:
        assert r.status == 200 and r.headers["Content-Type"].startswith("text/event-stream")
        for raw in r:
            line = raw.decode().strip()
            if not line.startswith("data: "):
                continue
            payload = line[len("data: "):]
            events.append(payload if payload == "[DONE]" else json.loads(payload))
            times.append(time.perf_counter() - t0)
    return events, times


def test_streaming_emits_chunks_during_decode(server):
    """a 64-token completion streams >= 2 content chunks before [DONE] (one per
    host readback of the decode loop), and the chunks concatenate to the non-streamed text (greedy)."""
    body = {"messages": [{"role": "user", "content": "Vertel over de ronde tafel"}], "max_tokens": 64,
            "temperature": 0, "ignore_eos": True}
    want = json.loads(_post(server.url + "/v1/chat/completions", body)[1])["choices"][0]["message"]["content"]
    events, times = _stream_events(server.url + "/v1/chat/completions", dict(body, stream=True))
    assert events[-1] == "[DONE]"
    content = [e["choices"][0]["delta"].get("content", "") for e in events[:-1]]
    pieces = [c for c in content if c]
    assert len(pieces) >= 2, content
    assert "".join(pieces) == want
    assert events[0]["choices"][0]["delta"]["role"] == "assistant"
    assert events[-2]["choices"][0]["finish_reason"] == "length"
    assert "usage" not in events[-2]
    ev_u, _ = _stream_events(server.url + "/v1/chat/completions",
                             dict(body, stream=True, stream_options={"include_usage": True}))
    assert ev_u[-2]["usage"]["completion_tokens"] == 64
    # the text arrives while decoding: the first content chunk well before the end of the stream
    first = next(i for i, c in enumerate(content) if c)
    assert times[first] < times[-1]
    # the completions endpoint and Ollama NDJSON stream the same way
    cb = {"prompt": "Onderwerp:", "max_tokens": 40, "temperature": 0, "ignore_eos": True}
    want_c = json.loads(_post(server.url + "/v1/completions", cb)[1])["choices"][0]["text"]
    ev_c, _ = _stream_events(server.url + "/v1/completions", dict(cb, stream=True))
    assert "".join(e["choices"][0]["text"] for e in ev_c[:-1]) == want_c
    ob = {"messages": [{"role": "user", "content": "q"}], "options": {"num_predict": 40, "temperature": 0}}
    want_o = json.loads(_post(server.url + "/api/chat", dict(ob, stream=False))[1])["message"]["content"]
    req = urllib.request.Request(server.url + "/api/chat", data=json.dumps(dict(ob, stream=True)).encode(),
                                 method="POST", headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=120) as r:
        lines = [json.loads(l) for l in r.read().decode().splitlines() if l.strip()]
    assert lines[-1]["done"] is True and all(not l["done"] for l in lines[:-1]) and len(lines) >= 3
    assert "".join(l["message"]["content"] for l in lines) == want_o


def test_sixty_four_concurrent_clients_all_served(server):
    """a burst of 64 clients connecting at once must get 64 x HTTP 200 (the
    listen backlog was socketserver's 5; an overflow is reset by the kernel)."""
    n = 64
    codes, errs = [], []
    bar = threading.Barrier(n)
    lock = threading.Lock()

    def go(i):
        bar.wait()
        try:
            c = _post(server.url + "/v1/completions", {"prompt": f"vraag {i}", "max_tokens": 2})[0]
            with lock:
                codes.append(c)
        except Exception as e:  # noqa: BLE001
            with lock:
                errs.append(repr(e))
    ts = [threading.Thread(target=go, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and codes == [200] * n, (errs[:3], len(codes))
    assert server.httpd.request_queue_size >= 128


def test_stream_client_disconnect_cancels_the_request(server):
    """A streaming client that goes away mid-stream must not keep the engine decoding for nobody:
    the request is cancelled at the next decode chunk and releases its KV."""
    import http.client
    from urllib.parse import urlparse
    u = urlparse(server.url)
    before = dict(server.sched.stats)
    conn = http.client.HTTPConnection(u.hostname, u.port, timeout=60)
    body = {"prompt": "Een lange monoloog:", "max_tokens": 3000, "ignore_eos": True, "temperature": 0, "stream": True}
    conn.request("POST", "/v1/completions", body=json.dumps(body), headers={"Content-Type": "application/json"})
    resp = conn.getresponse()
    assert resp.status == 200
    line = b""
    while not line.startswith(b"data: {"):
        line = resp.fp.readline()
    conn.sock.shutdown(2)          # the client disappears
    conn.close()
    deadline = time.time() + 120
    while server.sched.stats["requests"] == before["requests"] and time.time() < deadline:
        time.sleep(0.2)
    assert server.sched.stats["requests"] == before["requests"] + 1
    got = server.sched.stats["completion_tokens"] - before["completion_tokens"]
    assert got < 3000, got


def test_stop_strings_cut_the_reply(server):
    """OpenAI ``stop`` (string or list) / Ollama ``options.stop``: the reply ends before the earliest
    stop string, finish_reason "stop", decoding ends at the next chunk; streamed pieces never show
    a stop string and concatenate to the same text."""
    from theroundtaible_amd.serve import cut_at_stop_strings, stop_prefix_hold
    assert cut_at_stop_strings("abc STOP def", ["STOP", "de"]) == ("abc ", True)
    assert cut_at_stop_strings("abc", ["x"]) == ("abc", False)
    assert stop_prefix_hold("hello ST", ["STOP"]) == 2 and stop_prefix_hold("hello", ["STOP"]) == 0
    body = {"prompt": "Stop-test:", "max_tokens": 48, "temperature": 0, "ignore_eos": True}
    full = json.loads(_post(server.url + "/v1/completions", body)[1])["choices"][0]["text"]
    assert len(full) > 20
    stop = full[len(full) // 2:len(full) // 2 + 3]
    want = full[:full.find(stop)]
    d = json.loads(_post(server.url + "/v1/completions", dict(body, stop=[stop]))[1])
    assert d["choices"][0]["text"] == want and d["choices"][0]["finish_reason"] == "stop"
    d = json.loads(_post(server.url + "/v1/completions", dict(body, stop=stop))[1])
    assert d["choices"][0]["text"] == want
    events, _ = _stream_events(server.url + "/v1/completions", dict(body, stop=[stop], stream=True))
    pieces = [e["choices"][0]["text"] for e in events[:-1]]
    assert "".join(pieces) == want and all(stop not in p for p in pieces)
    assert events[-2]["choices"][0]["finish_reason"] == "stop"
    code, msg = 0, ""
    try:
        _post(server.url + "/v1/completions", dict(body, stop=[1, 2]))
    except urllib.error.HTTPError as e:
        code = e.code
    assert code == 400


def test_context_length_exceeded_and_reply_clamped(server):
    """A prompt past the model's positions (tiny-llama: 4096) is the client's error — HTTP 400 with
    OpenAI's code, streamed or not; a prompt that fits gets its reply cut to the room left."""
    long = "woord " * 6000
    for stream in (False, True):
        with pytest.raises(urllib.error.HTTPError) as ei:
            _post(server.url + "/v1/chat/completions",
                  {"messages": [{"role": "user", "content": long}], "max_tokens": 4, "stream": stream})
        assert ei.value.code == 400
        err = json.loads(ei.value.read().decode())["error"]
        assert err["code"] == "context_length_exceeded" and "4096" in err["message"]
    eng = server.engine
    lo, hi = 1, 6000                         # the longest prompt of repeated words below the limit
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if len(eng.encode_prompt("woord " * mid)) < 4096:
            lo = mid
        else:
            hi = mid - 1
    words = lo
    n = len(eng.encode_prompt("woord " * words))
    assert 4096 - 50 < n < 4096
    code, body = _post(server.url + "/v1/completions", {"prompt": "woord " * words, "max_tokens": 50,
                                                       "temperature": 0})
    d = json.loads(body)
    assert code == 200 and d["usage"]["completion_tokens"] == 4096 - n
