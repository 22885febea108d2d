#!/usr/bin/env python3
"""Load test of ``roundtable serve`` (OpenAI dialect) on one GPU: aggregate completion tokens/s
and request latency under N concurrent clients (continuous batching, hipGraph decode).

    python tools/serve_bench.py [--model llama3-8b] [--clients 16] [--requests 32] [--prompt-words 400]
                                [--max-tokens 256] [--max-batch 16]

Synthetic prompts, random-init weights, ``ignore_eos`` so every request generates exactly
``--max-tokens``. Prints one JSON line. Every request is accounted for: a failed one is counted
(``failed_requests``, first errors in ``errors``), its client thread goes on with the next, and
the tool exits non-zero when any failed (round 5's version let a failed client thread die and
computed tok/s over the survivors). ``--stream``: requests stream (SSE) and the JSON adds
time-to-first-content-chunk percentiles and its share of the request latency.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import threading
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WORDS = ("ridder tafel consensus voorstel kernel geheugen rooster latency bandbreedte wachtrij graaf "
         "decoder prefill cache blok splitsing rangorde beslissing koning ronde").split()


def post(url, body, timeout=900):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read().decode())


def post_stream(url, body, timeout=900):
    """Stream a chat completion: (seconds to the first content chunk, content chunks, the usage the
    server reports with ``stream_options.include_usage``)."""
    req = urllib.request.Request(url, data=json.dumps(dict(body, stream=True, stream_options={"include_usage": True}))
                                 .encode(), method="POST", headers={"Content-Type": "application/json"})
    t0 = time.perf_counter()
    ttfc, n_chunks, done, usage = None, 0, False, None
    with urllib.request.urlopen(req, timeout=timeout) as r:
        for raw in r:
            line = raw.decode().strip()
            if not line.startswith("data: "):
                continue
            if line == "data: [DONE]":
                done = True
                continue
            ev = json.loads(line[6:])
            if "error" in ev:
                raise RuntimeError(ev["error"].get("message"))
            usage = ev.get("usage") or usage
            if ev["choices"][0]["delta"].get("content"):
                n_chunks += 1
                if ttfc is None:
                    ttfc = time.perf_counter() - t0
    if not done:
        raise RuntimeError("stream ended without [DONE]")
    return ttfc, n_chunks, usage


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--requests", type=int, default=32)
    ap.add_argument("--prompt-words", type=int, default=400)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--max-batch", type=int, default=16)
    ap.add_argument("--num-blocks", type=int, default=None)
    ap.add_argument("--stream", action="store_true", help="stream every request (SSE); report time to first chunk")
    a = ap.parse_args()
    from theroundtaible_amd.serve import build_server
    t_load = time.perf_counter()
    srv = build_server(a.model, weights="random:0", device=a.device, port=0, max_batch=a.max_batch,
                       max_tokens=a.max_tokens, num_blocks=a.num_blocks).start()
    load_s = time.perf_counter() - t_load
    rng = random.Random(0)
    prompts = [" ".join(rng.choice(WORDS) for _ in range(a.prompt_words)) for _ in range(a.requests)]
    url = srv.url + "/v1/chat/completions"

    def one(i):
        body = {"model": a.model, "messages": [{"role": "user", "content": prompts[i]}],
                "max_tokens": a.max_tokens, "ignore_eos": True, "temperature": 0.7, "top_p": 0.95}
        t0 = time.perf_counter()
        if a.stream:
            ttfc, n_chunks, u = post_stream(url, body)
            return time.perf_counter() - t0, dict(u or {"completion_tokens": 0, "prompt_tokens": 0},
                                                  ttfc=ttfc, chunks=n_chunks)
        d = post(url, body)
        return time.perf_counter() - t0, d["usage"]

    # warm-up: compiles/captures the decode graphs of the batch buckets used below
    post(url, {"messages": [{"role": "user", "content": "warm"}], "max_tokens": 8, "ignore_eos": True})
    lat, usage, errors = [], [], []
    lock = threading.Lock()
    nxt = iter(range(a.requests))

    def client():
        while True:
            with lock:
                i = next(nxt, None)
            if i is None:
                return
            try:
                dt, u = one(i)
            except Exception as e:  # noqa: BLE001 - counted, and this client goes on
                with lock:
                    errors.append(f"request {i}: {type(e).__name__}: {e}")
                continue
            with lock:
                lat.append(dt)
                usage.append(dict(u, lat=dt))

    t0 = time.perf_counter()
    th = [threading.Thread(target=client) for _ in range(a.clients)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    comp = sum(u["completion_tokens"] for u in usage)
    prompt = sum(u["prompt_tokens"] for u in usage)
    lat.sort()
    q = lambda xs, f: round(xs[int(f * (len(xs) - 1))], 3) if xs else None  # noqa: E731
    out = {"metric": "serve aggregate completion tokens/s", "value": round(comp / wall, 1), "unit": "tokens/s",
           "model": a.model, "dtype": "bf16", "data": "synthetic prompts, random-init weights",
           "clients": a.clients, "requests": a.requests, "completed_requests": len(usage),
           "failed_requests": len(errors), "errors": errors[:5], "max_batch": a.max_batch,
           "max_tokens": a.max_tokens, "stream": a.stream,
           "prompt_tokens_total": prompt, "completion_tokens_total": comp, "wall_s": round(wall, 2),
           "latency_s_p50": q(lat, 0.5), "latency_s_p99": q(lat, 0.99),
           "engine_load_s": round(load_s, 2), "scheduler": dict(srv.sched.stats) if hasattr(srv, "sched") else None}
    if a.stream and usage:
        tt = sorted(u["ttfc"] for u in usage if u["ttfc"] is not None)
        share = sorted(u["ttfc"] / u["lat"] for u in usage if u["ttfc"] is not None)
        out.update(ttfc_s_p50=q(tt, 0.5), ttfc_s_p99=q(tt, 0.99), ttfc_share_of_latency_p50=q(share, 0.5),
                   ttfc_share_of_latency_max=q(share, 1.0),
                   content_chunks_mean=round(sum(u["chunks"] for u in usage) / len(usage), 1))
    srv.close()
    print(json.dumps(out), flush=True)
    return 0 if not errors else 1


if __name__ == "__main__":
    sys.exit(main())
