"""Probe: why the one-launch sampler costs ~26 µs per step inside the bench's
decode graph but ~18 µs in isolation on randn rows.

Takes REAL decode logits of the bench's model (Llama-3-8B, random-init ``random:1234`` weights,
3 sequences with a ~2K-token prompt, a few eager decode steps), and times ``ops.sample`` at the
bench's sampling parameters (temperature 0.7, top-p 0.95) on them against randn rows of the same
shape, each (a) L2-hot (the same rows every call) and (b) after a 512 MB copy that evicts them
(the step's situation: the lm_head wrote the logits from every XCD), as hipGraph replays. Also
prints each row's logit statistics and nucleus size (how many tokens carry 95 % of the mass).

    python tools/probes/sampler_real_logits.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.engine import Engine, EngineConfig  # noqa: E402
from theroundtaible_amd.models.llama import AttnMeta  # noqa: E402

DEV = "cuda"


def graph_us(fn, calls=20, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / calls)
    return best


def main():
    e = Engine(EngineConfig(model="llama3-8b", weights="random:1234", device=DEV, use_graphs=False,
                            max_kv_tokens=16384))
    m, kv = e.model, e.kv
    g = torch.Generator().manual_seed(1)
    seqs = [kv.seq(f"s{i}") for i in range(3)]
    for s in seqs:
        e.prefill([(s, torch.randint(0, 128000, (2000,), generator=g).tolist())])
    toks = torch.randint(0, 128000, (3,), generator=g).to(DEV)
    for step in range(4):      # a few eager decode steps (their last logits are the sample)
        for s in seqs:
            kv.ensure_capacity(s, s.length + 1)
        pos = torch.tensor([s.length for s in seqs], device=DEV)
        slots = torch.tensor([s.blocks[p // 32] * 32 + p % 32 for s, p in zip(seqs, pos.tolist())], device=DEV)
        bt = torch.zeros(3, max(len(s.blocks) for s in seqs), dtype=torch.int32)
        for j, s in enumerate(seqs):
            bt[j, :len(s.blocks)] = torch.tensor(s.blocks)
        ws = ops.DecodeWorkspace(3, m.n_heads, m.head_dim, 8, DEV)
        meta = AttnMeta("decode", slots, bt.to(DEV), (pos + 1).to(torch.int32), num_splits=8, workspace=ws)
        logits = m.forward(toks, pos, kv, meta)
        for s, t in zip(seqs, toks.tolist()):
            s.tokens.append(t)
        toks = logits.float().argmax(-1)
    real = logits.contiguous()
    V = real.shape[1]
    rnd = torch.randn(3, V, device=DEV).to(real.dtype)
    T, P = 0.7, 0.95
    temp = torch.full((3,), T, device=DEV)
    top_p = torch.full((3,), P, device=DEV)
    top_k = torch.zeros(3, dtype=torch.int32, device=DEV)
    seeds = torch.arange(3, device=DEV, dtype=torch.int64)
    offs = torch.zeros(3, device=DEV, dtype=torch.int64)
    out = torch.empty(3, dtype=torch.int64, device=DEV)
    sw = ops.sample_workspace(3, DEV)
    flush_src = torch.empty(256 << 20, dtype=torch.uint8, device=DEV)
    flush_dst = torch.empty_like(flush_src)
    rows = []
    for b in range(3):
        z = real[b].float() / T
        pr = torch.softmax(z, 0)
        srt = pr.sort(descending=True).values
        nuc = int((srt.cumsum(0) < P).sum()) + 1
        rows.append({"row": b, "logit_std": round(float(real[b].float().std()), 4),
                     "logit_max_minus_mean": round(float(real[b].float().max() - real[b].float().mean()), 3),
                     "nucleus_tokens_p95": nuc, "top_token_prob": round(float(srt[0]), 6)})
    res = {"dtype": str(real.dtype), "V": V, "rows": rows}
    flush_us = graph_us(lambda: flush_dst.copy_(flush_src))
    # the captured step's form: the same launch also records the token and advances positions /
    # lengths / step and writes the next slots, offsets and embedding rows (DecodeGraph._body)
    maxb = 512
    bt = torch.arange(3 * maxb, device=DEV, dtype=torch.int32).reshape(3, maxb)
    st_out = torch.zeros(8192, 3, dtype=torch.int64, device=DEV)
    ids = torch.zeros(3, dtype=torch.int64, device=DEV)
    pos0 = torch.full((3,), 2100, dtype=torch.int64, device=DEV)
    pos = pos0.clone()
    ctx = (pos0 + 1).to(torch.int32)
    stepc = torch.zeros(1, dtype=torch.int64, device=DEV)
    slots = torch.zeros(3, dtype=torch.int64, device=DEV)
    hid = torch.zeros(3, m.cfg.hidden, dtype=real.dtype, device=DEV)
    offs2 = (pos0 + 1).clone()
    sw2 = ops.sample_workspace(3, DEV)

    def adv(lg):
        pos.copy_(pos0)     # keep the step inside the table (a tiny copy kernel, timed apart below)
        ops.sample_advance(lg, temp, top_p, top_k, seeds, offs2, sw2, out, st_out, ids, pos, ctx, stepc, slots, hid,
                           bt, m.w["embed"], 32)

    copy_us = graph_us(lambda: pos.copy_(pos0))
    for name, lg in (("real", real), ("randn", rnd)):
        hot = graph_us(lambda lg=lg: ops.sample(lg, temp, top_p, top_k, seeds, offs, out, ws=sw))
        cold = graph_us(lambda lg=lg: (flush_dst.copy_(flush_src),
                                       ops.sample(lg, temp, top_p, top_k, seeds, offs, out, ws=sw))) - flush_us
        res[f"{name}_hot_us"] = round(hot, 2)
        res[f"{name}_after_flush_us"] = round(cold, 2)
        stepc.zero_()
        res[f"{name}_step_form_hot_us"] = round(graph_us(lambda lg=lg: adv(lg)) - copy_us, 2)
        stepc.zero_()
        res[f"{name}_step_form_after_flush_us"] = round(
            graph_us(lambda lg=lg: (flush_dst.copy_(flush_src), adv(lg))) - flush_us - copy_us, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
