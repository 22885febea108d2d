"""Probe: which branch of the one-launch top-p sampler decides a row, how
often, and what each branch costs, on REAL decode logits of the bench's model.

Logits: Llama-3-8B random-init (``random:1234``), 3 sequences with a ~2K-token prompt, a few
eager decode steps (as ``sampler_real_logits.py``), saved to ``--logits``. For OFFSETS RNG
offsets (the Gumbel draw of each step) at the bench's parameters (temperature 0.7, top-p 0.95):

* ``--mode paths`` (run with ``RT_SMP_PROBE=5``): the decided path of each row
  (csrc/sampling.hip PATH_*: 1 accept, 2 rejected -> histogram rescan, 3 -> candidates,
  4 -> full histogram path; +10 when the accept test needed its exact pass over the row);
* ``--mode times`` (``RT_SMP_PROBE`` unset): µs per 3-row launch at each offset (hipGraph of 20
  replays, L2-hot), grouped by the slowest row's path from the paths file.

    python tools/probes/sampler_paths.py --mode gen   --logits L.pt
    RT_SMP_PROBE=5 python tools/probes/sampler_paths.py --mode paths --logits L.pt --out P.json
    python tools/probes/sampler_paths.py --mode times --logits L.pt --paths P.json
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from theroundtaible_amd import ops  # noqa: E402

DEV = "cuda"
T, P = 0.7, 0.95


def gen(path):
    from theroundtaible_amd.engine import Engine, EngineConfig
    from theroundtaible_amd.models.llama import AttnMeta
    e = Engine(EngineConfig(model="llama3-8b", weights="random:1234", device=DEV, use_graphs=False,
                            max_kv_tokens=16384))
    m, kv = e.model, e.kv
    g = torch.Generator().manual_seed(1)
    seqs = [kv.seq(f"s{i}") for i in range(3)]
    for s in seqs:
        e.prefill([(s, torch.randint(0, 128000, (2000,), generator=g).tolist())])
    toks = torch.randint(0, 128000, (3,), generator=g).to(DEV)
    rows = []
    for _ in range(6):
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
        rows.append(logits.contiguous().cpu())
        for s, t in zip(seqs, toks.tolist()):
            s.tokens.append(t)
        toks = logits.float().argmax(-1)
    torch.save(torch.cat(rows[-2:]).contiguous(), path)     # 6 rows: the last two steps
    print(json.dumps({"saved": path, "rows": 6}), flush=True)


def setup(path):
    lg = torch.load(path, weights_only=True).to(DEV)
    B = 3
    par = dict(temperature=torch.full((B,), T, device=DEV), top_p=torch.full((B,), P, device=DEV),
               top_k=torch.zeros(B, dtype=torch.int32, device=DEV), seeds=torch.arange(B, device=DEV,
                                                                                     dtype=torch.int64))
    return lg, par


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["gen", "paths", "times"], required=True)
    ap.add_argument("--logits", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--paths", default=None)
    ap.add_argument("--offsets", type=int, default=400)
    a = ap.parse_args()
    if a.mode == "gen":
        gen(a.logits)
        return
    lg, par = setup(a.logits)
    out = torch.empty(3, dtype=torch.int64, device=DEV)
    res = []
    for half in (0, 1):                      # the two saved steps' 3-row batches
        rows = lg[3 * half:3 * half + 3].contiguous()
        sw = ops.sample_workspace(3, DEV)
        offs = torch.zeros(3, dtype=torch.int64, device=DEV)
        ops.sample(rows, par["temperature"], par["top_p"], par["top_k"], par["seeds"], offs, out, ws=sw)  # grid scale
        for o in range(a.offsets):
            offs.fill_(1000 + o)
            if a.mode == "paths":
                ops.sample(rows, par["temperature"], par["top_p"], par["top_k"], par["seeds"], offs, out, ws=sw)
                res.append(out.tolist())
            else:
                fn = lambda: ops.sample(rows, par["temperature"], par["top_p"], par["top_k"], par["seeds"], offs,  # noqa: E731
                                        out, ws=sw)
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    fn()
                torch.cuda.current_stream().wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(20):
                        fn()
                g.replay()
                torch.cuda.synchronize()
                best = float("inf")
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
                res.append(round(best, 2))
            if o % 100 == 0:
                print(json.dumps({"half": half, "offset": o}), flush=True)
    if a.mode == "paths":
        rows = collections.Counter(p for r in res for p in r)
        steps = collections.Counter(max(r, key=lambda p: (p % 10, p)) for r in res)
        summary = {"row_paths": dict(sorted(rows.items())), "slowest_row_path_per_step": dict(sorted(steps.items())),
                   "launches": len(res)}
        json.dump({"paths": res, "summary": summary}, open(a.out, "w"))
        print(json.dumps(summary), flush=True)
    else:
        paths = json.load(open(a.paths))["paths"]
        by = collections.defaultdict(list)
        for p3, us in zip(paths, res):
            by[str(sorted(p3))].append(us)
        table = {k: {"n": len(v), "mean_us": round(sum(v) / len(v), 2), "min_us": min(v), "max_us": max(v)}
                 for k, v in sorted(by.items(), key=lambda kv: -len(kv[1]))}
        summary = {"launches": len(res), "mean_us": round(sum(res) / len(res), 2), "by_row_paths": table}
        if a.out:
            json.dump(summary, open(a.out, "w"), indent=1)
        print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
