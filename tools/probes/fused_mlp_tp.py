"""Probe: the decode MLP of a tensor-parallel shard as ONE persistent launch
(tools/experiments/fused_mlp.hip: gate_up split-K over all CUs, a device-scope hand-off, down over
all CUs) against the product's two launches (split-K gate_up + SwiGLU, then down + residual), at
the Llama-3-8B tp 4 / tp 8 (and tp 2) shard shapes, M = 3 rows.

Timing: each path captured as a hipGraph of CALLS back-to-back MLPs over rotating weight copies
(> 256 MB, so the MALL cannot serve repeats), min over passes. Numerics: both paths against the
fp32 oracle (RMSNorm -> gate_up -> SwiGLU -> bf16 g -> down + residual in fp32), and the fused path twice on the same input (bit-equal:
deterministic). Needs ``python tools/experiments/build_exp.py``.

    python tools/probes/fused_mlp_tp.py [--tp 2,4,8] [--calls 40]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "experiments"))

import torch  # noqa: E402

from theroundtaible_amd import ops  # noqa: E402

DEV = "cuda"


def timed(fn, reps=5, tag=""):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
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
        best = min(best, a.elapsed_time(b) * 1e3)
    print(f"  timed {tag}: {best:.1f} us per graph", flush=True)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", default="2,4,8")
    ap.add_argument("--calls", type=int, default=40)
    a = ap.parse_args()
    from build_exp import load
    exp = load()
    H, F, M, eps = 4096, 14336, 3, 1e-5
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    grid = exp.decode_layer_grid()
    out = {"rows": []}
    torch.manual_seed(0)
    for tp in (int(t) for t in a.tp.split(",")):
        I = F // tp
        T = I // 16
        S = max(1, ops.native().splitk_parts(T, H // 32, cus, ops.SPLIT_WS_INTS))
        per = (2 * I * H + H * I) * 2
        copies = max(2, math.ceil(2 ** 30 / per))
        gamma = (1.0 + 0.1 * torch.randn(H)).to(torch.bfloat16).to(DEV)
        Wg = [(torch.randn(2 * I, H, device=DEV) * H ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        Wd = [(torch.randn(H, I, device=DEV) * I ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        Wgs = [ops.shuffle_weight(w, gamma, swiglu=True) for w in Wg]
        Wds = [ops.shuffle_weight(w) for w in Wd]
        x0 = torch.randn(M, H, device=DEV).to(torch.bfloat16)
        res = x0.clone()
        g = torch.empty(M, I, dtype=torch.bfloat16, device=DEV)
        sw = ops.split_workspace(DEV)
        sync = torch.zeros(576, dtype=torch.int32, device=DEV)   # legacy words 0-1, sharded words (fused_mlp.hip)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        sk = dict(split_ws=sw, split_mode=ops.SPLIT_K)

        def two_launches(i):
            gg = ops.skinny_gemm(res, Wgs[i], ops.PRO_NORM, ops.EPI_SWIGLU, eps=eps, **sk)
            ops.skinny_gemm(gg, Wds[i], ops.PRO_PLAIN, ops.EPI_RESID, res=res, **sk)

        def fused(i, phases=3):
            exp.fused_mlp(res, g, Wgs[i], Wds[i], sw, S, sync, err, eps, grid, phases)

        def gate_up_only(i):
            ops.skinny_gemm(res, Wgs[i], ops.PRO_NORM, ops.EPI_SWIGLU, eps=eps, **sk)

        def down_only(i):
            ops.skinny_gemm(g, Wds[i], ops.PRO_PLAIN, ops.EPI_RESID, res=res, **sk)

        # numerics on copy 0: both paths vs the fp32 oracle, fused twice bit-equal
        xr = x0.float()
        nrm = xr * torch.rsqrt((xr * xr).mean(-1, keepdim=True) + eps) * gamma.float()
        gu = nrm @ Wg[0].float().t()
        gref = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
        rref = xr + gref.to(torch.bfloat16).float() @ Wd[0].float().t()
        res.copy_(x0)
        two_launches(0)
        r_two = res.clone()
        res.copy_(x0)
        fused(0)
        r_f1 = res.clone()
        res.copy_(x0)
        fused(0)
        r_f2 = res.clone()
        torch.cuda.synchronize()
        e_two = (r_two.float() - rref).abs().max().item()
        e_f = (r_f1.float() - rref).abs().max().item()
        row = {"tp": tp, "I": I, "gate_up_tiles": T, "split_parts": S, "grid": grid,
               "err_two_vs_fp32": round(e_two, 4), "err_fused_vs_fp32": round(e_f, 4),
               "fused_deterministic": bool(torch.equal(r_f1, r_f2)), "fused_equals_two": bool(torch.equal(r_f1, r_two)),
               "poll_expired": int(err.item())}
        t2 = timed(lambda: [two_launches(i % copies) for i in range(a.calls)]) / a.calls
        tf = timed(lambda: [fused(i % copies) for i in range(a.calls)]) / a.calls
        # the phases apart: each product launch alone, each persistent phase alone (same launch)
        tgu = timed(lambda: [gate_up_only(i % copies) for i in range(a.calls)]) / a.calls
        tdn = timed(lambda: [down_only(i % copies) for i in range(a.calls)]) / a.calls
        tf1 = timed(lambda: [fused(i % copies, 1) for i in range(a.calls)]) / a.calls
        tf2 = timed(lambda: [fused(i % copies, 2) for i in range(a.calls)]) / a.calls
        tf5 = timed(lambda: [fused(i % copies, 5) for i in range(a.calls)]) / a.calls   # phase 1, plain stores
        # round 6: the synchronisation apart — no in-launch sync at all (timing only),
        # and the hand-off + exit re-arm on 8 sharded counters
        tf9 = timed(lambda: [fused(i % copies, 9) for i in range(a.calls)]) / a.calls     # phase 1, no sync
        tf10 = timed(lambda: [fused(i % copies, 10) for i in range(a.calls)]) / a.calls   # phase 2, no sync
        tf11 = timed(lambda: [fused(i % copies, 11) for i in range(a.calls)]) / a.calls   # both, no sync (wrong g)
        tf17 = timed(lambda: [fused(i % copies, 17) for i in range(a.calls)]) / a.calls   # phase 1, sharded
        tf18 = timed(lambda: [fused(i % copies, 18) for i in range(a.calls)]) / a.calls   # phase 2, sharded
        tf19 = timed(lambda: [fused(i % copies, 19) for i in range(a.calls)]) / a.calls   # both, sharded
        res.copy_(x0)
        fused(0, 19)
        r_sh = res.clone()
        torch.cuda.synchronize()
        row.update(fused_phase1_nosync_us=round(tf9, 2), fused_phase2_nosync_us=round(tf10, 2),
                   fused_nosync_us=round(tf11, 2), fused_phase1_sharded_us=round(tf17, 2),
                   fused_phase2_sharded_us=round(tf18, 2), fused_sharded_us=round(tf19, 2),
                   sharded_saving_us=round(t2 - tf19, 2), sharded_equals_fused=bool(torch.equal(r_sh, r_f1)))
        row.update(two_launch_us=round(t2, 2), fused_us=round(tf, 2), saving_us=round(t2 - tf, 2),
                   gate_up_launch_us=round(tgu, 2), down_launch_us=round(tdn, 2),
                   fused_phase1_only_us=round(tf1, 2), fused_phase2_only_us=round(tf2, 2),
                   fused_phase1_plain_stores_us=round(tf5, 2),
                   mlp_bytes_mb=round(per / 1e6, 1), poll_expired_after=int(err.item()))
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
        del Wg, Wd, Wgs, Wds
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
