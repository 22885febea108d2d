#!/usr/bin/env python3
"""EXPERIMENT: loader-wave LDS-ring decode GEMM (csrc/ring_gemm.hip) vs the register-streaming
skinny GEMM, M = 3, Llama-3-8B shapes, cold weights (>= 1 GiB rotation). Correctness first."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from theroundtaible_amd import ops  # noqa: E402
from tools.microbench import bf, timed  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nat = ops.native()
    torch.manual_seed(0)
    for name, N, K in [("o", 4096, 4096), ("down", 4096, 14336), ("gate_up (plain)", 28672, 4096),
                       ("lm_head", 128256, 4096)]:
        x = bf(M, K)
        W = bf(N, K, scale=0.02)
        Ws = ops.shuffle_weight(W)
        want = (x.float() @ W.float().t())
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        for grid, var in ((256, 0), (512, 3)):
            out.zero_()
            nat.ring_gemm_exp(out, x, Ws, grid, var)
            torch.cuda.synchronize()
            err = (out.float() - want).abs().max().item()
            assert err < 0.05 * want.abs().max().item() + 1e-2, (name, grid, err)
        copies = max(2, math.ceil(2**30 / (N * K * 2)))
        Wc = [ops.shuffle_weight(bf(N, K, scale=0.02)) for _ in range(copies)]
        nbytes = N * K * 2
        us = timed(lambda i: ops.skinny_gemm(x, Wc[i % copies], ops.PRO_PLAIN, ops.EPI_STORE))
        print(f"{name:16s} skinny          {us:8.2f} us {nbytes / us / 1e6:6.2f} TB/s", flush=True)
        for var in range(6):
            for grid in (256,):
                us = timed(lambda i, g=grid, v=var: nat.ring_gemm_exp(out, x, Wc[i % copies], g, v))
                print(f"{name:16s} ring v{var} grid={grid:4d} {us:8.2f} us {nbytes / us / 1e6:6.2f} TB/s", flush=True)
        del Wc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
