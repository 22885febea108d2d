"""Probe: hipBLASLt bf16 GEMM time vs the row count M for the Llama-3-8B prefill shapes (does
padding M to a tile multiple pay?). Prints one JSON line per (shape, M)."""
import json

import torch

DEV = "cuda"
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
torch.manual_seed(0)
for name, (N, K) in shapes.items():
    W = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    for M in (1417, 1440, 1472, 1536, 1664, 2048):
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        for _ in range(3):
            torch.nn.functional.linear(x, W)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                torch.nn.functional.linear(x, W)
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b) * 1e3 / 10)
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "us": round(best, 1),
                          "pflops": round(2 * M * N * K / best / 1e9, 3)}), flush=True)
