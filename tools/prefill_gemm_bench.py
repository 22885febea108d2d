#!/usr/bin/env python3
"""Prefill GEMM backends on MI355X: time the Llama-3-8B prefill linears (M = tokens prefilled per
round, ~1.9K at the driver config) under each BLAS library torch can dispatch to on ROCm
(hipBLASLt = "cublaslt", rocBLAS = "cublas", composable_kernel = "ck").

Usage: python tools/prefill_gemm_bench.py [--m 1900,4096]
"""
import argparse

import torch


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1900,4096")
    a = ap.parse_args()
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    dev = "cuda"
    print("| backend | M | op | us | TF/s |\n|---|---|---|---|---|")
    for backend in ("cublaslt", "cublas", "ck"):
        try:
            torch.backends.cuda.preferred_blas_library(backend)
        except Exception as ex:  # noqa: BLE001
            print(f"| {backend} | - | unavailable: {type(ex).__name__} | | |")
            continue
        for M in (int(m) for m in a.m.split(",")):
            for name, (N, K) in shapes.items():
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
                try:
                    us = timed(lambda: torch.nn.functional.linear(x, w))
                except Exception as ex:  # noqa: BLE001
                    print(f"| {backend} | {M} | {name} | failed: {type(ex).__name__} | |")
                    continue
                print(f"| {backend} | {M} | {name} | {us:.1f} | {2 * M * N * K / us / 1e6:.0f} |", flush=True)
    torch.backends.cuda.preferred_blas_library("cublaslt")


if __name__ == "__main__":
    main()
