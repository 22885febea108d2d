"""Probe: are hipBLASLt GEMMs of the prefill's shapes correct in a process whose queues carry a CU
mask (ROC_GLOBAL_CU_MASK)? Prints max error vs an fp32 matmul per shape.
    ROC_GLOBAL_CU_MASK=0xffffffffffffffffffffffffffffffff python tools/probes/cu_mask_gemm.py"""
import json
import os

import torch

torch.manual_seed(0)
rows = []
for M, N, K in [(1417, 28672, 4096), (1417, 4096, 14336), (1417, 6144, 4096), (1417, 4096, 4096), (64, 4096, 4096)]:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    got = (a @ b.t()).float()
    rows.append({"M": M, "N": N, "K": K, "max_rel_err": round(float((got - ref).abs().max() / ref.abs().max()), 5)})
print(json.dumps({"mask": os.environ.get("ROC_GLOBAL_CU_MASK"), "rows": rows}))
