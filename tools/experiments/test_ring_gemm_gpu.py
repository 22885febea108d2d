"""EXPERIMENT (not adopted): the loader-wave LDS-ring GEMM (ring_gemm.hip) stays numerically
correct. Needs ``python tools/experiments/build_exp.py`` first."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from theroundtaible_amd import ops  # noqa: E402
from build_exp import load  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("variant", [0, 2, 4])
def test_ring_gemm_experiment_matches(variant):
    """The loader-wave LDS-ring GEMM experiment (tools/experiments/ring_gemm.hip) stays numerically correct."""
    M, N, K = 3, 512, 2048
    x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    for grid in (7, 32):        # several tiles per workgroup: ring reuse across tiles
        out.zero_()
        load().ring_gemm_exp(out, x, ops.shuffle_weight(W), grid, variant)
        want = x.float() @ W.float().t()
        assert torch.allclose(out.float(), want, atol=2e-2, rtol=2e-2)
