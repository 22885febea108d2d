"""K9 one-shot all-reduce (csrc/oneshot_ar.hip) across processes sharing the GPU via IPC."""
import json
import os
import subprocess
import sys

import pytest

from test_distributed_cpu import ROOT, free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_allreduce_ranks_on_one_gpu(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tools", "oneshot_check.py")]
    env = dict(os.environ, ROUNDTABLE_DIST_BACKEND="gloo", OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"ranks"')]
    assert len(recs) == 1, r.stdout[-2000:]
    ranks = recs[0]["ranks"]
    assert sorted(o["rank"] for o in ranks) == list(range(world))
    assert all(o["checks"] == 6 + 15 for o in ranks)
    # creation ran the exact self-tests: K9 values over both slots, then the fused GEMM + exchange
    # (EPI_AR) bit-identical to GEMM + K9 at three shard shapes
    assert all(o["fused_gemm_ar"] is True and o["self_test_latency_us"] > 0 for o in ranks), ranks
    assert next(o for o in ranks if o["rank"] == 0).get("expiry_flagged") is True
