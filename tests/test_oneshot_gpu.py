"""K9 one-shot all-reduce (csrc/oneshot_ar.hip) across processes sharing the GPU via IPC."""
import json
import os
import subprocess
import sys

import pytest

from test_distributed_cpu import ROOT, free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,fused_mode", [(2, "1"), (4, "auto"), (2, "probe")])
def test_oneshot_allreduce_ranks_on_one_gpu(world, fused_mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tools", "oneshot_check.py")]
    # ROUNDTABLE_FUSED_AR: 1 = fused GEMM + exchange forced although the ranks share the GPU;
    # auto = the default (ranks sharing a GPU keep the separate K9); probe = self-test + the timed
    # decision the default takes when every rank owns its GPU
    env = dict(os.environ, ROUNDTABLE_DIST_BACKEND="gloo", OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0",
               ROUNDTABLE_FUSED_AR=fused_mode)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"ranks"')]
    assert len(recs) == 1, r.stdout[-2000:]
    ranks = recs[0]["ranks"]
    assert sorted(o["rank"] for o in ranks) == list(range(world))
    # (6 eager sizes + 2 residual-form calls + 1 fused check when fused) x both protocols (LL and
    # push + fence + flag) + 15 graph replays + 3 gather replays
    assert all(o["checks"] == 2 * (6 + 2 + int(o["fused_gemm_ar"])) + 15 + 3 and o["gather_ok"] is True
               for o in ranks), ranks
    # the protocol choice: both forms passed the self-test and were timed; identical on every rank
    assert len({(o["ll"], o["flag_latency_us"], o["ll_latency_us"]) for o in ranks}) == 1, ranks
    assert all(o["flag_latency_us"] > 0 and o["ll_latency_us"] > 0 for o in ranks), ranks
    assert all(o.get("fused_residual_checked", False) == o["fused_gemm_ar"] for o in ranks), ranks
    # creation ran the exact self-tests: K9 values over both slots, then the fused GEMM + exchange
    # (EPI_AR) bit-identical to GEMM + K9 at three shard shapes
    assert all(o["self_test_latency_us"] > 0 for o in ranks), ranks
    if fused_mode == "1":
        assert all(o["fused_gemm_ar"] is True for o in ranks), ranks
    elif fused_mode == "auto":        # ranks share the GPU: separate K9 launches, no probe
        assert all(o["fused_gemm_ar"] is False and o["fused_saving_us"] is None for o in ranks), ranks
    else:                             # timed decision, identical on every rank
        assert len({(o["fused_gemm_ar"], o["fused_saving_us"]) for o in ranks}) == 1, ranks
        assert all(o["fused_gemm_ar"] is (o["fused_saving_us"] >= 0.5) for o in ranks), ranks
    assert next(o for o in ranks if o["rank"] == 0).get("expiry_flagged") is True
