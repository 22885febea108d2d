"""Self-launch of the SPMD ranks a project's knight placement needs.

The reference runs ``roundtable discuss "<topic>"`` as ONE command (/root/reference/src/index.ts:68-77).
Here a knight with ``engine.tp > 1`` needs one process per GPU of its tensor-parallel group
(torch.distributed / RCCL), so ``discuss``, ``summon``, ``apply`` and ``code-red`` check the
loaded config BEFORE anything touches a GPU and, when a placement needs ranks, re-run
themselves as a child ``torch.distributed.run`` with that many ranks (every rank runs the
command SPMD: knights/spmd.py; rank 0 owns the terminal and the project files) and exit with
its code. A tp > 1 knight is never silently run at tp = 1.

Knights with ``tp == 1`` on different GPUs need no ranks: one process drives every GPU (one
engine and host thread per GPU, knights/engine_backend.py EnginePool).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional, Tuple

from ..config import engine_settings
from ..errors import ConfigError
from ..types import RoundtableConfig

LAUNCHED_ENV = "ROUNDTABLE_SPMD_CHILD"


def _uses_engine(config: RoundtableConfig, adapter_id: str, st: dict) -> bool:
    from ..knights.external import wants_external
    if st.get("backend") == "fake" or adapter_id.startswith("fake"):
        return False
    ac = config.adapter_config.get(adapter_id) or {}
    return not (isinstance(ac, dict) and wants_external(adapter_id, ac))


def ranks_needed(config: RoundtableConfig) -> Tuple[int, str, bool]:
    """(ranks, reason, cpu): 1 when every engine knight has tp 1; else enough ranks for every
    tensor-parallel group and every explicit ``engine.gpus`` entry. ``cpu``: all engine knights
    run on the CPU (gloo ranks, tests)."""
    need, why, cpu, tps = 1, "", True, []
    gpu_max = 0
    for k in config.knights:
        st = engine_settings(config, k.adapter)
        if not _uses_engine(config, k.adapter, st):
            continue
        tp = int(st.get("tp", 1) or 1)
        gpus = st.get("gpus")
        if isinstance(gpus, list) and gpus:
            gpu_max = max(gpu_max, max(int(g) for g in gpus) + 1)
            if tp > 1 and len(gpus) != tp:
                raise ConfigError(f"{k.adapter}: engine.tp={tp} but engine.gpus lists {len(gpus)} GPU(s)",
                                  hint="Give a tensor-parallel knight exactly tp GPUs (or omit gpus).")
        if str(st.get("device", "")) != "cpu":
            cpu = False
        if tp > 1:
            tps.append((k.name, tp))
            need = max(need, tp)
    if need > 1:
        need = max(need, gpu_max)
        why = ", ".join(f"{n} tp={t}" for n, t in tps)
    return need, why, cpu


def launch_command() -> List[str]:
    """argv prefix of a child rank: the same interpreter, our package."""
    return [sys.executable, "-m", "theroundtaible_amd"]


def maybe_relaunch(argv: List[str], root: Optional[str] = None, quiet: bool = False) -> Optional[int]:
    """Run ``argv`` under a child torchrun when the project's placement needs ranks; return its
    exit code, or None when this process should run the command itself (no config, tp = 1
    everywhere, or already a rank)."""
    if "WORLD_SIZE" in os.environ or os.environ.get(LAUNCHED_ENV):
        return None
    root = root or os.getcwd()
    if not os.path.exists(os.path.join(root, ".roundtable", "config.json")):
        return None
    from ..config import load_config
    try:
        config = load_config(root)
    except Exception:  # noqa: BLE001 - the command itself reports config errors
        return None
    n, why, cpu = ranks_needed(config)
    if n <= 1:
        return None
    if not cpu:
        import torch     # device_count() does not initialise the GPU on this image (no HIP context)
        have = torch.cuda.device_count()
        if have < n:
            raise ConfigError(f"the knight placement needs {n} GPU ranks ({why}) but {have} GPU(s) are visible",
                              hint="Lower engine.tp / engine.gpus in .roundtable/config.json, or run on a "
                                   "node with enough GPUs.")
    return launch_ranks(n, argv, cpu, why, quiet)


def launch_ranks(n: int, argv: List[str], cpu: bool, why: str, quiet: bool = False) -> int:
    """Run ``roundtable <argv>`` as ``n`` SPMD ranks (a child ``torch.distributed.run``, started
    before this process touches a GPU) and return its exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", "-m", "theroundtaible_amd", *argv]
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    env[LAUNCHED_ENV] = "1"
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    if cpu:
        env.setdefault("OMP_NUM_THREADS", "1")
    else:
        from .cluster import limit_shared_gpu_queues
        limit_shared_gpu_queues(env, n)
    if not quiet:
        print(f"  Launching {n} ranks ({why})", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def collective_timeout_s(config: RoundtableConfig, world: Optional[int] = None) -> int:
    """Process-group timeout of an SPMD command (containment outside the bench).
    A rank waits in a collective at most while the ranks it waits for run their turns: the turn
    timeout (``rules.timeout_per_turn_seconds``, 120 s by default) times the most knight groups one
    rank runs one after another, plus a minute of margin — 180 s for the usual one group per rank,
    instead of torch's 30-minute default. Waits on a person (the King) use the cluster's
    long-timeout wait group instead."""
    env = os.environ.get("ROUNDTABLE_COLLECTIVE_TIMEOUT_S")   # explicit override (operators, tests)
    if env:
        return max(1, int(float(env)))
    t = float(getattr(config.rules, "timeout_per_turn_seconds", 120) or 120)
    world = world or int(os.environ.get("WORLD_SIZE", "1"))
    per_rank = 1
    try:
        from ..knights.spmd import plan_placement
        pl = plan_placement(config, max(1, world))
        counts: dict = {}
        for ranks in {tuple(r) for r in pl.values()}:
            for r in ranks:
                counts[r] = counts.get(r, 0) + 1
        per_rank = max(counts.values(), default=1)
    except Exception:  # noqa: BLE001 - a bad placement is reported by the backend factory
        pass
    return int(max(120.0, per_rank * t + 60.0))
