"""The single-process multi-engine path: knights placed on different engines of
ONE process (``EnginePool`` — on a node, one engine per GPU via ``engine.gpus``; here CPU
stand-ins with distinct weights so every knight gets its own engine) run a parallel round as
one batched decode per engine, the engines concurrently on their own threads
(orchestrator.execute_plan), and the per-device KV split of ``EnginePool.finalize``."""
import threading

from theroundtaible_amd.knights.registry import BackendFactory, initialize_backends
from theroundtaible_amd.orchestrator import Orchestrator, RunOptions
from theroundtaible_amd.types import RoundtableConfig


def _config(n):
    knights = [{"name": f"Ridder{i}", "adapter": f"local-llm-r{i}", "capabilities": ["x"], "priority": i + 1}
               for i in range(n)]
    return RoundtableConfig.from_dict({
        "version": "1.0", "project": "pool", "language": "nl", "knights": knights,
        "rules": {"max_rounds": 1, "consensus_threshold": 9, "timeout_per_turn_seconds": 300,
                  "escalate_to_user_after": 5, "auto_execute": False, "ignore": [".git"], "round_mode": "parallel"},
        "chronicle": ".roundtable/chronicle.md",
        "engine": {"default_model": "tiny-llama", "max_new_tokens": 6, "ignore_eos": True, "temperature": 0.0,
                   "device": "cpu"},
        # one engine per knight: distinct weights = distinct EnginePool keys (a GPU node gives each
        # its own `gpus: [i]`; the pool / thread / KV-split logic is the same)
        "adapter_config": {f"local-llm-r{i}": {"engine": {"weights": f"random-full:{i + 1}"}} for i in range(n)}})


def test_engines_of_one_process_decode_concurrently(tmp_path):
    cfg = _config(3)
    factory = BackendFactory(cfg)
    backends = initialize_backends(cfg, factory=factory)
    assert len(backends) == 3
    engines = list(factory.pool.engines.values())
    assert len(engines) == 3 and all(e.kv_allocated for e in engines)
    # each engine's batch must run on its own thread AT THE SAME TIME: a barrier all three engines
    # must reach inside their run_turns (a sequential loop would time out on it)
    barrier = threading.Barrier(3, timeout=60)
    seen = {}
    for i, e in enumerate(engines):
        real = e.run_turns

        def wrapped(turns, real=real, i=i):
            seen[i] = (threading.get_ident(), len(turns))
            barrier.wait()
            return real(turns)

        e.run_turns = wrapped
    orch = Orchestrator(cfg, backends, str(tmp_path), options=RunOptions(shuffle_seed=3, max_new_tokens=6,
                                                                         write_chronicle=False),
                        store_root=str(tmp_path))
    res = orch.run("Een onderwerp voor drie motoren in een proces")
    assert not orch.failures, orch.failures
    assert sorted(seen) == [0, 1, 2] and len({t for t, _ in seen.values()}) == 3
    assert all(n == 1 for _, n in seen.values())
    assert len([e for e in orch.all_rounds if e.round == 1]) == 3
    assert res is not None


def test_pool_shares_an_engine_between_knights_of_one_setting(tmp_path):
    """Two knights with the same effective settings share ONE engine (one batched decode)."""
    cfg = _config(2)
    for ac in cfg.adapter_config.values():
        ac["engine"]["weights"] = "random-full:9"
    factory = BackendFactory(cfg)
    backends = initialize_backends(cfg, factory=factory)
    assert len(backends) == 2 and len(factory.pool.engines) == 1
    e = next(iter(factory.pool.engines.values()))
    calls = []
    real = e.run_turns
    e.run_turns = lambda turns: calls.append(len(turns)) or real(turns)
    orch = Orchestrator(cfg, backends, str(tmp_path), options=RunOptions(shuffle_seed=1, max_new_tokens=6,
                                                                         write_chronicle=False),
                        store_root=str(tmp_path))
    orch.run("Twee ridders, een motor")
    assert calls == [2] and not orch.failures
