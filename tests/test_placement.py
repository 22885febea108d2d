"""GPU scouting + automatic knight placement for `roundtable init` (parallel/placement.py),
against faked inventories (no GPU needed)."""
import json

from theroundtaible_amd.cli import main
from theroundtaible_amd.parallel.costmodel import split_plans
from theroundtaible_amd.parallel.placement import (GIB, GpuInfo, Inventory, PlacementPolicy, kv_bytes_per_token,
                                                   model_bytes, parse_topotype, plan_placement)

PACK = PlacementPolicy(mode="pack")
SPREAD = PlacementPolicy(mode="spread")


def node(n=8, hbm=288):
    gpus = [GpuInfo(i, "AMD Instinct MI355X", "gfx950", hbm * GIB, (hbm - 2) * GIB, 256) for i in range(n)]
    links = {f"{i}-{j}": "XGMI" for i in range(n) for j in range(i + 1, n)}
    return Inventory(gpus, links)


def test_model_sizes():
    assert 14.5 * GIB < model_bytes("llama3-8b") < 15.5 * GIB
    assert 130 * GIB < model_bytes("llama3-70b") < 133 * GIB
    assert kv_bytes_per_token("llama3-8b") == 128 * 1024 and kv_bytes_per_token("llama3-70b") == 320 * 1024


def test_pack_policy_same_model_knights_share_one_gpu():
    plans = plan_placement([{"name": n, "model": "llama3-8b"} for n in "ABC"], node(), PACK)
    assert len(plans) == 1 and plans[0].tp == 1 and plans[0].gpus == [0] and plans[0].knights == ["A", "B", "C"]


def test_pack_policy_70b_tp_by_latency_target_and_by_memory():
    p = plan_placement([{"name": n, "model": "llama3-70b"} for n in "AB"], node(), PACK)
    assert p[0].tp == 4 and p[0].gpus == [0, 1, 2, 3] and p[0].step_ms < 8
    assert plan_placement([{"name": "A", "model": "llama3-70b"}], node(1), PACK)[0].tp == 1   # fits alone
    small = plan_placement([{"name": "A", "model": "llama3-70b"}], node(4, hbm=64), PACK)
    assert small[0].tp == 4 and small[0].reason == "memory fit"


def test_auto_lone_8b_table_gets_tensor_parallel_from_the_model():
    """a lone 3 x Llama-3-8B table on an 8-GPU node must not idle 7 GPUs — the
    cost model's fastest layout (one batched tp engine) is what the planner returns."""
    plans = plan_placement([{"name": n, "model": "llama3-8b"} for n in "ABC"], node())
    best_ms, best = split_plans("llama3-8b", 3, 8)[0]
    assert [(len(p.knights), p.tp) for p in plans] == best and plans[0].tp > 1
    assert abs(sum(p.round_ms for p in plans[:1]) - best_ms) < 1.0
    assert sorted(g for p in plans for g in p.gpus) == list(range(sum(p.tp for p in plans)))


def test_spread_config3_mistral_one_per_gpu_and_config5_70b_tp4_each():
    """BASELINE config 3 (8 Mistral knights one-per-GPU) and config 5 (2 x Llama-3-70B, TP=4 each,
    disjoint groups) under the ``spread`` policy."""
    p3 = plan_placement([{"name": f"M{i}", "model": "mistral-7b"} for i in range(8)], node(), SPREAD)
    assert [(p.tp, p.gpus, p.knights) for p in p3] == [(1, [i], [f"M{i}"]) for i in range(8)]
    p5 = plan_placement([{"name": n, "model": "llama3-70b"} for n in "AB"], node(), SPREAD)
    assert [(p.tp, p.gpus) for p in p5] == [(4, [0, 1, 2, 3]), (4, [4, 5, 6, 7])]


def test_auto_memory_fit_and_sequential_mode():
    assert plan_placement([{"name": "A", "model": "llama3-70b"}], node(1))[0].tp == 1   # one GPU: fits alone
    small = plan_placement([{"name": "A", "model": "llama3-70b"}], node(4, hbm=64))
    assert small[0].tp == 4                                                               # memory forces tp 4
    seq = plan_placement([{"name": n, "model": "llama3-8b"} for n in "ABC"], node(),
                         PlacementPolicy(round_mode="sequential"))
    assert sum(p.tp for p in seq) <= 8 and max(p.tp for p in seq) > 1


def test_heterogeneous_models_get_disjoint_groups_then_share():
    ks = [{"name": "A", "model": "llama3-8b"}, {"name": "B", "model": "llama3-70b"}, {"name": "C", "model": "mistral-7b"}]
    p = {pl.model: pl for pl in plan_placement(ks, node())}
    assert p["llama3-70b"].gpus == [0, 1, 2, 3] and p["llama3-8b"].gpus == [4] and p["mistral-7b"].gpus == [5]
    p2 = {pl.model: pl for pl in plan_placement(ks[:1] + ks[2:], node(1))}
    assert p2["llama3-8b"].gpus == [0] and p2["mistral-7b"].gpus == [0]
    assert "shares GPUs" in p2["mistral-7b"].reason or "shares GPUs" in p2["llama3-8b"].reason


def test_parse_rocm_smi_topotype():
    text = json.dumps({"system": {"(Topology) Link type between DRM devices 0 and 1": "XGMI",
                                  "(Topology) Link type between DRM devices 1 and 0": "XGMI",
                                  "(Topology) Link type between DRM devices 0 and 2": "PCIE"}})
    assert parse_topotype(text) == {"0-1": "XGMI", "0-2": "PCIE"}
    assert parse_topotype("not json") == {}


def test_init_writes_automatic_placement(project, monkeypatch):
    monkeypatch.setenv("ROUNDTABLE_FAKE_GPUS", json.dumps(node().to_json()))
    assert main(["--quiet", "init", "--yes", "--model", "llama3-70b", "--knights", "2"]) == 0
    cfg = json.load(open(project / ".roundtable" / "config.json"))
    best = split_plans("llama3-70b", 2, 8)[0][1]          # the cost model's layout (auto policy)
    assert best == [(2, 8)]
    for aid in ("claude-cli", "gemini-cli"):
        eng = cfg["adapter_config"][aid]["engine"]
        assert eng["tp"] == 8 and eng["gpus"] == list(range(8))
    grp = cfg["engine"]["placement"]["groups"]
    assert grp[0]["model"] == "llama3-70b" and grp[0]["tp"] == 8 and grp[0]["round_ms"] > 0
    assert len(cfg["engine"]["placement"]["inventory"]["gpus"]) == 8


def test_init_manual_tp_overrides_placement(project, monkeypatch):
    monkeypatch.setenv("ROUNDTABLE_FAKE_GPUS", json.dumps(node().to_json()))
    assert main(["--quiet", "init", "--yes", "--model", "llama3-8b", "--knights", "3", "--tp", "2"]) == 0
    cfg = json.load(open(project / ".roundtable" / "config.json"))
    assert [cfg["adapter_config"][a]["engine"]["gpus"] for a in ("claude-cli", "gemini-cli", "openai-cli")] == \
        [[0, 1], [2, 3], [4, 5]]
    assert "placement" not in cfg["engine"]


def test_measured_calibration_changes_the_plan(tmp_path, monkeypatch):
    """$ROUNDTABLE_CALIBRATION (bench.py --write-calibration after an N-GPU run) replaces the
    assumed K9 latency: a slow measured xGMI all-reduce makes the planner give the lone 8B
    table fewer GPUs than the default, a fused form that saves most of it gives it more."""
    from theroundtaible_amd.parallel import costmodel
    knights = [{"name": n, "model": "llama3-8b"} for n in "ABC"]
    default_tp = plan_placement(knights, node())[0].tp
    path = tmp_path / "cal.json"
    path.write_text(json.dumps({"ar_us": 60.0, "fused_ar_saving_us": 0.0, "source": "test"}))
    monkeypatch.setenv(costmodel.CALIBRATION_ENV, str(path))
    assert costmodel.default_calibration().ar_us == 60.0
    slow_tp = plan_placement(knights, node())[0].tp
    assert slow_tp < default_tp
    path.write_text(json.dumps({"ar_us": 60.0, "fused_ar_saving_us": 58.0}))
    import os
    os.utime(path, (os.path.getatime(path), os.path.getmtime(path) + 5))   # new content, new mtime
    assert costmodel.default_calibration().fused_ar_saving_us == 58.0
    assert plan_placement(knights, node())[0].tp >= default_tp
