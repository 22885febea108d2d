"""GPU scouting + automatic knight placement for `roundtable init` (parallel/placement.py),
against faked inventories (no GPU needed)."""
import json

from theroundtaible_amd.cli import main
from theroundtaible_amd.parallel.placement import (GIB, GpuInfo, Inventory, kv_bytes_per_token, model_bytes,
                                                   parse_topotype, plan_placement)


def node(n=8, hbm=288):
    gpus = [GpuInfo(i, "AMD Instinct MI355X", "gfx950", hbm * GIB, (hbm - 2) * GIB, 256) for i in range(n)]
    links = {f"{i}-{j}": "XGMI" for i in range(n) for j in range(i + 1, n)}
    return Inventory(gpus, links)


def test_model_sizes():
    assert 14.5 * GIB < model_bytes("llama3-8b") < 15.5 * GIB
    assert 130 * GIB < model_bytes("llama3-70b") < 133 * GIB
    assert kv_bytes_per_token("llama3-8b") == 128 * 1024 and kv_bytes_per_token("llama3-70b") == 320 * 1024


def test_same_model_knights_share_one_gpu():
    plans = plan_placement([{"name": n, "model": "llama3-8b"} for n in "ABC"], node())
    assert len(plans) == 1 and plans[0].tp == 1 and plans[0].gpus == [0] and plans[0].knights == ["A", "B", "C"]


def test_70b_tp_by_latency_target_and_by_memory():
    p = plan_placement([{"name": n, "model": "llama3-70b"} for n in "AB"], node())
    assert p[0].tp == 4 and p[0].gpus == [0, 1, 2, 3] and p[0].step_ms < 8      # config 5: TP=4
    assert plan_placement([{"name": "A", "model": "llama3-70b"}], node(1))[0].tp == 1   # one GPU: fits alone
    small = plan_placement([{"name": "A", "model": "llama3-70b"}], node(4, hbm=64))
    assert small[0].tp == 4 and small[0].reason == "memory fit"


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
    for aid in ("claude-cli", "gemini-cli"):
        eng = cfg["adapter_config"][aid]["engine"]
        assert eng["tp"] == 4 and eng["gpus"] == [0, 1, 2, 3]
    grp = cfg["engine"]["placement"]["groups"]
    assert grp[0]["model"] == "llama3-70b" and grp[0]["tp"] == 4
    assert len(cfg["engine"]["placement"]["inventory"]["gpus"]) == 8


def test_init_manual_tp_overrides_placement(project, monkeypatch):
    monkeypatch.setenv("ROUNDTABLE_FAKE_GPUS", json.dumps(node().to_json()))
    assert main(["--quiet", "init", "--yes", "--model", "llama3-8b", "--knights", "3", "--tp", "2"]) == 0
    cfg = json.load(open(project / ".roundtable" / "config.json"))
    assert [cfg["adapter_config"][a]["engine"]["gpus"] for a in ("claude-cli", "gemini-cli", "openai-cli")] == \
        [[0, 1], [2, 3], [4, 5]]
    assert "placement" not in cfg["engine"]
