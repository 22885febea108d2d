"""Local checkpoint discovery (utils/local_detect.py) and its use by `roundtable init`."""
import json
import os

from theroundtaible_amd.utils.local_detect import (detect_local_models, is_non_chat_model, match_preset,
                                                    prettify_model_name)

LLAMA8B_HF = {"model_type": "llama", "hidden_size": 4096, "num_hidden_layers": 32, "num_attention_heads": 32,
              "num_key_value_heads": 8, "intermediate_size": 14336, "vocab_size": 128256,
              "max_position_embeddings": 131072, "rope_theta": 500000.0, "rms_norm_eps": 1e-5}


def _ckpt(d, hf):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(hf, f)
    open(os.path.join(d, "model-00001-of-00001.safetensors"), "wb").close()


def test_prettify_and_filters():
    assert prettify_model_name("meta-llama/Meta-Llama-3-8b-instruct") == "Meta Llama 3 8B Instruct"
    assert prettify_model_name("qwen2.5_coder-14b") == "Qwen2.5 Coder 14B"
    assert is_non_chat_model("nomic-embed-text") and is_non_chat_model("bge-reranker-v2")
    assert not is_non_chat_model("llama-3-8b")


def test_detect_and_match(tmp_path):
    _ckpt(str(tmp_path / "Meta-Llama-3-8B"), LLAMA8B_HF)
    hub = tmp_path / "hub" / "models--mistralai--Mistral-7B-v0.3" / "snapshots" / "abc"
    _ckpt(str(hub), dict(LLAMA8B_HF, model_type="mistral", vocab_size=32768, rope_theta=1e6,
                         max_position_embeddings=32768))
    _ckpt(str(tmp_path / "all-MiniLM-embed"), LLAMA8B_HF)                 # skipped: embedding model
    os.makedirs(tmp_path / "no-weights")
    with open(tmp_path / "no-weights" / "config.json", "w") as f:       # skipped: no safetensors
        json.dump(LLAMA8B_HF, f)
    found = {m.model_id: m for m in detect_local_models([str(tmp_path), str(tmp_path / "hub")])}
    assert set(found) == {"Meta-Llama-3-8B", "mistralai/Mistral-7B-v0.3"}
    assert found["Meta-Llama-3-8B"].preset == "llama3-8b" and found["Meta-Llama-3-8B"].overrides == {}
    mis = found["mistralai/Mistral-7B-v0.3"]
    assert mis.preset == "mistral-7b" and mis.overrides == {"vocab": 32768}
    assert mis.adapter_slug() == "mistral-7b-v0-3"


def test_detect_qwen2_family(tmp_path):
    """Qwen2.5 checkpoints (model_type qwen2) map to the Qwen presets with q/k/v biases; a Llama
    variant with biased o / MLP projections is not offered (the engine's block has none)."""
    qwen7b = {"model_type": "qwen2", "hidden_size": 3584, "num_hidden_layers": 28, "num_attention_heads": 28,
              "num_key_value_heads": 4, "intermediate_size": 18944, "vocab_size": 152064,
              "max_position_embeddings": 32768, "rope_theta": 1000000.0, "rms_norm_eps": 1e-6,
              "tie_word_embeddings": False}
    _ckpt(str(tmp_path / "Qwen2.5-7B-Instruct"), qwen7b)
    _ckpt(str(tmp_path / "Qwen2.5-Coder-0.5B"), dict(qwen7b, hidden_size=896, num_hidden_layers=24,
                                                     num_attention_heads=14, num_key_value_heads=2,
                                                     intermediate_size=4864, vocab_size=151936,
                                                     tie_word_embeddings=True))
    _ckpt(str(tmp_path / "llama-attn-bias"), dict(LLAMA8B_HF, attention_bias=True))
    found = {m.model_id: m for m in detect_local_models([str(tmp_path)])}
    assert set(found) == {"Qwen2.5-7B-Instruct", "Qwen2.5-Coder-0.5B"}
    assert found["Qwen2.5-7B-Instruct"].preset == "qwen2.5-7b" and found["Qwen2.5-7B-Instruct"].overrides == {}
    assert found["Qwen2.5-Coder-0.5B"].preset == "qwen2.5-0.5b" and found["Qwen2.5-Coder-0.5B"].overrides == {}
    from theroundtaible_amd.models.config import get_config
    # preset shapes = the published parameter counts (Qwen2.5 0.5-72B, Llama 3.1-8B, 3.2-1B / 3B)
    for name, b in (("qwen2.5-0.5b", 0.49), ("qwen2.5-7b", 7.62), ("qwen2.5-14b", 14.77), ("qwen2.5-32b", 32.76),
                    ("qwen2.5-72b", 72.71), ("llama3.1-8b", 8.03), ("llama3.2-1b", 1.24), ("llama3.2-3b", 3.21)):
        assert abs(get_config(name).n_params() / 1e9 - b) < 0.01, name


def test_rope_scaling_and_theta_formats(tmp_path):
    """Llama 3.1 (rope_scaling llama3, old file format), a transformers-5 file (rope_parameters
    with rope_theta inside) and an unsupported scaling type (not offered)."""
    from theroundtaible_amd.utils.local_detect import checkpoint_model
    l31 = dict(LLAMA8B_HF, rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                         "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    _ckpt(str(tmp_path / "Llama-3.1-8B"), l31)
    preset, ov = checkpoint_model(str(tmp_path / "Llama-3.1-8B"))
    assert preset == "llama3.1-8b" and ov == {}
    v5 = {k: v for k, v in LLAMA8B_HF.items() if k != "rope_theta"}
    v5["rope_parameters"] = {"rope_theta": 500000.0, "rope_type": "default"}
    _ckpt(str(tmp_path / "v5"), v5)
    assert checkpoint_model(str(tmp_path / "v5")) == ("llama3-8b", {})
    _ckpt(str(tmp_path / "longrope"), dict(LLAMA8B_HF, rope_scaling={"rope_type": "longrope", "factor": 4.0}))
    assert checkpoint_model(str(tmp_path / "longrope")) is None


def test_match_gpt2():
    preset, diff = match_preset({"arch": "gpt2", "n_layers": 12, "hidden": 768, "n_heads": 12, "n_kv_heads": 12,
                                 "head_dim": 64, "ffn": 3072, "vocab": 50257, "max_pos": 1024, "rope_theta": 0.0,
                                 "norm_eps": 1e-5, "tie_embeddings": True})
    assert preset == "gpt2-small" and diff == {"max_pos": 1024}


def test_init_seats_local_checkpoints(tmp_path, monkeypatch):
    from theroundtaible_amd.cli import main
    _ckpt(str(tmp_path / "models" / "Meta-Llama-3-8B"), LLAMA8B_HF)
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("HF_HOME", str(tmp_path / "nohf"))
    monkeypatch.delenv("ROUNDTABLE_MODELS_DIR", raising=False)
    assert main(["--quiet", "init", "--yes", "--knights", "2", "--local-models"]) == 0
    cfg = json.load(open(tmp_path / ".roundtable" / "config.json"))
    adapters = [k["adapter"] for k in cfg["knights"]]
    assert "local-llm-meta-llama-3-8b" in adapters
    eng = cfg["adapter_config"]["local-llm-meta-llama-3-8b"]["engine"]
    assert eng["model"] == "llama3-8b" and eng["weights"].endswith("Meta-Llama-3-8B")


def test_detect_local_servers_and_cli_fallback():
    from theroundtaible_amd.knights.external import HttpResponse
    from theroundtaible_amd.utils.local_detect import detect_local_servers, fetch_models_from_ollama_cli

    def http(method, url, body, headers, timeout):
        assert timeout == 3.0 and url.endswith("/v1/models")
        if ":1234" in url:
            return HttpResponse(200, json.dumps({"data": [{"id": "qwen2.5-coder-14b"}, {"id": "nomic-embed-text"}]}))
        raise OSError("connection refused")

    listing = "NAME              ID      SIZE\nllama3.1:8b   abc  4.7 GB\nmistral:latest def 4 GB\n"
    found = detect_local_servers(http=http, ollama_cli=lambda: listing)
    assert [(m.model_id, m.source) for m in found] == [("qwen2.5-coder-14b", "LM Studio"), ("llama3.1:8b", "Ollama"),
                                                     ("mistral", "Ollama")]
    assert found[0].adapter_config() == {"endpoint": "http://localhost:1234", "model": "qwen2.5-coder-14b",
                                         "name": "Qwen2.5 Coder 14B", "source": "LM Studio"}
    assert found[1].adapter_slug() == "llama3-1-8b" and found[2].name == "Mistral"
    assert fetch_models_from_ollama_cli(run=lambda: (_ for _ in ()).throw(OSError("no ollama"))) == []


def test_init_seats_running_server(tmp_path, monkeypatch):
    from theroundtaible_amd import cli
    from theroundtaible_amd.utils import local_detect
    from theroundtaible_amd.knights.registry import BackendFactory
    from theroundtaible_amd.knights.external import LocalLlmHttpBackend
    from theroundtaible_amd.config import load_config
    sm = local_detect.ServerModel("Llama3.1 8B", "llama3.1:8b", "http://127.0.0.1:11434", "Ollama")
    monkeypatch.setattr(local_detect, "detect_local_servers", lambda: [sm])
    monkeypatch.setattr(cli, "detect_tools", lambda: {"claude": True, "gemini": False, "codex": False})
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("HF_HOME", str(tmp_path / "nohf"))
    assert cli.main(["--quiet", "init", "--yes", "--knights", "2", "--servers", "--external-clis"]) == 0
    raw = json.load(open(tmp_path / ".roundtable" / "config.json"))
    assert raw["adapter_config"]["local-llm-llama3-1-8b"]["endpoint"] == "http://127.0.0.1:11434"
    assert "engine" not in raw["adapter_config"]["local-llm-llama3-1-8b"]
    assert raw["adapter_config"]["claude-cli"]["backend"] == "external"
    assert "backend" not in raw["adapter_config"]["gemini-cli"]
    cfg = load_config(str(tmp_path))
    b = BackendFactory(cfg).create("local-llm-llama3-1-8b")
    assert isinstance(b, LocalLlmHttpBackend) and b.source == "Ollama"


def test_update_check():
    from theroundtaible_amd.knights.external import HttpResponse
    from theroundtaible_amd.utils.update_check import check_for_update, is_newer
    assert is_newer("0.2.0", "0.1.9") and not is_newer("0.1.0", "0.1.0") and is_newer("1.0", "0.9.9")
    assert check_for_update(url=None) is None or os.environ.get("ROUNDTABLE_UPDATE_URL")
    ok = lambda *a: HttpResponse(200, json.dumps({"info": {"version": "9.0.0"}}))
    assert check_for_update("http://pypi/x", "0.1.0", http=ok) == "9.0.0"
    assert check_for_update("http://pypi/x", "9.0.0", http=ok) is None
    assert check_for_update("http://pypi/x", "0.1.0", http=lambda *a: (_ for _ in ()).throw(OSError())) is None
