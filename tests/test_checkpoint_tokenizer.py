"""Checkpoint tokenizers: a weights directory that ships ``tokenizer.json`` (+ chat template and
end ids) is tokenized with its own vocabulary, every turn wrapped as one user message, and
generation stops at the checkpoint's end-of-turn ids (engine/tokenizer.py::HFTokenizer)."""
import json

import pytest
import torch

transformers = pytest.importorskip("transformers")
tokenizers = pytest.importorskip("tokenizers")

from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn  # noqa: E402
from theroundtaible_amd.engine.engine import cut_at_stop  # noqa: E402
from theroundtaible_amd.engine.tokenizer import HFTokenizer  # noqa: E402

SPECIAL = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"]
LLAMA3_TEMPLATE = (
    "{% for message in messages %}{% set content = '<|start_header_id|>' + message['role'] + "
    "'<|end_header_id|>\\n\\n' + message['content'] | trim + '<|eot_id|>' %}{% if loop.index0 == 0 %}"
    "{% set content = bos_token + content %}{% endif %}{{ content }}{% endfor %}{% if add_generation_prompt %}"
    "{{ '<|start_header_id|>assistant<|end_header_id|>\\n\\n' }}{% endif %}")


def _checkpoint(d, template=LLAMA3_TEMPLATE):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    corpus = ["De ridders van de ronde tafel bespreken de kernel en de cache.",
              "Consensus score negen: het voorstel wordt aangenomen door de koning."] * 20
    tok.train_from_iterator(corpus, trainers.BpeTrainer(vocab_size=400, special_tokens=SPECIAL,
                                                        initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    tok.save(str(d / "tokenizer.json"))
    V = tok.get_vocab_size()
    bos, end, eot = (tok.token_to_id(s) for s in ("<|begin_of_text|>", "<|end_of_text|>", "<|eot_id|>"))
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(transformers.LlamaConfig(
        hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
        vocab_size=V, max_position_embeddings=4096, rope_theta=10000.0, rms_norm_eps=1e-5, tie_word_embeddings=False,
        bos_token_id=bos, eos_token_id=end))
    m.save_pretrained(str(d), safe_serialization=True)   # writes config.json + generation_config.json
    cfg = {"bos_token": "<|begin_of_text|>", "eos_token": "<|eot_id|>"}
    if template:
        cfg["chat_template"] = template
    (d / "tokenizer_config.json").write_text(json.dumps(cfg))
    (d / "generation_config.json").write_text(json.dumps({"bos_token_id": bos, "eos_token_id": [end, eot]}))
    return tok, V


def _engine(d, V):
    return Engine(EngineConfig(model="tiny-llama", weights=str(d), device="cpu", dtype="fp32", num_blocks=64,
                               model_overrides={"vocab": V}))


def test_checkpoint_tokenizer_chat_wrap_and_stops(tmp_path):
    tok, V = _checkpoint(tmp_path)
    e = _engine(tmp_path, V)
    t = e.tokenizer
    assert isinstance(t, HFTokenizer) and t.family.startswith("hf:")
    assert t.stop_ids == {tok.token_to_id("<|end_of_text|>"), tok.token_to_id("<|eot_id|>")}
    text = "De ridders bespreken de cache."
    ids = e.encode_prompt(text)
    want = tok.encode("<|begin_of_text|><|start_header_id|>user<|end_header_id|>\n\n" + text +
                      "<|eot_id|><|start_header_id|>assistant<|end_header_id|>\n\n").ids
    assert ids == want
    assert t.decode(t.encode(text)) == text
    # the wrap is constant: a longer prompt re-prefills only the suffix + the new content
    sp = SamplingParams(temperature=0.0, max_new_tokens=5, ignore_eos=True, stop_on_consensus=False)
    r1 = e.run_turns([Turn("K", text, sp)])[0]
    r2 = e.run_turns([Turn("K", text + " Het voorstel wordt aangenomen.", sp)])[0]
    assert r1.error is None and r2.error is None and len(r2.ids) == 5
    assert r2.metrics["reused_tokens"] >= len(t.chat_prefix) + len(t.encode(text)) - 1
    eot = tok.token_to_id("<|eot_id|>")
    assert cut_at_stop([5, 6, eot, 7], t.stop_ids) == [5, 6, eot]


def test_checkpoint_without_template_gets_bos_only(tmp_path):
    tok, V = _checkpoint(tmp_path, template=None)
    e = _engine(tmp_path, V)
    assert e.tokenizer.chat_prefix == (tok.token_to_id("<|begin_of_text|>"),) and e.tokenizer.chat_suffix == ()
    assert e.encode_prompt("kernel")[0] == tok.token_to_id("<|begin_of_text|>")


def test_serve_checkpoint_dir_uses_its_template(tmp_path):
    """`roundtable serve --weights <checkpoint>`: architecture from config.json, conversation
    rendered by the checkpoint's chat template (all messages, one generation prompt)."""
    import urllib.request
    from theroundtaible_amd.serve import build_server
    tok, V = _checkpoint(tmp_path)
    srv = build_server("llama3-8b", weights=str(tmp_path), device="cpu", port=0, max_batch=2, max_tokens=6,
                       num_blocks=64).start()
    try:
        msgs = [{"role": "system", "content": "Wees kort."}, {"role": "user", "content": "Wat zegt de koning?"}]
        req = urllib.request.Request(srv.url + "/v1/chat/completions", method="POST",
                                     data=json.dumps({"messages": msgs, "max_tokens": 4, "ignore_eos": True}).encode(),
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            d = json.loads(r.read().decode())
        rendered = ("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\nWees kort.<|eot_id|>"
                    "<|start_header_id|>user<|end_header_id|>\n\nWat zegt de koning?<|eot_id|>"
                    "<|start_header_id|>assistant<|end_header_id|>\n\n")
        assert d["usage"]["prompt_tokens"] == len(tok.encode(rendered).ids)
        assert d["usage"]["completion_tokens"] == 4
    finally:
        srv.close()


def test_knight_on_checkpoint_dir_without_overrides(tmp_path):
    """A config seat that only names the checkpoint directory: preset + shape come from config.json."""
    from theroundtaible_amd.knights.registry import BackendFactory
    from theroundtaible_amd.types import RoundtableConfig
    (tmp_path / "ckpt").mkdir()
    tok, V = _checkpoint(tmp_path / "ckpt")
    cfg = RoundtableConfig.from_dict({
        "version": "1.0", "project": "t", "knights": [{"name": "Local", "adapter": "local-llm-ckpt",
                                                       "capabilities": [], "priority": 1}],
        "rules": {}, "chronicle": ".roundtable/chronicle.md",
        "adapter_config": {"local-llm-ckpt": {"engine": {"model": "llama3-8b", "weights": str(tmp_path / "ckpt"),
                                                         "device": "cpu", "max_new_tokens": 3}}}})
    b = BackendFactory(cfg).create("local-llm-ckpt")
    assert b.engine.cfg.vocab == V and b.engine.cfg.hidden == 256
    res = b.execute("De koning spreekt.", 60.0, seq_key="Local")
    assert isinstance(res.text, str) and len(res.ids) == 3


QWEN_SPECIAL = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]
CHATML_TEMPLATE = (   # Qwen2.5's ChatML with its default system turn (trimmed to the parts a turn uses)
    "{%- if messages[0]['role'] != 'system' %}{{- '<|im_start|>system\\nYou are Qwen, created by Alibaba Cloud. "
    "You are a helpful assistant.<|im_end|>\\n' }}{%- endif %}{%- for message in messages %}"
    "{{- '<|im_start|>' + message['role'] + '\\n' + message['content'] + '<|im_end|>' + '\\n' }}{%- endfor %}"
    "{%- if add_generation_prompt %}{{- '<|im_start|>assistant\\n' }}{%- endif %}")


def test_qwen_chatml_checkpoint(tmp_path):
    """A Qwen2.5-style checkpoint: ChatML template with its default system turn, no BOS, stops at
    <|im_end|> and <|endoftext|>; the architecture (q/k/v biases, tied head) comes from config.json."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from theroundtaible_amd.utils.local_detect import resolve_model
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    corpus = ["You are Qwen, created by Alibaba Cloud. You are a helpful assistant.",
              "De ridders van de ronde tafel bespreken de kernel en de cache."] * 20
    tok.train_from_iterator(corpus, trainers.BpeTrainer(vocab_size=400, special_tokens=QWEN_SPECIAL,
                                                        initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    tok.save(str(tmp_path / "tokenizer.json"))
    V = tok.get_vocab_size()
    end, ims, ime = (tok.token_to_id(s) for s in QWEN_SPECIAL)
    torch.manual_seed(0)
    m = transformers.Qwen2ForCausalLM(transformers.Qwen2Config(
        hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
        vocab_size=V, max_position_embeddings=4096, rope_theta=1e6, rms_norm_eps=1e-6, tie_word_embeddings=True,
        bos_token_id=end, eos_token_id=ime, use_sliding_window=False))
    m.save_pretrained(str(tmp_path), safe_serialization=True)
    (tmp_path / "tokenizer_config.json").write_text(json.dumps({"bos_token": None, "eos_token": "<|im_end|>",
                                                                "chat_template": CHATML_TEMPLATE}))
    (tmp_path / "generation_config.json").write_text(json.dumps({"bos_token_id": end, "eos_token_id": [ime, end]}))
    model, ov = resolve_model("tiny-llama", str(tmp_path))
    assert ov.get("qkv_bias", True) and ov.get("vocab") == V
    e = Engine(EngineConfig(model=model, weights=str(tmp_path), device="cpu", dtype="fp32", num_blocks=64,
                            model_overrides=ov))
    assert e.cfg.qkv_bias and e.cfg.tie_embeddings and e.tokenizer.stop_ids == {ime, end}
    text = "De ridders bespreken de cache."
    want = tok.encode("<|im_start|>system\nYou are Qwen, created by Alibaba Cloud. You are a helpful assistant."
                      "<|im_end|>\n<|im_start|>user\n" + text + "<|im_end|>\n<|im_start|>assistant\n").ids
    assert e.encode_prompt(text) == want
    sp = SamplingParams(temperature=0.0, max_new_tokens=4, ignore_eos=True, stop_on_consensus=False)
    r = e.run_turns([Turn("K", text, sp)])[0]
    assert r.error is None and len(r.ids) == 4
    with torch.no_grad():    # the engine's greedy tokens are transformers' on the same prompt
        gen = m.generate(torch.tensor([want]), max_new_tokens=4, do_sample=False, pad_token_id=end,
                         eos_token_id=None)[0, len(want):].tolist()
    assert r.ids == gen
