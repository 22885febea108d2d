"""Numerical parity with Hugging Face ``transformers`` on real checkpoint files.

A tiny Llama / Mistral / GPT-2 is random-initialised *in transformers*, written with
``save_pretrained`` (safetensors), loaded by our engine through ``models/weights.py`` (HF names,
fused qkv / gate_up, Conv1D transposes) and compared against transformers' own forward: full
prefill logits, chunked prefill over the paged prefix, and token-by-token greedy decode. This pins
the conventions a user switching with real weights depends on (RoPE pairing and theta, GQA
grouping, norm placement, tied embeddings, GELU variant). CPU tests run fp32 on the reference ops;
the GPU test runs the bf16 HIP kernels (fused decode path, hipGraphs) against transformers fp32.
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn  # noqa: E402
from theroundtaible_amd.models.config import get_config  # noqa: E402


def _sharpen(m, gain=4.0):
    """Scale q / k projections so attention is peaked: with the default init the scores are
    nearly uniform and a wrong RoPE (theta, scaling) would still match to 2e-4."""
    with torch.no_grad():
        for layer in m.model.layers:
            layer.self_attn.q_proj.weight.mul_(gain)
            layer.self_attn.k_proj.weight.mul_(gain)


def _save_llama(path, mistral=False, big=False, seed=0, rope_scaling=None, sharp=True):
    kw = dict(hidden_size=512 if big else 256, intermediate_size=1024 if big else 512, num_hidden_layers=2,
              num_attention_heads=4, num_key_value_heads=1 if big else 2, vocab_size=32000,
              max_position_embeddings=8192 if big else 4096, rms_norm_eps=1e-5, tie_word_embeddings=False,
              initializer_range=0.08)
    torch.manual_seed(seed)
    if mistral:
        cfg = transformers.MistralConfig(rope_theta=1e6, sliding_window=None, **kw)
        m = transformers.MistralForCausalLM(cfg)
    else:
        cfg = transformers.LlamaConfig(rope_theta=500000.0 if big else 10000.0, rope_scaling=rope_scaling, **kw)
        m = transformers.LlamaForCausalLM(cfg)
    if sharp and not big:
        _sharpen(m)
    m.eval().save_pretrained(str(path), safe_serialization=True)
    return m


def _save_qwen2(path, big=False, seed=0, rope_scaling=None):
    """Qwen2 (Qwen2.5 / Qwen2.5-Coder): the Llama block with q/k/v biases; the small config ties
    the embeddings (as Qwen2.5-0.5B does) and uses head_dim 64 with 2 KV heads."""
    kw = dict(hidden_size=512 if big else 256, intermediate_size=1024 if big else 512, num_hidden_layers=2,
              num_attention_heads=4, num_key_value_heads=1 if big else 2, vocab_size=32000,
              max_position_embeddings=8192 if big else 4096, rms_norm_eps=1e-6, rope_theta=1e6,
              tie_word_embeddings=not big, initializer_range=0.08, use_sliding_window=False,
              rope_scaling=rope_scaling)
    torch.manual_seed(seed)
    m = transformers.Qwen2ForCausalLM(transformers.Qwen2Config(**kw))
    if not big:
        _sharpen(m)
    with torch.no_grad():   # HF initialises the biases to zero: make them matter
        for layer in m.model.layers:
            for lin in (layer.self_attn.q_proj, layer.self_attn.k_proj, layer.self_attn.v_proj):
                lin.bias.normal_(0.0, 0.5)
    m.eval().save_pretrained(str(path), safe_serialization=True)
    return m


def _save_gpt2(path, seed=0):
    cfg = transformers.GPT2Config(n_embd=128, n_layer=2, n_head=2, n_inner=512, vocab_size=32000, n_positions=2048,
                                  layer_norm_epsilon=1e-5, activation_function="gelu_new", initializer_range=0.08,
                                  resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    torch.manual_seed(seed)
    m = transformers.GPT2LMHeadModel(cfg).eval()
    m.save_pretrained(str(path), safe_serialization=True)
    return m


def _ids(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(5, 31000, (n,), generator=g).tolist()


def _check_cpu(engine_model, hf, path, overrides=None):
    if overrides is None:   # the architecture from config.json, as the knights / serve resolve it
        from theroundtaible_amd.utils.local_detect import resolve_model
        engine_model, overrides = resolve_model(engine_model, str(path))
    e = Engine(EngineConfig(model=engine_model, weights=str(path), device="cpu", dtype="fp32", num_blocks=64,
                            model_overrides=dict(overrides)))
    ids = _ids(97)
    with torch.no_grad():
        ref = hf(torch.tensor([ids])).logits[0].float()
    got = e.prefill([(e.kv.seq("a"), ids)])[0]
    assert torch.allclose(got, ref[-1], atol=2e-4, rtol=1e-3), float((got - ref[-1]).abs().max())
    # chunked prefill: the second chunk attends over the paged prefix
    s = e.kv.seq("b")
    e.prefill([(s, ids[:61])])
    got2 = e.prefill([(s, ids[61:])])[0]
    assert torch.allclose(got2, ref[-1], atol=2e-4, rtol=1e-3)
    # greedy, one token at a time, against transformers' greedy generate
    with torch.no_grad():
        gen = hf.generate(torch.tensor([ids]), max_new_tokens=8, do_sample=False, pad_token_id=0)[0, len(ids):].tolist()
    ours, logits = [], got
    for _ in range(8):
        t = int(torch.argmax(logits))
        ours.append(t)
        logits = e.prefill([(e.kv.seq("a"), [t])])[0]
    assert ours == gen


def test_llama_matches_transformers(tmp_path):
    _check_cpu("tiny-llama", _save_llama(tmp_path), tmp_path)


def test_mistral_matches_transformers(tmp_path):
    _check_cpu("tiny-llama", _save_llama(tmp_path, mistral=True), tmp_path)


def test_llama31_rope_scaling_matches_transformers(tmp_path):
    """Llama 3.1 / 3.2 checkpoints carry rope_type "llama3" (long wavelengths divided by the
    factor, a smooth band between): read from config.json and folded into the RoPE table."""
    rs = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
          "original_max_position_embeddings": 64}
    _check_cpu("tiny-llama", _save_llama(tmp_path, rope_scaling=rs), tmp_path)


def test_qwen2_yarn_rope_scaling_matches_transformers(tmp_path):
    """Qwen2.5's long-context YaRN setting: blended frequencies and scaled cos / sin."""
    rs = {"rope_type": "yarn", "factor": 4.0, "original_max_position_embeddings": 64}
    _check_cpu("tiny-qwen", _save_qwen2(tmp_path, rope_scaling=rs), tmp_path)


def test_wrong_rope_is_detected(tmp_path):
    """The parity check is sensitive to RoPE: the same checkpoint with a different theta fails."""
    hf = _save_llama(tmp_path, mistral=True)
    with pytest.raises(AssertionError):
        _check_cpu("tiny-llama", hf, tmp_path, {"rope_theta": 10000.0})


def test_qwen2_matches_transformers(tmp_path):
    """q/k/v biases before RoPE, tied embeddings (the lm_head is the embedding), theta 1e6."""
    from theroundtaible_amd.utils.local_detect import checkpoint_model
    hf = _save_qwen2(tmp_path)
    preset, ov = checkpoint_model(str(tmp_path))      # config.json alone maps it to the Qwen family
    assert preset is not None and get_config(preset, **ov).qkv_bias
    _check_cpu("tiny-qwen", hf, tmp_path)


def test_gpt2_matches_transformers(tmp_path):
    _check_cpu("tiny-gpt2", _save_gpt2(tmp_path), tmp_path)


def _check_gpu(engine_model, hf, path):
    hf = hf.float()
    e = Engine(EngineConfig(model=engine_model, weights=str(path), device="cuda", num_blocks=256))
    ids = _ids(300, seed=3)
    with torch.no_grad():
        ref = hf(torch.tensor([ids])).logits[0, -1].float()
        gen = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False, pad_token_id=0)[0, len(ids):].tolist()
    got = e.prefill([(e.kv.seq("p"), ids)])[0].float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=0)
    assert float(cos) > 0.999, float(cos)
    # the decode loop proper (captured graphs): a Turn whose prompt tokenizes to `ids`
    text = e.tokenizer.decode(ids)
    sp = SamplingParams(temperature=0.0, max_new_tokens=6, ignore_eos=True, stop_on_consensus=False)
    out = e.run_turns([Turn("K", text, sp)])[0]
    prompt_ids = e.encode_prompt(text)
    with torch.no_grad():
        gen2 = hf.generate(torch.tensor([prompt_ids]), max_new_tokens=6, do_sample=False,
                           pad_token_id=0)[0, len(prompt_ids):].tolist()
    assert out.ids[:3] == gen2[:3], (out.ids, gen2)
    assert gen[:1] == [int(torch.argmax(got))]


@pytest.mark.gpu
def test_llama_gpu_kernels_match_transformers(tmp_path):
    """bf16 HIP path (prefill kernels, fused decode GEMMs + paged decode attention in hipGraphs)."""
    _check_gpu("tiny-llama-128", _save_llama(tmp_path, big=True), tmp_path)


@pytest.mark.gpu
def test_qwen2_gpu_kernels_match_transformers(tmp_path):
    """Qwen2 on the HIP path: the q/k/v bias rides in the fused qkv GEMM's RoPE epilogue."""
    _check_gpu("tiny-qwen-128", _save_qwen2(tmp_path, big=True), tmp_path)
