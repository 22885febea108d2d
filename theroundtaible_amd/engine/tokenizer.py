"""Engine tokenizer.

No network means no Llama-3/Mistral/GPT-2 vocab files, so the engine bundles a
deterministic 32K byte-level BPE (``assets/bpe32k.json``, trained offline by
``tools/train_tokenizer.py``). The *model* keeps its real vocabulary size; ids the
BPE does not know (random-init models sample all of ``[0, vocab)``) are decoded via a
printable byte fallback so every generated id maps to stable text.

Segments are encoded independently (see :mod:`theroundtaible_amd.prompt`) so the
token prefix of a knight's prompt is stable across turns, which is what makes the
resident-KV prefix reuse exact.
"""
from __future__ import annotations

import functools
import os
from typing import Iterable, List, Optional, Sequence

ASSET = os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets", "bpe32k.json")
_PRINTABLE = [chr(c) for c in range(0x20, 0x7F)]


class EngineTokenizer:
    name = "rt-bpe32k"
    chat_prefix = ()          # no chat template: prompts are plain text (random-init benchmarks)
    chat_suffix = ()

    @property
    def stop_ids(self) -> frozenset:
        return frozenset({self.eos_id})

    def __init__(self, model_vocab: int, path: str = ASSET):
        from tokenizers import Tokenizer
        self._tok = Tokenizer.from_file(path)
        self.base_vocab = self._tok.get_vocab_size()
        self.model_vocab = model_vocab
        self.bos_id = self._tok.token_to_id("<|begin_of_text|>")
        self.eos_id = self._tok.token_to_id("<|end_of_text|>")
        # tokenizer family id: token-id sharing across knights requires the same (name, vocab)
        self.family = f"{self.name}/{model_vocab}"

    def encode(self, text: str) -> List[int]:
        if not text:
            return []
        ids = self._tok.encode(text, add_special_tokens=False).ids
        if self.model_vocab < self.base_vocab:
            # a model with a smaller vocab than the BPE (not used by the presets): fold ids
            ids = [i % self.model_vocab for i in ids]
        return ids

    def encode_batch(self, texts: Sequence[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(list(texts), add_special_tokens=False)]

    def decode(self, ids: Iterable[int]) -> str:
        out: List[str] = []
        run: List[int] = []
        for i in ids:
            i = int(i)
            if 0 <= i < self.base_vocab:
                run.append(i)
                continue
            if run:
                out.append(self._tok.decode(run, skip_special_tokens=False))
                run = []
            out.append(_fallback_piece(i))
        if run:
            out.append(self._tok.decode(run, skip_special_tokens=False))
        return "".join(out)


@functools.lru_cache(maxsize=65536)
def _fallback_piece(i: int) -> str:
    # deterministic printable 1-3 char piece for ids outside the BPE
    n = 1 + (i % 3)
    s = []
    x = i
    for _ in range(n):
        s.append(_PRINTABLE[x % len(_PRINTABLE)])
        x //= len(_PRINTABLE)
    return "".join(s)


def _read_json(d: str, name: str) -> dict:
    import json
    p = os.path.join(d, name)
    try:
        with open(p, encoding="utf-8") as f:
            v = json.load(f)
        return v if isinstance(v, dict) else {}
    except (OSError, ValueError):
        return {}


def _token_str(v) -> Optional[str]:
    if isinstance(v, str):
        return v
    if isinstance(v, dict) and isinstance(v.get("content"), str):   # AddedToken serialisation
        return v["content"]
    return None


class HFTokenizer:
    """A checkpoint's own tokenizer (``tokenizer.json``, HF fast format) and chat template.

    Used whenever the engine's ``weights`` is a checkpoint directory that ships one, so a knight
    on real Llama-3 / Mistral weights reads and writes real text. The prompt of every turn is
    wrapped as ONE user message with the checkpoint's chat template (rendered once with a marker
    and split into constant prefix / suffix ids), which is exactly how the reference hands each
    knight its whole prompt (`src/adapters/local-llm.ts:112-122`: a single user message) and keeps
    the append layout's KV reuse: only the few suffix tokens plus the new content are re-prefilled.
    Generation stops at any of the checkpoint's end ids (``generation_config.json`` /
    ``config.json`` ``eos_token_id`` + the tokenizer's eos token, e.g. Llama-3's ``<|eot_id|>``).
    Only JSON / the tokenizer file are read; nothing in the checkpoint is executed.
    """

    _MARK = "\u0000RT_CONTENT\u0000"

    def __init__(self, path: str, model_vocab: int, chat: bool = True):
        from tokenizers import Tokenizer
        self._tok = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
        self.base_vocab = self._tok.get_vocab_size(with_added_tokens=True)
        self.model_vocab = model_vocab
        tc, gc, mc = (_read_json(path, n) for n in ("tokenizer_config.json", "generation_config.json", "config.json"))
        bos, eos = _token_str(tc.get("bos_token")), _token_str(tc.get("eos_token"))
        self.bos_id = self._tok.token_to_id(bos) if bos else None
        if self.bos_id is None:
            self.bos_id = gc.get("bos_token_id", mc.get("bos_token_id"))
        stops = set()
        for src in (gc.get("eos_token_id"), mc.get("eos_token_id")):
            if isinstance(src, int):
                stops.add(src)
            elif isinstance(src, list):
                stops.update(i for i in src if isinstance(i, int))
        if eos and self._tok.token_to_id(eos) is not None:
            stops.add(self._tok.token_to_id(eos))
        self.stop_ids = frozenset(stops)
        self.eos_id = min(stops) if stops else (self.bos_id if self.bos_id is not None else 0)
        self.name = "hf:" + os.path.basename(os.path.normpath(path))
        self.family = f"{self.name}/{model_vocab}"
        self.chat_prefix, self.chat_suffix = self._chat_wrap(tc, bos, eos) if chat else ((), ())
        if not self.chat_prefix and tc.get("add_bos_token", True) and self.bos_id is not None:
            self.chat_prefix = (int(self.bos_id),)

    def _chat_wrap(self, tc: dict, bos: Optional[str], eos: Optional[str]):
        tmpl = tc.get("chat_template")
        if isinstance(tmpl, list):   # named templates: use "default"
            tmpl = next((t.get("template") for t in tmpl if isinstance(t, dict) and t.get("name") == "default"), None)
        self._template = None
        if not isinstance(tmpl, str):
            return (), ()
        import jinja2
        from jinja2.sandbox import ImmutableSandboxedEnvironment

        def raise_exception(msg):
            raise jinja2.TemplateError(msg)
        env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
        env.globals["raise_exception"] = raise_exception
        try:
            compiled = env.from_string(tmpl)
            text = compiled.render(messages=[{"role": "user", "content": self._MARK}],
                                   add_generation_prompt=True, bos_token=bos or "", eos_token=eos or "")
        except Exception:  # noqa: BLE001 - a template we cannot render: plain prompt
            return (), ()
        self._template = (compiled, bos or "", eos or "")
        if self._MARK not in text:
            return (), ()
        pre, suf = text.split(self._MARK, 1)
        enc = lambda s: tuple(self._tok.encode(s, add_special_tokens=False).ids) if s else ()
        return enc(pre), enc(suf)

    def render_chat(self, messages: List[dict]) -> Optional[str]:
        """A whole conversation through the checkpoint's chat template (ends in an open assistant
        turn); None when the checkpoint has no renderable template."""
        if getattr(self, "_template", None) is None:
            return None
        compiled, bos, eos = self._template
        try:
            return compiled.render(messages=messages, add_generation_prompt=True, bos_token=bos, eos_token=eos)
        except Exception:  # noqa: BLE001 - e.g. a template that rejects this role order
            return None

    def encode(self, text: str) -> List[int]:
        return self._tok.encode(text, add_special_tokens=False).ids if text else []

    def encode_batch(self, texts: Sequence[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(list(texts), add_special_tokens=False)]

    def decode(self, ids: Iterable[int]) -> str:
        out: List[str] = []
        run: List[int] = []
        for i in ids:
            i = int(i)
            if 0 <= i < self.base_vocab:
                run.append(i)
                continue
            if run:
                out.append(self._tok.decode(run, skip_special_tokens=True))
                run = []
            out.append(_fallback_piece(i))
        if run:
            out.append(self._tok.decode(run, skip_special_tokens=True))
        return "".join(out)


def has_checkpoint_tokenizer(weights: Optional[str]) -> bool:
    return bool(weights) and os.path.isdir(weights) and os.path.isfile(os.path.join(weights, "tokenizer.json"))


@functools.lru_cache(maxsize=8)
def get_tokenizer(model_vocab: int, weights: Optional[str] = None, chat: bool = True):
    """The checkpoint's tokenizer when ``weights`` is a directory shipping ``tokenizer.json``,
    else the bundled 32K BPE (random-init benchmarks)."""
    if has_checkpoint_tokenizer(weights):
        return HFTokenizer(weights, model_vocab, chat)
    return EngineTokenizer(model_vocab)
