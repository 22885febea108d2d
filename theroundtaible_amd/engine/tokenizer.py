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


@functools.lru_cache(maxsize=8)
def get_tokenizer(model_vocab: int) -> EngineTokenizer:
    return EngineTokenizer(model_vocab)
