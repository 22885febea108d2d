"""Train the bundled byte-level BPE tokenizer (offline; no downloads).

There is no network, so the real Llama-3 / Mistral / GPT-2 vocabularies are not
available. The engine ships one deterministic 32K byte-level BPE trained on local
text (CPython's stdlib sources + this repo's Dutch prompt template). Model vocab
sizes stay the real ones (128256 / 32000 / 50257): ids >= the tokenizer's size are
decoded through a byte fallback so random-init models always produce valid text.
"""
import glob
import os
import sys

from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..",
                                                          "theroundtaible_amd", "assets", "bpe32k.json")
files = sorted(glob.glob("/usr/lib/python3.10/**/*.py", recursive=True))[:1500]
files.append(os.path.join(os.path.dirname(__file__), "..", "theroundtaible_amd", "templates", "system-prompt.md"))
tok = Tokenizer(models.BPE())
tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
tok.decoder = decoders.ByteLevel()
trainer = trainers.BpeTrainer(vocab_size=32000, min_frequency=2, show_progress=False,
                              special_tokens=["<|begin_of_text|>", "<|end_of_text|>", "<|pad|>"],
                              initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
tok.train(files, trainer)
tok.save(out)
print("saved", out, tok.get_vocab_size())
