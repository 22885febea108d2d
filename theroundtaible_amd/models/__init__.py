"""Model families: Llama-3 (8B/70B), Mistral-7B, GPT-2-small (+ tiny test presets)."""
from .config import ModelConfig, PRESETS, get_config
from .gpt2 import build_model
