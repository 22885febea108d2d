"""MI355X inference engine: paged resident KV, chunked prefill, hipGraph decode, sampling."""
from .engine import Engine, EngineConfig, Turn, TurnOutput
from .sampler import SamplingParams
