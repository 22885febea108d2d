"""theroundtaible_amd — an MI355X-native multi-LLM roundtable engine.

Host side (format-compatible with polatinos/TheRoundtAIble): config, consensus,
sessions/chronicle/manifest/decrees, prompt/context/tools, the round orchestrator
and the CLI. Device side: locally hosted knights (Llama-3 / Mistral / GPT-2) on a
paged-KV engine with hand-written CDNA4 HIP kernels (``csrc/``), hipGraph decode and
RCCL over xGMI for knight placement and tensor parallelism.
"""
__version__ = "0.1.0"
REFERENCE_VERSION = "0.5.1"
