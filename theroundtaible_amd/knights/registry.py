"""Adapter-id -> backend factory and bring-up (`src/utils/adapters.ts:15-106`).

Reference semantics kept: the backend map is keyed by *adapter id* (two knights on
one adapter share a backend); an unavailable primary with an available fallback is
stored under the primary's key. Unknown adapter ids are reported and skipped.
Seats configured with ``backend: "external"`` (or reference-shaped ``local-llm`` entries
with an ``endpoint``) use the reference's transports (:mod:`.external`).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

from ..config import engine_settings
from ..engine.engine import EngineConfig
from ..engine.sampler import SamplingParams
from ..types import RoundtableConfig
from ..utils.local_detect import resolve_model
from ..utils.ui import NULL_UI, UI
from .base import KnightBackend
from .engine_backend import ADAPTER_DISPLAY_NAMES, EngineBackend, EnginePool
from .external import create_external, wants_external
from .script import ConsensusScript
from .fake import FakeBackend

KNOWN_PREFIXES = ("claude-", "gemini-", "openai-", "local-llm", "engine", "fake")


def _device_count() -> int:
    try:
        import torch
        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:  # noqa: BLE001
        return 0


def display_name(adapter_id: str, config: RoundtableConfig) -> str:
    ac = config.adapter_config.get(adapter_id) or {}
    if isinstance(ac, dict) and ac.get("name"):
        return str(ac["name"])
    return ADAPTER_DISPLAY_NAMES.get(adapter_id, adapter_id)


class BackendFactory:
    def __init__(self, config: RoundtableConfig, pool: Optional[EnginePool] = None,
                 device_override: Optional[str] = None):
        self.config = config
        self.pool = pool or EnginePool()
        self.device_override = device_override
        self._auto_next = 0
        self._auto: Dict[str, str] = {}
        self.defer_kv = False    # initialize_backends: KV pools sized after every engine's weights load

    def _device_for(self, adapter_id: str, st: dict) -> str:
        if self.device_override:
            return self.device_override
        if st.get("device") and st["device"] != "auto":
            return str(st["device"])
        gpus = st.get("gpus")
        if isinstance(gpus, list) and gpus:
            return f"cuda:{int(gpus[0])}"
        n = _device_count()
        if n == 0:
            return "cpu"
        key = st.get("model", "")
        if adapter_id not in self._auto:
            self._auto[adapter_id] = f"cuda:{self._auto_next % n}"
            self._auto_next += 1
        return self._auto[adapter_id]

    def create(self, adapter_id: str) -> Optional[KnightBackend]:
        if not adapter_id or not adapter_id.startswith(KNOWN_PREFIXES):
            return None
        st = engine_settings(self.config, adapter_id)
        name = display_name(adapter_id, self.config)
        if st.get("backend") == "fake" or adapter_id.startswith("fake"):
            return FakeBackend(name=name, adapter_id=adapter_id)
        ac = self.config.adapter_config.get(adapter_id) or {}
        if isinstance(ac, dict) and wants_external(adapter_id, ac):
            return create_external(adapter_id, ac, name)
        tp = int(st.get("tp", 1) or 1)
        if tp > 1:
            # never silently run a tensor-parallel knight at tp = 1 on its first GPU: the CLI
            # launches the ranks itself (parallel/launch.py); anything else must run under torchrun
            from ..errors import ConfigError
            raise ConfigError(f"{adapter_id}: engine.tp={tp} needs one process per GPU of its group",
                              hint="Run it through `roundtable discuss/summon/apply/code-red` (they launch the "
                                   "ranks), or under `torchrun --nproc-per-node N -m theroundtaible_amd ...`.")
        weights = str(st.get("weights", "random:0"))
        model, overrides = resolve_model(st["model"], weights, st.get("model_overrides"))
        ecfg = EngineConfig(model=model, weights=weights,
                            dtype=str(st.get("dtype", "bf16")), device=self._device_for(adapter_id, st),
                            block_size=int(st.get("kv_block_size", 32)),
                            kv_cache_fraction=float(st.get("kv_cache_fraction", 0.85)),
                            max_kv_tokens=st.get("max_kv_tokens"),
                            use_graphs=bool(st.get("use_graphs", True)),
                            model_overrides=overrides)
        if ecfg.device == "cpu":
            ecfg.dtype = "fp32" if st.get("dtype") in (None, "bf16") and st.get("cpu_fp32", True) else ecfg.dtype
            ecfg.use_graphs = False
        engine, lock = self.pool.get(ecfg, defer_kv=self.defer_kv)
        params = SamplingParams(temperature=float(st.get("temperature", 0.7)), top_p=float(st.get("top_p", 0.95)),
                                top_k=int(st.get("top_k", 0)), seed=int(st.get("seed", 0)),
                                max_new_tokens=int(st.get("max_new_tokens", 512)),
                                ignore_eos=bool(st.get("ignore_eos", False)),
                                stop_on_consensus=bool(st.get("stop_on_consensus", True)))
        return EngineBackend(name, adapter_id, engine, params, lock,
                             script=ConsensusScript.from_config(st.get("scripted_consensus")))

    __call__ = create


def initialize_backends(config: RoundtableConfig, ui: UI = NULL_UI,
                        factory: Optional[BackendFactory] = None) -> Dict[str, KnightBackend]:
    factory = factory or BackendFactory(config)
    factory.defer_kv = True
    out: Dict[str, KnightBackend] = {}
    for knight in config.knights:
        if knight.adapter in out:
            continue
        try:
            primary = factory.create(knight.adapter)
        except Exception as e:  # noqa: BLE001 - a knight whose model cannot load is absent
            ui.warn(f"  ✗ {knight.name}: {knight.adapter} failed to start ({e})")
            primary = None
            if not knight.fallback:
                continue
        if primary is None and not knight.fallback:
            ui.warn(f'  ? {knight.name}: unknown adapter "{knight.adapter}"')
            continue
        if primary is not None and primary.is_available():
            out[knight.adapter] = primary
            ui.ok(f"  ✓ {knight.name} ready ({knight.adapter})")
            continue
        if knight.fallback:
            ui.dim(f"  {knight.name}: {knight.adapter} unavailable, trying fallback...")
            try:
                fb = factory.create(knight.fallback)
            except Exception:  # noqa: BLE001
                fb = None
            if fb is not None and fb.is_available():
                out[knight.adapter] = fb
                ui.ok(f"  ✓ {knight.name} ready (fallback: {knight.fallback})")
                continue
        ui.warn(f"  ✗ {knight.name} not available")
    # every engine's weights are resident: split each GPU's free HBM between its engines' KV pools
    factory.pool.finalize()
    factory.defer_kv = False     # engines created later (runtime fallbacks) size their pool at once
    return out
