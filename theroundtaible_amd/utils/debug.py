"""Debug run mode: ``ROUNDTABLE_DEBUG=1``.

Turns on, before the first HIP call of the process:

* ``AMD_SERIALIZE_KERNEL=3`` / ``AMD_SERIALIZE_COPY=3`` — the ROCm runtime waits for every kernel and
  copy before and after it is issued, so a fault is reported at the launch that caused it;
* ``HIP_LAUNCH_BLOCKING=1`` — synchronous launches (errors surface at the Python call site);
* ``ROUNDTABLE_DEBUG_CHECKS=1`` — host bounds asserts on paging metadata before every forward
  plus the device-side paging guard inside captured decode graphs (csrc/decode_step.hip).

Values already present in the environment win. GPU AddressSanitizer (xnack+) is not available
on the MI355X pool; the host side of csrc/ is sanitizer-tested instead
(tests/test_native_host_sanitizers.py).
"""
from __future__ import annotations

import os
import warnings
from typing import MutableMapping, Optional

DEBUG_ENV = {
    "AMD_SERIALIZE_KERNEL": "3",
    "AMD_SERIALIZE_COPY": "3",
    "HIP_LAUNCH_BLOCKING": "1",
    "ROUNDTABLE_DEBUG_CHECKS": "1",
}


def apply_debug_env(environ: Optional[MutableMapping[str, str]] = None) -> bool:
    """Apply the debug settings when ROUNDTABLE_DEBUG=1; returns whether debug mode is on."""
    env = os.environ if environ is None else environ
    if env.get("ROUNDTABLE_DEBUG", "") not in ("1", "true", "yes"):
        return False
    for k, v in DEBUG_ENV.items():
        env.setdefault(k, v)
    if environ is None:
        try:
            import torch
            if torch.cuda.is_initialized():
                warnings.warn("ROUNDTABLE_DEBUG set after the GPU runtime started: kernel serialisation "
                              "takes effect only for new processes")
        except Exception:  # noqa: BLE001 - torch missing / not built with ROCm
            pass
    return True
