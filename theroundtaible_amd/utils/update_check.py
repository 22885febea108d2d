"""Update notice (`src/utils/update-check.ts:8-51`).

The reference asks the npm registry for the latest version with a 3 s timeout after every
command and swallows every error. MI355X nodes usually have no egress, so the probe is opt-in:
it runs only when ``ROUNDTABLE_UPDATE_URL`` names a JSON endpoint (PyPI-style
``{"info": {"version": ...}}`` or npm-style ``{"version": ...}``).
"""
from __future__ import annotations

import os
import re
from typing import Callable, Optional, Tuple

from .. import __version__


def _parts(v: str) -> Tuple[int, ...]:
    return tuple(int(x) for x in re.findall(r"\d+", v.split("-")[0])[:3]) or (0,)


def is_newer(latest: str, current: str) -> bool:
    """Numeric major.minor.patch comparison (update-check.ts:42-51)."""
    a, b = _parts(latest), _parts(current)
    n = max(len(a), len(b))
    return a + (0,) * (n - len(a)) > b + (0,) * (n - len(b))


def check_for_update(url: Optional[str] = None, current: str = __version__, timeout_s: float = 3.0,
                     http: Optional[Callable] = None) -> Optional[str]:
    """The newer version string, or None (no URL configured, offline, malformed, up to date)."""
    url = url or os.environ.get("ROUNDTABLE_UPDATE_URL")
    if not url:
        return None
    try:
        from ..knights.external import http_request
        r = (http or http_request)("GET", url, None, {}, timeout_s)
        if not r.ok:
            return None
        d = r.json()
        latest = (d.get("info") or {}).get("version") or d.get("version")
        return latest if isinstance(latest, str) and is_newer(latest, current) else None
    except Exception:  # noqa: BLE001 - never fail a command over an update notice
        return None
