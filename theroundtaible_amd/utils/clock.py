"""Time helpers producing the reference's JS ``Date.toISOString()`` formats."""
from __future__ import annotations

import datetime as _dt
import os


def _now() -> _dt.datetime:
    # ROUNDTABLE_FAKE_NOW (ISO string) pins the clock for golden-file tests.
    fake = os.environ.get("ROUNDTABLE_FAKE_NOW")
    if fake:
        return _dt.datetime.fromisoformat(fake.replace("Z", "+00:00")).astimezone(_dt.timezone.utc)
    return _dt.datetime.now(_dt.timezone.utc)


def iso_now() -> str:
    """``new Date().toISOString()`` -> ``2026-10-15T21:12:03.123Z`` (UTC, millisecond precision)."""
    n = _now()
    return n.strftime("%Y-%m-%dT%H:%M:%S.") + f"{n.microsecond // 1000:03d}Z"


def iso_date() -> str:
    return iso_now()[:10]
