"""Key store ``~/.theroundtaible/keys.json`` (`src/utils/keys.ts:11-69`).

Local engine knights need no keys; this exists so configs that name ``*-api``
fallbacks keep working and ``init`` can record them with the same 0600/0700 modes.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

from ..utils.atomic import atomic_write_text, read_text


def keys_dir() -> str:
    return os.path.join(os.path.expanduser("~"), ".theroundtaible")


def keys_path() -> str:
    return os.path.join(keys_dir(), "keys.json")


def load_keys() -> Dict[str, str]:
    p = keys_path()
    if not os.path.exists(p):
        return {}
    try:
        d = json.loads(read_text(p))
        return d if isinstance(d, dict) else {}
    except (OSError, ValueError):
        return {}


def save_key(name: str, value: str) -> None:
    os.makedirs(keys_dir(), exist_ok=True)
    keys = load_keys()
    keys[name] = value
    atomic_write_text(keys_path(), json.dumps(keys, indent=2))
    try:
        os.chmod(keys_path(), 0o600)
        os.chmod(keys_dir(), 0o700)
    except OSError:
        pass


def get_key(env_var: str) -> Optional[str]:
    v = os.environ.get(env_var)
    if v:
        return v
    return load_keys().get(env_var) or None
