"""Shipped example configs stay valid (reference schema + engine extensions)."""
import glob
import json
import os

import pytest

from theroundtaible_amd.config import engine_settings, validate_config
from theroundtaible_amd.types import RoundtableConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "examples", "*.json"))))
def test_example_configs_validate(path):
    cfg = json.load(open(path))
    validate_config(cfg)
    rc = RoundtableConfig.from_dict(cfg)
    for k in rc.knights:
        st = engine_settings(rc, k.adapter)
        assert st["model"]


def test_shared_scripted_example_carries_script():
    cfg = RoundtableConfig.from_dict(json.load(open(os.path.join(ROOT, "examples", "config.shared-scripted.json"))))
    assert cfg.rules.prompt_layout == "shared"
    st = engine_settings(cfg, "claude-cli")
    assert st["scripted_consensus"]["scores"] == [6, 8, 9]
