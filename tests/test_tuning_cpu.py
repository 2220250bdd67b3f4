"""Override tables (ops/tuning.py): an experiment table lists only what it changes."""
import json

from docker_dist_nn_amd.ops import tuning


def test_override_table_applies_over_default(tmp_path):
    base = tuning.load_table(tuning.DEFAULT_PATH)
    k_change, k_drop = sorted(base)[:2]
    p = tmp_path / "ov.json"
    p.write_text(json.dumps({"base": "default", "override": {
        k_change: {"tile": [64, 64], "splits": 3, "stages": 2}, k_drop: None,
        "fwd:8x8x8": {"tile": [64, 64], "splits": 1, "stages": 2}}}))
    t = tuning.load_table(str(p))
    assert t[k_change]["splits"] == 3 and k_drop not in t and "fwd:8x8x8" in t
    assert all(t[k] == base[k] for k in base if k not in (k_change, k_drop))
