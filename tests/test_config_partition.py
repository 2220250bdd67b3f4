"""Config/schema compatibility and partitioner parity with the reference.

Fixtures ``tests/fixtures/{config_sample,example_inputs_sample}.json`` are the reference's own
sample files (/root/reference/config/...)."""
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from docker_dist_nn_amd.config import load_model_config, model_config_from_dict
from docker_dist_nn_amd.data import load_examples
from docker_dist_nn_amd.models import MLPSpec, NAMED_MODELS
from docker_dist_nn_amd.partition import (balanced_distribution, calculate_layer_mappings,
                                          plan_stages)
from docker_dist_nn_amd.weights_io import export_model_json, stage_files_from_model

FIX = os.path.join(os.path.dirname(__file__), "fixtures")
SAMPLE = os.path.join(FIX, "config_sample.json")
INPUTS = os.path.join(FIX, "example_inputs_sample.json")


def test_sample_config_loads_and_fails_dim_check_like_reference():
    mc = load_model_config(SAMPLE)
    assert [L.out_dim for L in mc.layers] == [3, 6, 2]
    assert [L.in_dim for L in mc.layers] == [2, 2, 3]
    assert mc.layer_distribution is None and mc.distribution == [1]
    with pytest.raises(ValueError, match="expected input dim 3, got 2"):
        mc.spec()


def test_reference_mappings_parity():
    """E2: [1,1,1] -> ports 5101/5201/5301, expected_input 3/3/6; [1,0,2] skips stage 1."""
    mc = load_model_config(SAMPLE)
    ex = json.load(open(INPUTS))["examples"]
    m = calculate_layer_mappings(mc.layer_dicts(), [1, 1, 1], ex)
    assert [m[i]["listen_port"] for i in range(3)] == [5101, 5201, 5301]
    assert [m[i]["expected_input"] for i in range(3)] == [3, 3, 6]
    assert [m[i]["container_name"] for i in range(3)] == [
        "layer_container_0", "layer_container_1", "layer_container_2"]
    assert m[0]["next_nodes"] == [{"host": "layer_container_1", "port": "5201"}]
    assert m[2]["next_nodes"] == []
    assert list(m[0]["neurons_config"]) == ["layer_1"]
    m2 = calculate_layer_mappings(mc.layer_dicts(), [1, 0, 2], ex)
    assert sorted(m2) == [0, 2]
    assert m2[0]["next_nodes"] == [{"host": "layer_container_2", "port": "5301"}]
    assert list(m2[2]["neurons_config"]) == ["layer_1", "layer_2"]
    with pytest.raises(ValueError, match="Sum of layer_distribution"):
        calculate_layer_mappings(mc.layer_dicts(), [1, 1], ex)


def test_plan_stages_handles_leading_zero():
    plans = plan_stages(3, [0, 2, 1])
    assert [(p.stage, p.container, p.layer_start, p.layer_end) for p in plans] == [
        (0, 1, 0, 2), (1, 2, 2, 3)]
    assert plans[0].port == 5201


def test_wrapped_notebook_form_and_stage_file(tmp_path):
    rng = np.random.default_rng(0)
    ws = [rng.standard_normal((5, 4)), rng.standard_normal((3, 5))]
    bs = [rng.standard_normal(5), rng.standard_normal(3)]
    p = tmp_path / "m.json"
    export_model_json(str(p), ws, bs, ["relu", "softmax"], wrapped=True,
                      inference_metrics={"accuracy": 0.5})
    mc = load_model_config(str(p))
    assert mc.wrapped and mc.inference_metrics == {"accuracy": 0.5}
    np.testing.assert_allclose(mc.layers[1].weight, ws[1])
    spec = mc.spec()
    assert spec.widths == [4, 5, 3] and spec.layers[1].activation == "softmax"
    envs = stage_files_from_model(mc, str(tmp_path / "cache"), 4, [1, 1])
    assert "NEURONS_FILE_CONFIG" in envs[0] or "NEURONS_CONFIG" in envs[0]
    f = tmp_path / "cache" / "layer_container_1_neurons_config.json"
    if f.exists():
        st_cfg = load_model_config(str(f))
        assert st_cfg.stage_file and st_cfg.layers[0].out_dim == 3


def test_native_parser_matches_python(tmp_path):
    rng = np.random.default_rng(1)
    ws = [rng.standard_normal((16, 8)).astype(np.float32), rng.standard_normal((4, 16)).astype(np.float32)]
    bs = [rng.standard_normal(16).astype(np.float32), rng.standard_normal(4).astype(np.float32)]
    p = tmp_path / "m.json"
    export_model_json(str(p), ws, bs, ["relu", "softmax"], layer_distribution=[1, 1])
    a = load_model_config(str(p), native_parser=False)
    b = load_model_config(str(p), native_parser=True)
    assert a.layer_distribution == b.layer_distribution == [1, 1]
    for la, lb in zip(a.layers, b.layers):
        np.testing.assert_array_equal(la.weight.astype(np.float32), lb.weight)
        np.testing.assert_array_equal(la.bias.astype(np.float32), lb.bias)
        assert la.activation == lb.activation
    # native writer round-trips fp32 exactly
    from docker_dist_nn_amd.utils.native import native
    q = tmp_path / "n.json"
    native().write_neuron_json(str(q), ws, bs, ["relu", "softmax"], ["hidden", "output"], [2], False)
    c = load_model_config(str(q), native_parser=False)
    np.testing.assert_array_equal(c.layers[0].weight.astype(np.float32), ws[0])
    assert c.layer_distribution == [2]
    s = tmp_path / "s.json"
    native().write_neuron_json(str(s), ws, bs, ["relu", "softmax"], ["hidden", "output"], [], True)
    d = load_model_config(str(s), native_parser=True)
    assert d.stage_file and len(d.layers) == 2


def test_examples_loaders(tmp_path):
    e = load_examples(INPUTS)
    assert len(e) == 3 and e.dim == 6 and e.outer_len == 3
    assert list(e.labels) == [5, 2, 8]
    en = load_examples(INPUTS, native_parser=True)
    np.testing.assert_array_equal(e.x, en.x)
    raw = tmp_path / "raw.json"
    raw.write_text(json.dumps({"examples": [[0.1, 0.2], [0.3, 0.4]]}))
    r = load_examples(str(raw))
    assert r.raw_list and list(r.labels) == [-1, -1]
    rn = load_examples(str(raw), native_parser=True)
    assert rn.raw_list and np.allclose(rn.x, r.x)


def test_mixed_activation_warns():
    cfg = {"layers": [{"type": "hidden", "nodes": 2, "neurons": [
        {"weights": [1.0], "bias": 0.0, "activation": "relu"},
        {"weights": [2.0], "bias": 0.0, "activation": "sigmoid"}]}]}
    with pytest.warns(UserWarning, match="different activations"):
        mc = model_config_from_dict(cfg)
    assert mc.layers[0].activation == "relu"


def test_model_spec_parsing():
    assert MLPSpec.parse("784-1024x7-10").widths == [784] + [1024] * 7 + [10]
    assert len(NAMED_MODELS["mlp8"].layers) == 8
    assert NAMED_MODELS["mnist-fcnn"].widths == [784, 512, 256, 128, 10]
    assert NAMED_MODELS["mnist-fcnn"].layers[-1].activation == "softmax"


@settings(max_examples=60, deadline=None)
@given(st.lists(st.floats(0.1, 100.0), min_size=1, max_size=10), st.data())
def test_balanced_distribution_is_optimal(costs, data):
    S = data.draw(st.integers(1, len(costs)))
    d = balanced_distribution(costs, S)
    assert len(d) == S and all(k >= 1 for k in d) and sum(d) == len(costs)
    def worst(dd):
        g, m = 0, 0.0
        for k in dd:
            m = max(m, sum(costs[g:g + k]))
            g += k
        return m
    # brute force over all compositions for small cases
    if len(costs) <= 7:
        import itertools
        best = min(worst([b - a for a, b in zip((0,) + c, c + (len(costs),))])
                   for c in itertools.combinations(range(1, len(costs)), S - 1))
        assert worst(d) <= best + 1e-9
