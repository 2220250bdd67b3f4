"""CPU-side contract of the fused classifier tail and the library-GEMM switches: the unfused
reference (ops.reference.mlp_tail) partial grouping, the Stage gating rules, the per-file build
flags, and the DNN_BLAS parser."""
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops import kernels as K
from docker_dist_nn_amd.ops import reference as ref


def test_reference_tail_partials_sum_to_column_sums():
    g = torch.Generator().manual_seed(0)
    rows, k3, n3, n4, nc = 512, 64, 64, 64, 10
    x = torch.relu(torch.randn(rows, k3, generator=g)).to(torch.bfloat16)
    w3 = (torch.randn(n3, k3, generator=g) * 0.1).to(torch.bfloat16)
    w4 = torch.zeros(n4, n3, dtype=torch.bfloat16)
    w4[:nc] = (torch.randn(nc, n3, generator=g) * 0.1).to(torch.bfloat16)
    b3, b4 = torch.zeros(n3), torch.zeros(n4)
    labels = torch.randint(0, nc, (rows,), generator=g, dtype=torch.int32)
    nb = ops.tail_blocks(rows)
    bf = torch.bfloat16
    h3, dz3 = torch.empty(rows, n3, dtype=bf), torch.empty(rows, n3, dtype=bf)
    dz4, dz2 = torch.empty(rows, n4, dtype=bf), torch.empty(rows, k3, dtype=bf)
    loss, corr = torch.zeros(nb), torch.zeros(nb, dtype=torch.int32)
    cs4, cs3, cs2 = torch.zeros(nb, n4), torch.zeros(nb, n3), torch.zeros(nb, k3)
    ops.mlp_tail(x, w3, b3, w4, b4, labels, h3, dz4, dz3, dz2, nc, 1.0 / rows,
                 loss_part=loss, correct=corr, cs4=cs4, cs3=cs3, cs2=cs2)
    torch.testing.assert_close(cs2.sum(0), dz2.float().sum(0), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(cs3.sum(0), dz3.float().sum(0), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(cs4.sum(0), dz4.float().sum(0), rtol=1e-5, atol=1e-6)
    assert int(corr.sum()) <= rows and float(loss.sum()) > 0
    # dz2 is the relu-masked dgrad of dz3 through w3
    want = torch.where(x.float() > 0, dz3.float() @ w3.float(), torch.zeros(rows, k3))
    torch.testing.assert_close(dz2.float(), want, rtol=2e-2, atol=1e-4)


def test_tail_geometry_gate():
    assert ops.tail_supported(256, 128, 64, 10)
    assert ops.tail_supported(64, 64, 128, 16)
    assert not ops.tail_supported(512, 128, 64, 10)  # W3 would not fit in LDS
    assert not ops.tail_supported(256, 256, 64, 10)
    assert not ops.tail_supported(256, 128, 64, 17)  # more classes than one MFMA block


def test_stage_enables_tail_only_on_gpu_last_stage(monkeypatch):
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.engine.stage import Stage

    st = Stage(NAMED_MODELS["mnist-fcnn"], 0, 4, micro_batch=256, num_micro=1,
               device=torch.device("cpu"))
    assert not st.tail  # the fused kernel is a GPU path; CPU runs the unfused reference


def test_build_reads_per_file_flags():
    from docker_dist_nn_amd._build import CSRC, _file_flags

    assert _file_flags(CSRC / "kernels" / "mlp_tail.hip") == ["-fno-slp-vectorize"]
    assert _file_flags(CSRC / "kernels" / "gemm.hip") == []


def test_blas_switch(monkeypatch):
    monkeypatch.delenv("DNN_BLAS", raising=False)
    assert K._blas_requested("fwd", {"blas": 1}) and not K._blas_requested("fwd", {"tile": [64, 64]})
    assert not K._blas_requested("fwd", None)
    monkeypatch.setenv("DNN_BLAS", "0")
    assert not K._blas_requested("fwd", {"blas": 1})
    monkeypatch.setenv("DNN_BLAS", "1")
    assert K._blas_requested("wgrad", None)
    monkeypatch.setenv("DNN_BLAS", "fwd=1,wgrad=0")
    assert K._blas_requested("fwd", None) and not K._blas_requested("wgrad", {"blas": 1}) and not K._blas_requested("dgrad", None)


def test_reference_tail_waves_match_kernel_forms():
    assert ref.tail_waves(1, 1) == 16  # branch-free ReLU form: 16 waves
    assert ref.tail_waves(2, 1) == 8 and ref.tail_waves(0, 0) == 8


def test_tuner_signatures_include_logits_candidate():
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench"))
    from tune import signatures

    from docker_dist_nn_amd import NAMED_MODELS

    sigs = signatures(NAMED_MODELS["mnist-fcnn"], 65536)
    logits = [s for s in sigs if s[4] == "logits"]
    assert [(op, M, N, K) for op, M, N, K, _ in logits] == [("fwd", 65536, 64, 128)]
    wg = [s for s in sigs if s[0] == "wgrad"]
    assert len(wg) == 4 and all(isinstance(s[4], list) and s[4] for s in wg)


def test_wgrad_group_is_a_gpu_path():
    x = torch.zeros(64, 64, dtype=torch.bfloat16)
    items = [(x, x, torch.zeros(1, 64, 64), 1, False)] * 3
    assert K.linear_wgrad_group(items) == [0, 1, 2]  # CPU: nothing launched, caller runs all
