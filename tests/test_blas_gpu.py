"""hipBLASLt library GEMM path (csrc/runtime/blaslt.cpp): the three Linear products against the
hand-written kernels, the activation-derivative + column-sum epilogue kernel, and whole
training steps with DNN_BLAS=1 against DNN_BLAS=0 (library and MFMA kernels accumulate in a
different order: tolerance, not bitwise)."""
import pytest
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops import KMAJ, MNMAJ

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _comparison_build(dev):
    """The library path is in the comparison build only (python -m docker_dist_nn_amd._build
    --blas); the product module links no vendor GEMM library."""
    if not ops.kernels.blas_built():
        pytest.skip("hipBLASLt comparison path not in this build (_build --blas)")


def _close(a, b, tol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), rtol=tol, atol=tol)


@pytest.mark.parametrize("M,K,N", [(4096, 832, 1024), (2048, 1024, 256), (1024, 256, 128)])
def test_blas_products_match_mfma_kernels(dev, M, K, N):
    g = torch.Generator(device=dev).manual_seed(M + K + N)
    x = torch.relu(torch.randn(M, K, device=dev, generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g) * 0.1
    dz = (torch.randn(M, N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    # fwd with bias + ReLU in the library epilogue
    y0 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    y1 = torch.empty_like(y0)
    ops.gemm(x, w, y0, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b, act="relu")
    ops.blas_gemm(x, w, y1, trans_a=False, trans_b=True, M=M, N=N, K=K, bias=b, relu=True)
    _close(y1, y0)
    assert torch.all(y1 >= 0)
    # dgrad
    d0 = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    d1 = torch.empty_like(d0)
    ops.gemm(dz, w, d0, layout_a=KMAJ, layout_b=MNMAJ, M=M, N=K, K=N)
    ops.blas_gemm(dz, w, d1, trans_a=False, trans_b=False, M=M, N=K, K=N)
    _close(d1, d0)
    # wgrad, fp32 output, then accumulate
    g0 = torch.empty(1, N, K, device=dev)
    g1 = torch.empty(N, K, device=dev)
    ops.gemm(dz, x, g0, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K, K=M, k_total=M, splits=1,
             tiles=(64, 64))
    ops.blas_gemm(dz, x, g1, trans_a=True, trans_b=False, M=N, N=K, K=M)
    torch.testing.assert_close(g1, g0[0], rtol=1e-3, atol=1e-3)
    ops.blas_gemm(dz, x, g1, trans_a=True, trans_b=False, M=N, N=K, K=M, accumulate=True)
    torch.testing.assert_close(g1, 2 * g0[0], rtol=1e-3, atol=2e-3)


def test_dact_colsum(dev):
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(1024, 192, device=dev, generator=g).to(torch.bfloat16)
    y = torch.relu(torch.randn(1024, 192, device=dev, generator=g)).to(torch.bfloat16)
    want = torch.where(y > 0, x, torch.zeros_like(x))
    part = torch.zeros(8, 192, device=dev)
    ops.dact_colsum(x, y, "relu", part, 8)
    assert torch.equal(x, want)
    torch.testing.assert_close(part, want.float().view(8, 128, 192).sum(1), rtol=1e-5,
                               atol=1e-4)
    ops.dact_colsum(x, y, "relu")  # no partials requested: no write
    assert torch.equal(x, want)


@pytest.mark.parametrize("model", ["784-1024-1024-10", "mnist-fcnn"])
def test_engine_blas_steps_match_mfma_steps(dev, monkeypatch, model):
    from docker_dist_nn_amd import NAMED_MODELS, MLPSpec
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    spec = NAMED_MODELS.get(model) or MLPSpec.parse(model)
    x, y = synthetic_mnist(4096, seed=6)
    xb = torch.zeros(4096, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_BLAS", flag)
        tr = Trainer(spec, micro_batch=2048, num_micro=2, optim=OptimConfig(lr=0.05),
                     device=dev)
        losses = []
        for _ in range(3):
            tr.set_batch(xb, yb)
            tr.step()
            losses.append(tr.loss())
        res.append((losses, tr.stages[0].params.master.clone()))
    for a, b in zip(res[0][0], res[1][0]):
        assert abs(a - b) <= 2e-3 * abs(a) + 1e-4
    torch.testing.assert_close(res[1][1], res[0][1], rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("M,K,N", [(65536, 1024, 1024), (16384, 8192, 8192)])
def test_blas_is_deterministic(dev, M, K, N):
    """Training stays bitwise reproducible with library GEMMs in the step (same algorithm,
    same inputs -> same bits), including the stream-K solutions the heuristic picks."""
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    dz = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.blas_gemm(x, w, y, trans_a=False, trans_b=True, M=M, N=N, K=K)
        d = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        ops.blas_gemm(dz, w, d, trans_a=False, trans_b=False, M=M, N=K, K=N)
        gw = torch.empty(N, K, device=dev)
        ops.blas_gemm(dz, x, gw, trans_a=True, trans_b=False, M=N, N=K, K=M)
        outs.append((y, d, gw))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("replay", ["graph", "native"])
def test_inference_with_library_gemms_in_graph_and_program(dev, monkeypatch, replay):
    """Serving buckets capture the forward in a HIP graph (or a recorded Program); a library
    GEMM inside must capture and replay like the kernels (65536-row bucket of the headline
    model hits the tuned 512->256 library forward)."""
    import numpy as np

    from docker_dist_nn_amd.config import LayerWeights
    from docker_dist_nn_amd.engine.inference import InferenceEngine

    monkeypatch.setenv("DNN_SERVE_REPLAY", replay)
    dims = [784, 512, 256, 128, 10]
    rng = np.random.default_rng(0)
    layers = [LayerWeights(rng.standard_normal((dims[i + 1], dims[i])) / np.sqrt(dims[i]),
                           rng.standard_normal(dims[i + 1]) * 0.1,
                           "softmax" if i == len(dims) - 2 else "relu")
              for i in range(len(dims) - 1)]
    x = rng.standard_normal((65536, 784))
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DNN_BLAS", flag)
        eng = InferenceEngine([[l] for l in layers], dev, expected_input=784)
        eng.predict(x)
        outs.append(eng.predict(x))
    np.testing.assert_allclose(outs[1], outs[0], rtol=3e-2, atol=3e-3)


def test_blas_probe_and_fallback(dev, monkeypatch):
    """The per-signature probe finds algorithms for the products the tuned table routes to the
    library; a forced-library product still runs (and matches) through linear_fwd."""
    from docker_dist_nn_amd.ops import kernels as K

    x = torch.randn(4096, 1024, device=dev).to(torch.bfloat16)
    w = (torch.randn(1024, 1024, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.zeros(1024, device=dev)
    y = torch.empty(4096, 1024, device=dev, dtype=torch.bfloat16)
    assert K._blas_ok(x, w, y, False, True, 4096, 1024, 1024, b, True, False)
    monkeypatch.setenv("DNN_BLAS", "1")
    K.linear_fwd(x, w, b, y, act="relu")
    monkeypatch.setenv("DNN_BLAS", "0")
    y0 = torch.empty_like(y)
    K.linear_fwd(x, w, b, y0, act="relu")
    _close(y, y0)
