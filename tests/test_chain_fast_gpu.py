"""Device-side serving chain (serve/fastpath.py, csrc/kernels/chain.hip) on one GPU: a 4-rank
chain with every stage on cuda:0 (gloo for the set-up collectives, IPC slots + flags for the
requests), brought up by run_grpc_fcnn.py --mode ranks and queried over the reference gRPC
protocol. Serving-size requests (<= 8 rows) take the device-side chain, larger ones the
message chain; both must match the fp64 reference forward. A stage that hangs is blamed by
name within the per-hop deadline; concurrent callers each get their own rows."""
import os
import socket
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import grpc
import numpy as np
import pytest

from docker_dist_nn_amd.config import load_model_config
from docker_dist_nn_amd.cpu_ref import model_forward
from docker_dist_nn_amd.data import write_examples
from docker_dist_nn_amd.serve.ingress import LayerClient
from docker_dist_nn_amd.weights_io import export_model_json

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def model4(tmp_path_factory):
    d = tmp_path_factory.mktemp("fast")
    rng = np.random.default_rng(3)
    dims = [784, 256, 128, 64, 10]
    ws = [rng.standard_normal((dims[i + 1], dims[i])) * (2.0 / np.sqrt(dims[i])) for i in range(4)]
    bs = [rng.standard_normal(dims[i + 1]) * 0.1 for i in range(4)]
    cfg = d / "model4.json"
    export_model_json(str(cfg), ws, bs, ["relu", "relu", "relu", "softmax"],
                      layer_distribution=[1, 1, 1, 1])
    x = rng.random((64, 784))
    inp = d / "inputs4.json"
    write_examples(str(inp), x, np.zeros(64, dtype=np.int64))
    return cfg, inp, x


def _start(cfg, inp, port, tmp, extra_env=None, args=()):
    env = dict(os.environ, PYTHONPATH=ROOT, DNN_FORCE_DEVICE="0", DNN_DIST_BACKEND="gloo",
               **(extra_env or {}))
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "src", "run_grpc_fcnn.py"),
                          "--config", str(cfg), "--inputs", str(inp), "--port", str(port),
                          "--mode", "ranks", "--device", "cuda", "--run-for", "120",
                          "--cache-dir", str(tmp / "cache"), *args],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    t0 = time.time()
    while time.time() - t0 < 120:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return p
        except OSError:
            if p.poll() is not None:
                raise RuntimeError(p.stdout.read())
            time.sleep(0.3)
    p.terminate()
    raise RuntimeError("server did not come up")


def _stop(p):
    p.terminate()
    try:
        out, _ = p.communicate(timeout=60)
    except subprocess.TimeoutExpired:
        p.kill()
        out, _ = p.communicate()
    return out


@pytest.mark.timeout(240)
def test_fast_chain_matches_reference_and_serves_concurrently(model4, tmp_path):
    cfg, inp, x = model4
    layers = load_model_config(str(cfg)).layers
    port = _port()
    p = _start(cfg, inp, port, tmp_path)
    ok = False
    try:
        c = LayerClient(f"127.0.0.1:{port}", timeout=60)
        for rows in (1, 3, 8, 40, 1):  # 40 rows: the message chain
            q = x[:rows] if rows != 3 else x[10:13]
            np.testing.assert_allclose(c.process(q), model_forward(layers, q), atol=2e-2)
        chunks = [x[i:i + 1 + i % 8] for i in range(48)]
        with ThreadPoolExecutor(8) as pool:
            outs = list(pool.map(c.process, chunks))
        for ch, out in zip(chunks, outs):
            np.testing.assert_allclose(out, model_forward(layers, ch), atol=2e-2)
        ts = []
        for _ in range(50):
            t0 = time.perf_counter()
            c.process(x[:1])
            ts.append(time.perf_counter() - t0)
        print(f"fast chain batch-1 p50 {np.median(ts) * 1e3:.3f} ms")
        c.close()
        ok = True
    finally:
        out = _stop(p)
        if not ok:  # the servers' side of a failure
            print(out[-12000:])
    assert "device-side chain" in out, out[-3000:]
    assert "Shutdown complete." in out, out[-3000:]


@pytest.mark.timeout(240)
def test_fast_chain_blames_the_hung_stage(model4, tmp_path):
    cfg, inp, x = model4
    port = _port()
    p = _start(cfg, inp, port, tmp_path,
               {"DNN_FAULT_STAGE": "2", "DNN_FAULT_KIND": "hang", "DNN_FAULT_AFTER": "1"},
               args=("--hop-timeout", "1.0"))
    try:
        c = LayerClient(f"127.0.0.1:{port}", timeout=30)
        ref = model_forward(load_model_config(str(cfg)).layers, x[:1])
        np.testing.assert_allclose(c.process(x[:1]), ref, atol=2e-2)  # before the hang
        for _ in range(2):
            t0 = time.monotonic()
            with pytest.raises(grpc.RpcError) as ei:
                c.process(x[:1])
            assert ei.value.code() == grpc.StatusCode.DEADLINE_EXCEEDED, ei.value
            assert "Failed to forward request to layer_container_2" in ei.value.details(), \
                ei.value.details()
            assert time.monotonic() - t0 < 6.0
        c.close()
    finally:
        out = _stop(p)
    assert "device-side chain" in out, out[-3000:]


@pytest.mark.timeout(240)
def test_fast_chain_stage_error_is_reported(model4, tmp_path):
    cfg, inp, x = model4
    port = _port()
    p = _start(cfg, inp, port, tmp_path,
               {"DNN_FAULT_STAGE": "1", "DNN_FAULT_KIND": "raise", "DNN_FAULT_AFTER": "0"})
    try:
        c = LayerClient(f"127.0.0.1:{port}", timeout=30)
        with pytest.raises(grpc.RpcError) as ei:
            c.process(x[:2])
        assert ei.value.code() == grpc.StatusCode.INTERNAL, ei.value
        assert "layer_container_1" in ei.value.details(), ei.value.details()
        c.close()
    finally:
        _stop(p)


def test_chain_kernels_in_one_process(dev):
    """csrc/kernels/chain.hip on its own: a producer stream sends rows into a consumer's slot
    (flag, header), the consumer stream receives them into its cached buffer and acks; a
    producer whose consumer never drained the slot times out and blames the consumer; a
    consumer whose rows never arrive times out, and its send blames the producer."""
    import torch

    from docker_dist_nn_amd.utils.devmem import uncached_zeros
    from docker_dist_nn_amd.utils.native import native

    n = native()
    rows, width = 3, 64
    rb = width * 2
    flags_c = uncached_zeros((64,), torch.int32, dev)  # consumer: [0] in flag, [2:4] hdr,
    flags_p = uncached_zeros((64,), torch.int32, dev)  # producer: [8] ack, [9] err
    slot = uncached_zeros((8, width), torch.bfloat16, dev)
    src = torch.randn(8, width, device=dev).to(torch.bfloat16)
    dst = torch.zeros(8, width, dtype=torch.bfloat16, device=dev)
    lhdr = torch.zeros(4, dtype=torch.int32, device=dev)
    err_c = torch.zeros(4, dtype=torch.int32, device=dev)
    sp, sc = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    fp, fc = flags_p.data_ptr(), flags_c.data_ptr()

    def send(seq, ack_target, timeout=2.0):
        n.chain_send(sp.cuda_stream, src.data_ptr(), rb, slot.data_ptr(), rb, rows, rb,
                     fc + 8, 0, fp + 36, 0, 0, fp + 32, ack_target, fc, seq, 0, timeout)

    def recv(seq, timeout=2.0):
        n.chain_recv(sc.cuda_stream, fc, slot.data_ptr(), rb, fc + 8, dst.data_ptr(), rb,
                     lhdr.data_ptr(), rows, rb, err_c.data_ptr(), seq, fp + 32, timeout)

    recv(1)          # enqueued before the data exists: it waits
    send(1, 0)
    torch.cuda.synchronize(dev)
    assert torch.equal(dst[:rows], src[:rows])
    assert lhdr[:2].tolist() == [0, rows] and int(flags_p[8]) == 1 and int(err_c[0]) == 0
    # the consumer drained slot 1 (ack = 1): request 2 may reuse it
    src.mul_(2)
    send(2, 1)
    recv(2)
    torch.cuda.synchronize(dev)
    assert torch.equal(dst[:rows], src[:rows]) and int(flags_p[8]) == 2
    # request 3 needs ack >= 3, which never comes: the send gives up and blames stage 0 + 1
    send(3, 3, timeout=0.2)
    torch.cuda.synchronize(dev)
    assert int(flags_c[0]) == 3 and (int(flags_c[2]) & 0xFF) == 4
    assert (int(flags_c[2]) >> 8) & 0xFF == 1
    # request 9 never arrives: the receive times out, sets its error word, pulls nothing
    dst.zero_()
    recv(9, timeout=0.2)
    torch.cuda.synchronize(dev)
    assert int(err_c[0]) == 1 and float(dst.float().abs().sum()) == 0.0


@pytest.mark.parametrize("rows", [1, 3, 8])
def test_chain_gemv_send_in_one_process(dev, rows):
    """chain_gemv_send (a stage's last layer fused with its send): the rows it writes into the
    consumer's slot equal ops.gemv's bit for bit, the header / flag / counter protocol matches
    chain_send's, and a consumer that never acks is blamed with no rows written."""
    import torch

    from docker_dist_nn_amd import ops
    from docker_dist_nn_amd.utils.devmem import uncached_zeros
    from docker_dist_nn_amd.utils.native import native

    n = native()
    K, N = 832, 1024
    g = torch.Generator().manual_seed(rows)
    x = (torch.randn(8, K, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    ref = torch.empty(rows, N, dtype=torch.bfloat16, device=dev)
    ops.gemv(x[:rows], w, b, ref, act="relu")
    flags_c = uncached_zeros((64,), torch.int32, dev)  # consumer: [0] flag, [2:4] header
    flags_p = uncached_zeros((64,), torch.int32, dev)  # producer: [8] ack, [9] err
    slot = uncached_zeros((8, N), torch.bfloat16, dev)
    counter = torch.zeros(4, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    fp, fc = flags_p.data_ptr(), flags_c.data_ptr()

    def send(seq, ack_target, timeout=2.0):
        n.chain_gemv_send(s.cuda_stream, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0),
                          b.data_ptr(), 1, rows, N, K, 0, slot.data_ptr(), N, fc + 8, 0,
                          fp + 36, 0, 0, fp + 32, ack_target, fc, seq, 0, counter.data_ptr(),
                          timeout)

    send(1, 0)
    torch.cuda.synchronize(dev)
    assert torch.equal(slot[:rows], ref)
    assert int(flags_c[0]) == 1 and flags_c[2:4].tolist() == [0, rows]
    assert counter.tolist() == [0, 0, 0, 0]
    # the consumer never drained the slot (ack stays 0 < 2): blamed (stage 0 + 1), no rows
    slot.zero_()
    send(2, 2, timeout=0.2)
    torch.cuda.synchronize(dev)
    assert int(flags_c[0]) == 2 and (int(flags_c[2]) & 0xFF) == 4
    assert (int(flags_c[2]) >> 8) & 0xFF == 1
    assert float(slot.float().abs().sum()) == 0.0 and counter.tolist() == [0, 0, 0, 0]


def test_chain_one_launch_hop_in_one_process(dev):
    """chain_gemv_send with the receive folded in (in_flag): the kernel waits for the input
    slot's flag, reads the rows from the slot itself, writes the layer's rows into the next
    slot, raises its flag and acks the producer -- and a missing input blames the producer."""
    import torch

    from docker_dist_nn_amd import ops
    from docker_dist_nn_amd.utils.devmem import uncached_zeros
    from docker_dist_nn_amd.utils.native import native

    n = native()
    K, N, rows = 1024, 1024, 2
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(8, K, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    ref = torch.empty(rows, N, dtype=torch.bfloat16, device=dev)
    ops.gemv(x[:rows], w, b, ref, act="relu")
    f_in = uncached_zeros((64,), torch.int32, dev)    # this stage: [0] flag, [2:4] header
    f_out = uncached_zeros((64,), torch.int32, dev)   # consumer: [0] flag, [2:4] header
    f_prod = uncached_zeros((64,), torch.int32, dev)  # producer: [8] ack
    slot_in = uncached_zeros((8, K), torch.bfloat16, dev)
    slot_out = uncached_zeros((8, N), torch.bfloat16, dev)
    err = torch.zeros(4, dtype=torch.int32, device=dev)
    counter = torch.zeros(4, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)

    def hop(seq, timeout=2.0):
        n.chain_gemv_send(s.cuda_stream, slot_in.data_ptr(), K, w.data_ptr(), K, b.data_ptr(),
                          1, rows, N, K, 0, slot_out.data_ptr(), N, f_out.data_ptr() + 8,
                          f_in.data_ptr() + 8, err.data_ptr(), 1, 0, 0, 0, f_out.data_ptr(),
                          seq, f_prod.data_ptr() + 32, counter.data_ptr(), timeout,
                          in_flag=f_in.data_ptr())

    hop(1)  # enqueued before its input exists: it waits (on stream s; the writes below go
    slot_in.copy_(x)  # through the current stream -- no device-wide sync while it spins)
    f_in[2:4] = torch.tensor([0, rows], dtype=torch.int32, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    f_in[0] = 1  # the producer's flag
    torch.cuda.current_stream(dev).synchronize()
    s.synchronize()
    assert torch.equal(slot_out[:rows], ref)
    assert int(f_out[0]) == 1 and f_out[2:4].tolist() == [0, rows] and int(f_prod[8]) == 1
    # request 2 never arrives: no rows, the producer (stage 0) is blamed downstream
    slot_out.zero_()
    hop(2, timeout=0.2)
    s.synchronize()
    assert int(f_out[0]) == 2 and (int(f_out[2]) & 0xFF) == 4 and (int(f_out[2]) >> 8) == 0
    assert float(slot_out.float().abs().sum()) == 0.0 and counter.tolist() == [0, 0, 0, 0]
