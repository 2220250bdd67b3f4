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


def _persistent_stage(dev, K, N, act, nslot=4, out_f32=False, n_out=None):
    """A persistent stage kernel (chain_stage_run) between a simulated producer (this test
    writes the input slots, headers and flags) and a simulated consumer (it reads the output
    slots and writes the ack)."""
    import ctypes

    import torch

    from docker_dist_nn_amd.utils.devmem import uncached_zeros
    from docker_dist_nn_amd.utils.native import native

    n = native()
    st = type("S", (), {})()
    st.n, st.K, st.N, st.nslot = n, K, N, nslot
    st.n_out = n_out or N
    st.f_in = uncached_zeros((64,), torch.int32, dev)    # [0:nslot] flags, [16:] headers
    st.f_out = uncached_zeros((64,), torch.int32, dev)   # consumer: same layout
    st.f_ack = uncached_zeros((16,), torch.int32, dev)   # [0] the consumer's ack (ours)
    st.f_prod = uncached_zeros((16,), torch.int32, dev)  # [0] the producer's ack (we write)
    st.slots_in = uncached_zeros((nslot, 8, K), torch.bfloat16, dev)
    st.slots_out = uncached_zeros((nslot, 8, N), torch.float32 if out_f32 else torch.bfloat16,
                                  dev)
    st.sync = torch.zeros(2 * nslot + 4, dtype=torch.int32, device=dev)
    st.hp, st.dp = n.host_alloc_mapped(64)
    st.ctl = np.ctypeslib.as_array((ctypes.c_uint32 * 16).from_address(st.hp))
    g = torch.Generator().manual_seed(K + N)
    st.w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    st.b = torch.randn(N, generator=g).to(dev)
    # the persistent kernel's stream has a hardware queue of its own (as in serve/fastpath.py):
    # this test's writes on the current stream must never queue behind it
    st.s_ptr = n.stream_create_dedicated()
    st.s = torch.cuda.ExternalStream(st.s_ptr, device=dev)
    # ... and it is a blocking stream: the test's own work goes on a non-blocking stream, or
    # the null stream would wait for the kernel (serve/fastpath.py pauses it instead)
    st.side = torch.cuda.Stream(dev)
    st.act, st.out_f32 = act, out_f32
    st.epoch = 0

    def launch(start, idle=5.0, timeout=2.0):
        st.epoch += 1
        st.ctl[0] = 0
        es = st.slots_out.element_size()
        return n.chain_stage_run(
            st.s.cuda_stream, st.f_in.data_ptr(), st.f_in.data_ptr() + 64,
            st.slots_in.data_ptr(), K, st.f_prod.data_ptr(), st.w.data_ptr(), K, st.b.data_ptr(),
            {"relu": 1, "softmax": 3}[act], st.n_out, K, int(out_f32), st.slots_out.data_ptr(),
            8 * N * es, N, st.f_out.data_ptr() + 64, 2, st.f_out.data_ptr(), st.f_ack.data_ptr(),
            st.dp, st.dp + 4, st.sync.data_ptr(), start, st.epoch, 1, nslot, 8, idle, timeout)

    def feed(seq, x, status=0):
        slot = seq % nslot
        rows = x.shape[0]
        st.slots_in[slot, :rows].copy_(x)
        st.f_in[16 + 2 * slot:18 + 2 * slot] = torch.tensor([status, rows], dtype=torch.int32,
                                                            device=dev)
        torch.cuda.current_stream(dev).synchronize()
        st.f_in[slot] = seq
        torch.cuda.current_stream(dev).synchronize()

    def wait_out(seq, limit=10.0):
        slot = seq % nslot
        t0 = time.monotonic()
        while int(st.f_out[slot]) != seq:
            assert time.monotonic() - t0 < limit, f"request {seq} never reached the consumer"
            time.sleep(1e-3)
        return st.f_out[16 + 2 * slot:18 + 2 * slot].tolist(), st.slots_out[slot].clone()

    st.launch, st.feed, st.wait_out = launch, feed, wait_out
    return st


@pytest.mark.timeout(120)
def test_chain_stage_persistent_in_one_process(dev):
    """chain_stage_run: ONE launch serves a sequence of requests of varying rows -- each
    output bitwise equal to ops.gemv (chain_gemv_send's math), the producer acked and the
    progress counter published in host memory; an upstream failure travels on unchanged; a
    consumer that never drains is blamed; the host's stop word and the idle timer end the
    launch, and a relaunch from the published progress continues the sequence."""
    import torch

    K, N = 1024, 1024
    st = _persistent_stage(dev, K, N, "relu")
    prev = torch.cuda.current_stream(dev)
    torch.cuda.set_stream(st.side)
    try:
        _persistent_relu_body(st, dev, K, N)
    finally:
        torch.cuda.set_stream(prev)


def _persistent_relu_body(st, dev, K, N):
    import torch

    from docker_dist_nn_amd import ops

    g = torch.Generator().manual_seed(11)
    xs = (torch.randn(64, K, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    wg = st.launch(0)
    assert wg >= 16
    seq, off = 0, 0
    for rows in (1, 3, 8, 2, 5, 1, 8, 4, 7):
        seq += 1
        x = xs[off:off + rows]
        off += rows
        st.feed(seq, x)
        hdr, out = st.wait_out(seq)
        ref = torch.empty(rows, N, dtype=torch.bfloat16, device=dev)
        ops.gemv(x, st.w, st.b, ref, act="relu")
        assert hdr == [0, rows], (seq, hdr)
        assert torch.equal(out[:rows], ref), f"request {seq} ({rows} rows) differs"
        assert int(st.f_prod[0]) == seq and int(st.ctl[1]) == seq
        st.f_ack[0] = seq  # the consumer drained it
    # an upstream failure (stage 0 blamed for a deadline) travels on, no rows written
    seq += 1
    st.slots_out[seq % st.nslot].zero_()
    st.feed(seq, xs[:2], status=4 | (0 << 8))
    hdr, out = st.wait_out(seq)
    assert hdr == [4, 2] and float(out.float().abs().sum()) == 0.0
    # the consumer stops draining (its ack stays where it is): requests whose slots it drained
    # before still go; the first one reusing an undrained slot blames it (stage 2)
    acked = int(st.f_ack[0])
    while seq + 1 - st.nslot <= acked:
        seq += 1
        st.feed(seq, xs[:1])
        hdr, _ = st.wait_out(seq)
        assert hdr == [0, 1], (seq, hdr)
    seq += 1
    st.feed(seq, xs[:1])
    hdr, _ = st.wait_out(seq)
    assert (hdr[0] & 0xFF) == 4 and (hdr[0] >> 8) == 2, hdr
    st.f_ack[0] = seq
    # the host's stop word ends the launch promptly
    t0 = time.monotonic()
    st.ctl[0] = 1
    st.s.synchronize()
    assert time.monotonic() - t0 < 1.0
    done = int(st.ctl[1])
    assert done == seq
    # a relaunch from the progress counter continues; then the idle timer ends it alone
    st.launch(done, idle=0.3)
    seq += 1
    st.feed(seq, xs[:3])
    hdr, out = st.wait_out(seq)
    ref = torch.empty(3, N, dtype=torch.bfloat16, device=dev)
    ops.gemv(xs[:3], st.w, st.b, ref, act="relu")
    assert hdr == [0, 3] and torch.equal(out[:3], ref)
    t0 = time.monotonic()
    st.s.synchronize()
    assert time.monotonic() - t0 < 3.0 and int(st.sync[2 * st.nslot + 1]) == st.epoch
    assert st.sync[:st.nslot].tolist() == [0] * st.nslot  # counters left at zero
    st.n.host_free(st.hp)
    st.n.stream_destroy(st.s_ptr)


@pytest.mark.timeout(120)
def test_chain_stage_persistent_softmax_last_stage(dev):
    """The last stage's persistent kernel: one workgroup, fp32 rows into rank 0's result
    slot layout, row softmax over the real outputs against the fp32 torch reference."""
    import torch

    K, N, n_out = 1024, 64, 10
    st = _persistent_stage(dev, K, N, "softmax", out_f32=True, n_out=n_out)
    prev = torch.cuda.current_stream(dev)
    torch.cuda.set_stream(st.side)
    try:
        _persistent_softmax_body(st, dev, K, N, n_out)
    finally:
        torch.cuda.set_stream(prev)


def _persistent_softmax_body(st, dev, K, N, n_out):
    import torch

    g = torch.Generator().manual_seed(5)
    x = (torch.randn(8, K, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    assert st.launch(0) == 1
    for seq, rows in enumerate((1, 8, 3), start=1):
        st.feed(seq, x[:rows])
        hdr, out = st.wait_out(seq)
        z = x[:rows].float() @ st.w[:n_out].float().t() + st.b[:n_out]
        ref = torch.softmax(z, dim=1)
        assert hdr == [0, rows]
        torch.testing.assert_close(out[:rows, :n_out], ref, atol=1e-5, rtol=1e-4)
        st.f_ack[0] = seq
    st.ctl[0] = 1
    st.s.synchronize()
    st.n.host_free(st.hp)
    st.n.stream_destroy(st.s_ptr)
