"""The device-side chain's announcement ring (serve/fastpath.Announcer) across processes: a
reader attached to rank 0's ring sees every (seq, rows) in order, wraps around the ring, and
stops when told."""
import multiprocessing as mp
import os


def _reader(path, n, q):
    from docker_dist_nn_amd.serve.fastpath import Announcer

    a = Announcer(path, create=False)
    q.put("ready")
    got = []
    seq = 0
    while True:
        seq += 1
        rows = a.next(seq)
        if rows is None:
            break
        got.append((seq, rows))
    a.close()
    q.put(got)


def test_announcer_ring_in_order_and_stop(tmp_path):
    from docker_dist_nn_amd.serve.fastpath import ANN_SLOTS, Announcer

    path = str(tmp_path / "ring")
    a = Announcer(path, create=True)
    n = ANN_SLOTS + 500  # wraps around the ring
    q = mp.get_context("spawn").Queue()
    p = mp.get_context("spawn").Process(target=_reader, args=(path, n, q))
    p.start()
    assert q.get(timeout=120) == "ready"
    for s in range(1, n + 1):
        a.announce(s, 1 + s % 8)
        if s % 256 == 0:  # stay within one ring of the reader
            import time
            time.sleep(0.05)
    import time
    time.sleep(0.3)
    a.stop()
    got = q.get(timeout=60)
    p.join(30)
    a.close()
    assert got == [(s, 1 + s % 8) for s in range(1, n + 1)]
    assert not os.path.exists(path)  # the owner unlinks the ring


def test_lapped_reader_raises_and_stop_ends_a_wait(tmp_path):
    """A reader a whole ring behind sees the overrun (no silent spin); a reader waiting for an
    entry whose head moved but whose slot is not written returns None once the ring stops."""
    import pytest

    from docker_dist_nn_amd.serve.fastpath import ANN_SLOTS, Announcer

    a = Announcer(str(tmp_path / "ring"), create=True)
    a.announce(1 + ANN_SLOTS, 3)  # slot of request 1 now holds a later request
    with pytest.raises(RuntimeError, match="overrun"):
        a.next(1)
    a.a[0] = 5  # head past request 2, entry never written
    a.stop()
    assert a.next(2) is None
    a.close()


class _CR:
    names = ["layer_container_0", "layer_container_1"]
    rank = 1


def _bare_chain():
    import threading

    from docker_dist_nn_amd.serve.fastpath import FastChain

    fc = FastChain.__new__(FastChain)
    fc.cr, fc.rank, fc.lock, fc.inflight = _CR(), 1, threading.Lock(), 0
    fc.persist, fc.failed, fc.doorbell = False, False, False
    return fc


def test_back_pressure_bounds_requests_in_flight():
    """Rank 0 refuses a request (RESOURCE_EXHAUSTED) with half a ring in flight, and the
    in-flight count is released whether a request succeeds or fails."""
    import grpc
    import numpy as np
    import pytest

    from docker_dist_nn_amd.serve.fastpath import ANN_SLOTS
    from docker_dist_nn_amd.serve.ingress import StageFailure

    fc = _bare_chain()
    calls = []

    def ok(x, timeout):
        calls.append(fc.inflight)
        return x

    def bad(x, timeout):
        raise StageFailure("layer_container_1", grpc.StatusCode.INTERNAL, "boom")

    fc._predict = ok
    assert fc.predict(np.zeros((1, 4)), None).shape == (1, 4) and calls == [1]
    fc._predict = bad
    with pytest.raises(StageFailure):
        fc.predict(np.zeros((1, 4)), None)
    assert fc.inflight == 0
    fc.inflight = ANN_SLOTS // 2
    fc._predict = ok
    with pytest.raises(StageFailure) as ei:
        fc.predict(np.zeros((1, 4)), None)
    assert ei.value.code == grpc.StatusCode.RESOURCE_EXHAUSTED and len(calls) == 1


def test_chain_thread_failure_is_logged_not_silent(caplog):
    """A failure of a stage's device-side chain thread is logged and recorded; the stage's
    progress stops there, which is what rank 0's blame reads."""
    fc = _bare_chain()

    def boom():
        raise RuntimeError("announcement ring overrun at request 7")

    fc._host_loop = boom
    with caplog.at_level("ERROR"):
        fc.loop()
    assert fc.failed and "device-side chain thread failed" in caplog.text


def test_doorbell_result_ack_advances_over_contiguous_consumed_requests():
    """Rank 0's shared result-ring ack (the last rank reuses a result slot only behind it)
    advances over the contiguous run of consumed requests, whatever order concurrent callers
    finish in; an abandoned (timed-out) request counts as consumed."""
    import numpy as np

    from docker_dist_nn_amd.serve.fastpath import NSLOT

    fc = _bare_chain()
    fc.res_bytes = 256
    fc._res_flag_off = NSLOT * fc.res_bytes
    fc.res_np = np.zeros((fc._res_flag_off // 4 + NSLOT + 8,), dtype=np.int32)
    fc._res_acked, fc._res_done = 0, set()
    ack = lambda: int(fc.res_np[fc._res_flag_off // 4 + NSLOT])  # noqa: E731
    fc._consume(2)
    assert ack() == 0  # request 1 still out
    fc._consume(3)
    fc._consume(1)
    assert ack() == 3
    fc._consume(5)
    assert ack() == 3
    fc._consume(4)  # e.g. a caller that timed out: abandoned, slot free again
    assert ack() == 5 and not fc._res_done
