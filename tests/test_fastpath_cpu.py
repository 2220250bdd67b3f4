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
