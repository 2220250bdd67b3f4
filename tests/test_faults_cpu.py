"""Failure detection in multi-rank training (gloo, 2 ranks = a 2-stage pipeline, CPU):
``DNN_FAULT`` crash / hang / nan / raise injected into one rank must end the WHOLE job with a
non-zero status and the cause in the log, well within the bound -- never a silent hang. The
reference has no training and only a per-hop RPC deadline (grpc_node.py:133-140); these are the
engine's equivalents (docker_dist_nn_amd/faults.py: Watchdog, FaultInjector, check_finite)."""
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(fault=None, extra=(), timeout=150):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("DNN_FAULT", None)
    if fault:
        env["DNN_FAULT"] = fault
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "-m", "docker_dist_nn_amd.cli.train", "--device", "cpu", "--model", "784-64-10",
           "--synthetic", "2048", "--micro-batch", "64", "--num-micro-batches", "2",
           "--steps", "8", "--check-every", "1", *extra]
    t0 = time.monotonic()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    return r.returncode, r.stdout + r.stderr, time.monotonic() - t0


def test_no_fault_baseline():
    rc, out, _ = _train()
    assert rc == 0, out[-3000:]
    assert '"parallelism": "pp2dp1"' in out


@pytest.mark.parametrize("fault,needle,extra", [
    ("stage:1,step:3,kind:crash", "injecting fault 'crash' at stage 1, step 3", ()),
    ("stage:1,step:3,kind:raise", "injected fault at stage 1 step 3", ()),
    ("stage:0,step:2,kind:nan", "non-finite loss", ()),
    ("stage:1,step:3,kind:hang", "[watchdog:rank1] no progress", ("--watchdog", "4")),
])
def test_injected_fault_ends_the_job(fault, needle, extra):
    rc, out, dt = _train(fault, extra)
    assert rc != 0, out[-3000:]
    assert needle in out, out[-3000:]
    assert dt < 120, dt
