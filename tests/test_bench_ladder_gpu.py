"""bench.py's fail-safe ladder on the GPU: two ranks sharing cuda:0 (gloo),
launched by torch.distributed.run exactly as the driver launches bench.py. Rung 1 hangs on
rank 0 (the first-step watchdog ends it), rung 2 crashes on rank 1 (rank 0's child is killed
by its supervisor), rung 3 measures -- and rank 0 still prints ONE JSON line, with the
attempts listed, followed by the data-parallel comparison run the same way. (The literal
uniform grid: at N = 2 the planner's default is a co-located fan layout, whose own rungs
tests/test_fan_gpu.py covers.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_bench_ladder_survives_hang_and_crash(tmp_path):
    env = dict(os.environ)
    env.update(DNN_FORCE_DEVICE="0", DNN_DIST_BACKEND="gloo", DNN_FIRST_STEP_TIMEOUT="15",
               DNN_LADDER_STALL="60", TMPDIR=str(tmp_path),
               DNN_LADDER_FAULT="default=stage:0,step:0,kind:hang;"
                                "ipc-slotted=stage:1,step:0,kind:crash")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "2048",
                        "--parallelism", "uniform"],
                       env=env, stdout=subprocess.PIPE, stderr=None, text=True, timeout=280,
                       cwd=ROOT)  # stderr streams (run with -s): the attempts' progress
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0, r.stdout[-2000:]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["n_gpus"] == 2
    lad = out["ladder"]
    assert lad["rung"] == "rccl-slotted"
    att = lad["attempts"]
    assert [a["rung"] for a in att] == ["default", "ipc-slotted", "rccl-slotted"]
    assert att[0]["rc"]["0"] == "3" and att[0]["rc"]["1"] in ("killed", "3")  # watchdog exit
    # injected crash on rank 1; rank 0 is killed by its supervisor -- or gets there first
    # itself, failing on the closed gloo connection (rc 1): the race is the machine's
    assert att[1]["rc"]["1"] == "87" and att[1]["rc"]["0"] in ("killed", "1")
    assert att[2]["ok"] and att[2]["rc"] == {"0": "0", "1": "0"}
    assert out["ladder_rung"] == "rccl-slotted"
    assert out["dp_only"]["value"] > 0 and out["dp_only"]["parallelism"] == "dp2"
    assert [a["rung"] for a in lad["compare_attempts"]] == ["dp-native"]


@pytest.mark.timeout(300)
def test_bench_ladder_steady_state_hangs_and_sigterm(tmp_path):
    """rungs 1 and 2 hang AFTER their first step (steady state: only the
    heartbeat stall detector can see it), rung 3 hangs too, and the job is SIGTERMed at a set
    wall time, as the driver ends an overrunning bench. Rank 0 must still print exactly ONE
    JSON line, marked terminated, listing the stalled attempts -- within the SIGTERM grace."""
    import signal
    import time

    env = dict(os.environ)
    env.update(DNN_FORCE_DEVICE="0", DNN_DIST_BACKEND="gloo", DNN_FIRST_STEP_TIMEOUT="15",
               DNN_LADDER_STALL="12", TMPDIR=str(tmp_path),
               DNN_LADDER_FAULT="*=stage:0,step:3,kind:hang;"
                                "ipc-slotted=stage:1,step:3,kind:hang")
    t0 = time.monotonic()
    p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--steps", "20", "--warmup", "2", "--batch", "2048",
                          "--parallelism", "uniform"],
                         env=env, stdout=subprocess.PIPE, stderr=None, text=True, cwd=ROOT)
    # every rung hangs after its first steps: two stalled attempts (spawn + steps + 12 s
    # stall each, ~16-18 s on the box) fit well inside 75 s, and no rung can succeed
    deadline = t0 + 75
    while time.monotonic() < deadline and p.poll() is None:
        time.sleep(1)
    assert p.poll() is None, "the ladder ended before the SIGTERM"
    p.send_signal(signal.SIGTERM)
    t_term = time.monotonic()
    out, _ = p.communicate(timeout=60)
    assert time.monotonic() - t_term < 45  # printed and gone within the grace period
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    assert rec["terminated"] == "terminated" and rec["value"] is None
    att = rec["ladder"]["attempts"]
    assert [a["rung"] for a in att[:2]] == ["default", "ipc-slotted"], att
    for a in att[:2]:  # the hung rank and its blocked peer: whichever stall is seen first
        assert "stall" in a["rc"].values() and set(a["rc"].values()) <= {"stall", "killed"}, att
    assert "step" in att[0].get("last_heartbeat", ""), att  # it hung after stepping
