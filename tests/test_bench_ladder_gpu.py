"""bench.py's fail-safe ladder on the GPU: two ranks sharing cuda:0 (gloo),
launched by torch.distributed.run exactly as the driver launches bench.py. Rung 1 hangs on
rank 0 (the first-step watchdog ends it), rung 2 crashes on rank 1 (rank 0's child is killed
by its supervisor), rung 3 measures -- and rank 0 still prints ONE JSON line, with the
attempts listed, followed by the data-parallel comparison run the same way."""
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
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "2048"],
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
    assert att[1]["rc"]["1"] == "87" and att[1]["rc"]["0"] == "killed"      # injected crash
    assert att[2]["ok"] and att[2]["rc"] == {"0": "0", "1": "0"}
    assert out["ladder_rung"] == "rccl-slotted"
    assert out["dp_only"]["value"] > 0 and out["dp_only"]["parallelism"] == "dp2"
    assert [a["rung"] for a in lad["dp_attempts"]] == ["dp-native"]
