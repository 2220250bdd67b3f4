"""The fail-safe ladder's supervisors (docker_dist_nn_amd/ladder.py), on CPU.

Two supervisor ranks (under torch.distributed.run, so through the elastic agent's store, and
with rank 0 hosting the store) run a fake child per attempt: on rung "a" rank 0 hangs without
heartbeats (killed as stalled; rank 1, alive and beating, is killed because its peer failed),
on rung "b" rank 1 crashes (rank 0 killed), rung "c" succeeds. Every supervisor must agree on
every outcome and rank 0 must report rung c's result with all three attempts listed."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, {root!r})
    from docker_dist_nn_amd import ladder
    rank = int(os.environ["RANK"])
    if ladder.is_child():
        ladder.heartbeat("start")
        fault = os.environ.get("DNN_FAULT", "")
        mine = f"stage:{{rank}}," in fault + ","
        if fault and mine and "kind:hang" in fault:
            while True:          # a hang: no heartbeat, never exits
                time.sleep(1)
        if fault and mine and "kind:crash" in fault:
            os._exit(87)
        if fault:                # a healthy rank of a failing attempt: alive, beating, stuck
            while True:
                ladder.heartbeat("waiting for a peer")
                time.sleep(0.2)
        ladder.write_result({{"rung": os.environ[ladder.RUNG_ENV],
                              "port": os.environ["MASTER_PORT"]}})
        sys.exit(0)
    world = int(os.environ["WORLD_SIZE"])
    sup = ladder.Supervisor(lambda r: [sys.executable, __file__], rank=rank, world=world,
                            stall=3.0)
    res, rung = sup.climb([ladder.Rung("a"), ladder.Rung("b"), ladder.Rung("c")])
    print(json.dumps({{"rank": rank, "res": res, "rung": rung.name if rung else None,
                      "attempts": sup.attempts}}), flush=True)
""")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _check(outs):
    recs = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{")]
    assert sorted(r["rank"] for r in recs) == [0, 1], outs
    for r in recs:
        assert r["rung"] == "c"
        a = r["attempts"]
        assert [x["rung"] for x in a] == ["a", "b", "c"]
        assert [x["ok"] for x in a] == [False, False, True]
        assert a[0]["rc"] == {"0": "stall", "1": "killed"}, a[0]
        assert a[1]["rc"] == {"0": "killed", "1": "87"}, a[1]
        assert a[2]["rc"] == {"0": "0", "1": "0"}
    assert all(r["res"] == recs[0]["res"] for r in recs)  # every rank gets rank 0's result
    assert recs[0]["res"]["rung"] == "c"


FAULT = "a=stage:0,step:0,kind:hang;b=stage:1,step:0,kind:crash"


def _env(tmp_path):
    env = dict(os.environ)
    env.update(DNN_LADDER_FAULT=FAULT, TMPDIR=str(tmp_path), PYTHONPATH=ROOT)
    return env


@pytest.mark.timeout(120)
def test_ladder_supervisors_agree_torchrun(tmp_path):
    script = tmp_path / "sup.py"
    script.write_text(SCRIPT.format(root=ROOT))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), str(script)],
                       env=_env(tmp_path), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    _check([r.stdout])


@pytest.mark.timeout(120)
def test_ladder_supervisors_agree_own_store(tmp_path):
    script = tmp_path / "sup.py"
    script.write_text(SCRIPT.format(root=ROOT))
    port = _port()
    procs = []
    for rank in range(2):
        env = _env(tmp_path)
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        env.update(RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=110)
        assert p.returncode == 0, e[-3000:]
        outs.append(o)
    _check(outs)


def test_rung_fault_parse():
    from docker_dist_nn_amd.ladder import bench_rungs, rung_fault

    assert rung_fault("b", FAULT) == "stage:1,step:0,kind:crash"
    assert rung_fault("z", FAULT) == ""
    wild = "*=stage:0,step:3,kind:hang;b=stage:1,step:3,kind:hang"
    assert rung_fault("b", wild) == "stage:1,step:3,kind:hang"  # a named rung wins
    assert rung_fault("z", wild) == "stage:0,step:3,kind:hang"
    names = [r.name for r in bench_rungs(8)]
    assert names == ["default", "ipc-slotted", "rccl-slotted", "rccl-streams", "python",
                     "dp-native", "dp-python"]
    assert [r.name for r in bench_rungs(4, dp_only=True)] == ["dp-native", "dp-python"]
    assert bench_rungs(4)[-1].args == ["--parallelism", "dp4", "--graph", "off"]
    assert bench_rungs(4)[0].args == [] and bench_rungs(4)[1].args == ["--graph", "off"]


# Children that stay alive and keep beating forever (a slow or steady-state-stuck attempt the
# stall detector cannot see); supervisors with a deadline and rank 0's OneLine report.
DEADLINE_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, {root!r})
    from docker_dist_nn_amd import ladder
    rank = int(os.environ["RANK"])
    if ladder.is_child():
        while True:
            ladder.heartbeat("busy")
            time.sleep(0.2)
    world = int(os.environ["WORLD_SIZE"])
    sup = None
    def build(reason):
        return {{"value": None, "terminated": reason,
                 "attempts": list(sup.attempts) if sup else []}}
    line = ladder.OneLine(rank, build)
    line.install_sigterm()
    sup = ladder.Supervisor(lambda r: [sys.executable, __file__], rank=rank, world=world,
                            stall=3.0, deadline=time.monotonic() + float({deadline}))
    res, rung = sup.climb([ladder.Rung("a"), ladder.Rung("b")], budget_s=1.0)
    line.emit()
""")


@pytest.mark.timeout(120)
def test_ladder_deadline_kills_and_skips(tmp_path):
    """An attempt still running at the deadline is killed ("deadline") and no further rung is
    tried (skipped: "deadline"); rank 0 prints one line."""
    script = tmp_path / "sup.py"
    script.write_text(DEADLINE_SCRIPT.format(root=ROOT, deadline=6))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), str(script)],
                       env=_env(tmp_path), capture_output=True, text=True, timeout=110)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    att = json.loads(lines[0])["attempts"]
    assert att[0]["rung"] == "a" and not att[0]["ok"]
    assert set(att[0]["rc"].values()) <= {"deadline", "killed"} and \
        "deadline" in att[0]["rc"].values(), att
    assert att[1] == {"rung": "b", "ok": False, "skipped": "deadline"}, att


@pytest.mark.timeout(120)
def test_ladder_sigterm_still_prints_one_line(tmp_path):
    """The driver ends an overrunning bench with SIGTERM: rank 0's supervisor must still print
    exactly one JSON line (marked terminated) and take its child down."""
    import signal
    import time

    script = tmp_path / "sup.py"
    script.write_text(DEADLINE_SCRIPT.format(root=ROOT, deadline=600))
    p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(_port()), str(script)],
                         env=_env(tmp_path), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    time.sleep(8)  # supervisors up, first attempt's children running
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=90)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (out, err[-3000:])
    assert json.loads(lines[0])["terminated"] == "terminated"


def test_fan_rungs():
    from docker_dist_nn_amd.ladder import bench_rungs

    names = [r.name for r in bench_rungs(8, fan=True)]
    assert names == ["default", "fan-rccl", "fan-python", "uniform-rccl-slotted",
                     "uniform-python", "dp-native", "dp-python"]
    assert "--parallelism" in bench_rungs(8, fan=True)[3].args


# Main measurement + two comparisons (bench.py supervise: the literal uniform pipeline, then
# data parallelism), each run only while the deadline leaves room for one more attempt.
COMPARE_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, {root!r})
    from docker_dist_nn_amd import ladder
    rank = int(os.environ["RANK"])
    if ladder.is_child():
        ladder.heartbeat("start")
        rung = os.environ[ladder.RUNG_ENV]
        time.sleep({child_s} if rung.startswith("u") else 0.2)
        ladder.write_result({{"rung": rung, "value": len(rung)}})
        sys.exit(0)
    world = int(os.environ["WORLD_SIZE"])
    sup = ladder.Supervisor(lambda r: [sys.executable, __file__], rank=rank, world=world,
                            stall=30.0, deadline=time.monotonic() + float({deadline}))
    res, rung = sup.climb([ladder.Rung("main")])
    seen = []
    out = sup.comparisons([("uniform_pipeline", [ladder.Rung("u1")]),
                           ("dp_only", [ladder.Rung("dp1")])], need_s=float({need}),
                          on_done=lambda k, e: seen.append(k))
    print(json.dumps({{"rank": rank, "res": res, "out": out, "seen": seen}}), flush=True)
""")


def _compare_run(tmp_path, deadline, need, child_s):
    script = tmp_path / "cmp.py"
    script.write_text(COMPARE_SCRIPT.format(root=ROOT, deadline=deadline, need=need,
                                            child_s=child_s))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), str(script)],
                       env=_env(tmp_path), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = sorted((json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")),
                  key=lambda x: x["rank"])
    assert [x["rank"] for x in recs] == [0, 1]
    assert recs[0]["out"].keys() == recs[1]["out"].keys()
    for k in recs[0]["out"]:  # every rank took the same decision
        assert ("skipped" in recs[0]["out"][k]) == ("skipped" in recs[1]["out"][k])
    return recs[0]


@pytest.mark.timeout(120)
def test_comparisons_all_run_when_time_allows(tmp_path):
    r = _compare_run(tmp_path, deadline=100, need=5, child_s=0.2)
    assert r["res"]["rung"] == "main"
    assert r["out"]["uniform_pipeline"]["result"] == {"rung": "u1", "value": 2}
    assert r["out"]["dp_only"]["result"] == {"rung": "dp1", "value": 3}
    assert r["seen"] == ["uniform_pipeline", "dp_only"]


@pytest.mark.timeout(120)
def test_comparisons_skip_past_the_budget(tmp_path):
    """The uniform measurement runs (enough time left), takes long, and the data-parallel
    comparison is then skipped for the budget -- on every rank."""
    r = _compare_run(tmp_path, deadline=14, need=6, child_s=7)
    assert r["out"]["uniform_pipeline"]["result"]["rung"] == "u1"
    assert r["out"]["dp_only"]["skipped"] == "budget"
    assert r["out"]["dp_only"]["seconds_left"] < 6


@pytest.mark.timeout(120)
def test_comparisons_all_skipped_without_time(tmp_path):
    r = _compare_run(tmp_path, deadline=100, need=1000, child_s=0.2)
    assert all(e["skipped"] == "budget" for e in r["out"].values())


def test_uniform_rungs():
    from docker_dist_nn_amd.ladder import uniform_rungs

    rr = uniform_rungs()
    assert [r.name for r in rr] == ["uniform", "uniform-rccl-slotted", "uniform-python"]
    assert all(r.args[:2] == ["--parallelism", "uniform"] for r in rr)
