"""The native multi-rank step plans (parallel/native_step.py) on the CPU, for layouts the
one-GPU pool cannot run.

Every rank's StepPlan op list is built exactly as on a GPU (NativeStep._build over the real
schedule, the real StageParams flat layout of the stage's layers, and the IpcPipe flag / relay
layout), with fake device addresses for the activation buffers and fake communicator handles,
then executed by the timed plan simulator (parallel/plan_sim.py): per-stream FIFO order, event
edges, fork/join per plan run, RCCL point-to-point as blocking FIFO rendezvous per (communicator,
src, dst), RCCL groups, collectives as barriers over their communicator, IPC flags.

Checked, for every BASELINE layout (pp2, pp4, pp8, pp4dp2, pp2dp4) x hop format (bf16, fp8) x
DP exchange (sharded, all-reduce):
* deadlock freedom of both RCCL plan forms; the ``slotted`` form also with at most ONE RCCL
  kernel resident per rank (``serial_rccl``);
* the steady-state period per micro-batch of the ``streams`` form is max(compute, hop): the
  hop-in of micro-batch j+1 overlaps j's compute and hop-out;
* every WAIT is enqueued after the REC it names (a HIP event wait binds to the last record);
* the sharded DP collectives' pointers and counts equal GradSync's tensor slices for every
  replica (RS into grad_piece + e0/d, in-place AG shadow + p0 -> shadow + e0).
"""
from types import SimpleNamespace as NS

import pytest
import torch

from docker_dist_nn_amd import MLPSpec
from docker_dist_nn_amd.engine.stage import OptimConfig, StageParams
from docker_dist_nn_amd.models.mlp import LayerGeom
from docker_dist_nn_amd.parallel import native_step as nsmod
from docker_dist_nn_amd.parallel import plan_sim
from docker_dist_nn_amd.parallel.comm import (IpcPipe, RelayLayout, relay_assignment,
                                               relay_parts, relay_plan)
from docker_dist_nn_amd.parallel.pipeline import schedule_ops
from docker_dist_nn_amd.partition import plan_stages


class FakeTensor:
    def __init__(self, base, rows, cols, esize=2):
        self.base, self.rows, self.cols, self.esize = base, rows, cols, esize

    def __getitem__(self, sl):
        return FakeTensor(self.base + sl.start * self.cols * self.esize, sl.stop - sl.start,
                          self.cols, self.esize)

    def data_ptr(self):
        return self.base

    def numel(self):
        return self.rows * self.cols

    def element_size(self):
        return self.esize

    def stride(self, d):
        return self.cols if d == 0 else 1


KEYS = ["x_in", "grad_out", "output", "dx_send", "flags", "q_in", "s_in", "q_gin", "s_gin",
        "q_out", "s_out", "q_dx", "s_dx"] + [f"relay{i}" for i in range(16)]


def _addr(rank, key):
    return (rank + 1) << 40 | (KEYS.index(key) + 1) << 32


class FakeProg:
    def segments(self):
        return {"FINO", "W"}


def _stage(rank, pp, dp, nm, mb, spec, dist, boundary, dp_reduce):
    stage, replica = rank % pp, rank // pp
    plan = plan_stages(len(spec.layers), dist)[stage]
    geoms = [LayerGeom(i, spec.layers[i]) for i in range(plan.layer_start, plan.layer_end)]
    shard = (dp, replica) if dp_reduce == "shard" and dp > 1 else None
    params = StageParams(geoms, torch.device("cpu"), OptimConfig(), shard=shard)
    rows = mb * nm
    w_in, w_out = geoms[0].kp, geoms[-1].np_
    st = NS(nm=nm, mb=mb, boundary=boundary, _has_w=True, _o_native=True, _prog=FakeProg(),
            params=params, geoms=geoms, rows_of=lambda j: slice(j * mb, (j + 1) * mb))
    for key, w, es in (("x_in", w_in, 2), ("grad_out", w_out, 2), ("output", w_out, 2),
                       ("dx_send", w_in, 2), ("q_in", w_in, 1), ("s_in", 1, 4),
                       ("q_gin", w_out, 1), ("s_gin", 1, 4), ("q_out", w_out, 1),
                       ("s_out", 1, 4), ("q_dx", w_in, 1), ("s_dx", 1, 4)):
        setattr(st, key, FakeTensor(_addr(rank, key), rows, w, es))
    mesh = NS(rank=rank, pp=pp, dp=dp, stage=stage, replica=replica,
              prev_rank=rank - 1 if stage > 0 else None,
              next_rank=rank + 1 if stage + 1 < pp else None)
    return st, mesh


def _comms(mesh):
    r = mesh.rank
    c = {"dp": ("dp", mesh.stage)}
    if mesh.prev_rank is not None:
        c["f_in"], c["b_out"] = ("lf", mesh.prev_rank, r), ("lb", mesh.prev_rank, r)
    if mesh.next_rank is not None:
        c["f_out"], c["b_in"] = ("lf", r, mesh.next_rank), ("lb", r, mesh.next_rank)
    return c


def build_rccl(rank, pp, dp, nm, mb=256, spec="784-512-256-128-10", dist=None,
               boundary="bf16", dp_reduce="shard", mode="streams", sched="1f1b"):
    spec = MLPSpec.parse(spec)
    dist = dist or [len(spec.layers) // pp] * (pp - 1) + [len(spec.layers) - (pp - 1) *
                                                         (len(spec.layers) // pp)]
    st, mesh = _stage(rank, pp, dp, nm, mb, spec, dist, boundary, dp_reduce)
    ex = NS(stages=[st], ops=[schedule_ops(sched, pp, nm, mesh.stage)], kind=sched)
    return nsmod.NativeStep(ex, mesh, "rccl", comms=_comms(mesh), mode=mode, build_only=True)


def build_ipc(rank, pp, dp, nm, mb, k, width, sched, mode=None):
    """k: relays per hop (relay_assignment), or a per-hop table (relay_plan); mode: the IPC
    plan form (streams | slotted)."""
    spec = MLPSpec.parse("-".join([str(width)] * (pp + 1)))
    st, mesh = _stage(rank, pp, dp, nm, mb, spec, [1] * pp, "bf16", "allreduce")
    st._prog = NS(segments=lambda: {"FINO", "W"})
    assign = k if isinstance(k, dict) else (relay_assignment(pp, dp, k) if k else {})
    lay = RelayLayout(assign, rank, mesh.prev_rank, mesh.next_rank, nm, mb)
    ipc = NS(k=lay.kmax, nm=nm, seq=0, layout=lay, k_in=lay.k_in, k_out=lay.k_out,
             duties=lay.duties, ackf=lay.ackf, ackb=lay.ackb)
    for f in ("fidx", "bidx", "ridx"):
        setattr(ipc, f, getattr(IpcPipe, f).__get__(ipc))
    ipc.flags = FakeTensor(_addr(rank, "flags"), 1, 1, 4)
    ipc.row_bytes_f = ipc.row_bytes_b = width * 2
    ipc.duty_part_max = [lay.part_max(kk) for kk in lay.duty_k]
    ipc.relay_bufs = [(FakeTensor(_addr(rank, f"relay{d}"), 1, 1, 1), width * 2)
                      for d in range(len(ipc.duties))]

    def peer(r):
        if r is None:
            return None
        return {"x_in": _addr(r, "x_in"), "grad_out": _addr(r, "grad_out"),
                "flags": _addr(r, "flags")}

    ipc.prev, ipc.next = peer(mesh.prev_rank), peer(mesh.next_rank)

    ipc.relay_out = {"f": [], "b": []}
    for d, pr in (("f", mesh.next_rank), ("b", mesh.prev_rank)):
        if pr is None:
            continue
        for r in assign.get((rank, pr, d), []):
            di = lay.duty_index(r, (rank, pr, d))
            ipc.relay_out[d].append({"buf": _addr(r, f"relay{di}"), "flags": _addr(r, "flags"),
                                     "d": di, "part_max": lay.part_max(lay.k_out[d])})
    ipc.relay_dst = [{"buf": _addr(dst, "x_in" if d == "f" else "grad_out"),
                      "flags": _addr(dst, "flags")} for _s, dst, d, _p in ipc.duties]
    ex = NS(stages=[st], ops=[schedule_ops(sched, pp, nm, mesh.stage)], kind=sched)
    return nsmod.NativeStep(ex, mesh, "ipc", ipc=ipc, build_only=True, mode=mode)


def check_enqueue_order(ops):
    """Every WAIT on an event is enqueued after a REC of it; every event id is recorded once."""
    recorded = set()
    for o in nsmod.flatten(ops):
        if o["kind"] == nsmod.REC:
            assert o["event"] not in recorded, f"event {o['event']} recorded twice"
            recorded.add(o["event"])
        elif o["kind"] == nsmod.WAIT:
            assert o["event"] in recorded, f"WAIT on event {o['event']} before its REC"


def sim(builds, steps=2, serial=False, f=1.0, b=2.0, hop=1.0, w=0.25, coll=0.5):
    def seg_time(rank, seg):
        if seg[0] == "F" and seg[1:].isdigit():
            return f
        if seg[0] == "B" and seg[1:].isdigit():
            return b
        if seg.startswith(("W", "FIN")):
            return w
        return 0.01

    plans = {r: plan_sim.RankPlan(ns.ops, ns.n_streams) for r, ns in builds.items()}
    return plan_sim.simulate(plans, steps=steps, seg_time=seg_time,
                             p2p_time=lambda op: hop / (2 if op["dtype"] != nsmod.NCCL_BF16
                                                         else 1),
                             coll_time=lambda op: coll, serial_rccl=serial)


LAYOUTS = [(2, 1), (4, 1), (8, 1), (4, 2), (2, 4)]


def _spec(pp):
    return "784-1024-1024-1024-1024-1024-1024-1024-10" if pp == 8 else "784-512-256-128-10"


@pytest.mark.parametrize("pp,dp", LAYOUTS)
@pytest.mark.parametrize("boundary", ["bf16", "fp8"])
@pytest.mark.parametrize("dp_reduce", ["shard", "allreduce"])
@pytest.mark.parametrize("mode", ["streams", "slotted"])
def test_rccl_plans_deadlock_free(pp, dp, boundary, dp_reduce, mode):
    nm = 2 * pp
    builds = {r: build_rccl(r, pp, dp, nm, spec=_spec(pp), boundary=boundary,
                            dp_reduce=dp_reduce, mode=mode) for r in range(pp * dp)}
    for ns in builds.values():
        check_enqueue_order(ns.ops)
    assert sim(builds).makespan > 0
    if mode == "slotted":  # safe with one resident RCCL kernel per rank
        assert sim(builds, serial=True).makespan > 0


def test_streams_form_needs_concurrent_rccl_kernels():
    """The ``streams`` form relies on co-resident RCCL kernels (pre-posted receives): with one
    resident kernel per rank it can deadlock -- why it needs one hardware queue per stream and
    why ``auto`` falls back to ``slotted`` otherwise."""
    pp = 4
    builds = {r: build_rccl(r, pp, 1, 8, mode="streams") for r in range(pp)}
    with pytest.raises(plan_sim.Deadlock):
        sim(builds, serial=True)


@pytest.mark.parametrize("sched", ["gpipe", "1f1b", "1f1b_lh"])
@pytest.mark.parametrize("mode", ["streams", "slotted"])
def test_rccl_plans_per_schedule(sched, mode):
    builds = {r: build_rccl(r, 4, 2, 8, mode=mode, sched=sched) for r in range(8)}
    assert sim(builds, serial=mode == "slotted").makespan > 0


def _period(pp, mode, hop, sched="1f1b_lh", f=1.0, b=2.0):
    """Steady-state time per micro-batch: slope of the step time in the micro-batch count."""
    out = []
    for nm in (16, 32):
        builds = {r: build_rccl(r, pp, 1, nm, spec=_spec(pp), mode=mode, sched=sched)
                  for r in range(pp)}
        res = sim(builds, steps=1, hop=hop, f=f, b=b)
        out.append(res.makespan)
    return (out[1] - out[0]) / 16


@pytest.mark.parametrize("pp", [2, 4, 8])
@pytest.mark.parametrize("hop", [0.5, 3.0, 6.0])
def test_streams_period_is_max_of_compute_and_hop(pp, hop):
    """compute per micro-batch = F + B = 3; hop = one message per direction per micro-batch.
    The streams form with the latency-hiding 1F1B (1f1b_lh) overlaps hop-in, compute and
    hop-out: period = max(3, hop) (planner.Planner's model)."""
    per = _period(pp, "streams", hop)
    assert per <= 1.05 * max(3.0, hop) + 0.05, per


def test_classic_1f1b_exposes_hop_latency():
    """Why 1f1b_lh is the multi-GPU default: classic 1F1B keeps S - s micro-batches in flight,
    which cannot cover a hop of one micro-batch's compute (2.5x slower here)."""
    assert _period(4, "streams", 3.0, sched="1f1b") > 2 * _period(4, "streams", 3.0)


@pytest.mark.parametrize("hop", [0.5, 3.0])
def test_slotted_period_bounded(hop):
    """The slotted form pays for its serial safety: a hop-in waits for the previous group, so
    a micro-batch costs up to compute + hop (never more)."""
    per = _period(4, "slotted", hop)
    assert per <= 3.0 + hop + 0.1, per


@pytest.mark.parametrize("dp", [2, 4])
def test_sharded_collectives_match_gradsync_slices(dp):
    """Every REDUCE_SCATTER / ALL_GATHER of the sharded native plan names exactly the bytes
    GradSync (the Python executor) hands torch.distributed: RS input = grad16[e0:e1], output =
    grad_piece[e0/d : e1/d]; AG input = shadow[p0:p1] (this replica's piece), output =
    shadow[e0:e1] with sendbuff == recvbuff + rank * count (RCCL's in-place condition)."""
    pp = 2
    for r in range(pp * dp):
        ns = build_rccl(r, pp, dp, 4, dp_reduce="shard")
        p = ns.st.params
        replica = r // pp
        rs = [o for o in ns.ops if o["kind"] == nsmod.REDUCE_SCATTER]
        ag = [o for o in ns.ops if o["kind"] == nsmod.ALL_GATHER]
        assert len(rs) == len(ag) == len(p.shard_buckets) > 0
        for o, (e0, e1) in zip(rs, p.shard_buckets):
            src, dst = p.grad16[e0:e1], p.grad_piece[e0 // dp:e1 // dp]
            assert o["a"] == src.data_ptr() and o["b"] == dst.data_ptr()
            assert o["count"] == dst.numel() == src.numel() // dp
        for o, (e0, e1) in zip(ag, p.shard_buckets):
            p0, p1 = p.shard_piece(e0, e1)
            assert (p0, p1) == (e0 + replica * o["count"], e0 + (replica + 1) * o["count"])
            assert o["a"] == p.shadow[p0:p1].data_ptr()
            assert o["b"] == p.shadow[e0:e1].data_ptr()
            assert o["a"] == o["b"] + replica * o["count"] * 2  # bf16 bytes
        ar = [o for o in ns.ops if o["kind"] == nsmod.ALLREDUCE]
        assert len(ar) == 1 and ar[0]["a"] == p.grad[p.bias_lo:].data_ptr()
        assert ar[0]["count"] == p.numel - p.bias_lo


def test_link_channels_one_sender_one_receiver():
    """In the streams form every link communicator carries ONE direction: its sends all come
    from one rank and its receives all land on the other, in micro-batch order on both."""
    pp, dp, nm = 4, 2, 8
    chans = {}
    for r in range(pp * dp):
        ns = build_rccl(r, pp, dp, nm)
        for o in nsmod.flatten(ns.ops):
            if o["kind"] in (nsmod.SEND, nsmod.RECV):
                chans.setdefault(o["comm"], []).append((o["kind"], r, o["tag"]))
    for comm, lst in chans.items():
        senders = {r for k, r, _ in lst if k == nsmod.SEND}
        recvers = {r for k, r, _ in lst if k == nsmod.RECV}
        assert len(senders) == len(recvers) == 1 and senders != recvers, comm
        s_tags = [t for k, _, t in lst if k == nsmod.SEND]
        r_tags = [t for k, _, t in lst if k == nsmod.RECV]
        assert s_tags == r_tags, comm


def test_slotted_groups_match_partner_slots():
    """In the slotted form a rank's group t holds exactly the transfers whose partner op is in
    the partner's group t (what makes it safe with one resident RCCL kernel)."""
    pp, nm = 4, 8
    groups = {}
    for r in range(pp):
        ns = build_rccl(r, pp, 1, nm, mode="slotted")
        for o in ns.ops:
            if o["kind"] == nsmod.GROUP:
                for m in o["ops"]:
                    groups.setdefault((o["tag"], m["tag"]), []).append(
                        (r, m["kind"], m["gpeer"]))
    for key, lst in groups.items():
        assert len(lst) == 2, key
        (r1, k1, p1), (r2, k2, p2) = lst
        assert {k1, k2} == {nsmod.SEND, nsmod.RECV} and p1 == r2 and p2 == r1, key


# ---- IPC transport (xGMI peer copies + flags) ------------------------------------------------
# the headline model's boundaries (512, 256, 128 columns): the planner's per-hop relay table
HEAD_HOPS = [512, 256, 128]


def _plan_table(pp, dp):
    return relay_plan(pp, dp, [w * 2 * 65536 for w in (HEAD_HOPS * 3)[:pp - 1]])


@pytest.mark.parametrize("pp,dp,k", [(2, 1, 0), (3, 1, 0), (4, 1, 0), (3, 1, 1), (4, 1, 2),
                                     (4, 2, 0), (4, 2, 2), (8, 1, 2), (2, 4, 2), (4, 2, 4),
                                     (4, 2, 6), (8, 1, 6), (4, 1, "plan"), (4, 2, "plan"),
                                     (8, 1, "plan"), (2, 4, "plan")])
def test_ipc_plans_deadlock_free(pp, dp, k):
    nm = 2 * pp
    if k == "plan":
        k = _plan_table(pp, dp)
    builds = {r: build_ipc(r, pp, dp, nm, 64, k, 64, "1f1b") for r in range(pp * dp)}
    for ns in builds.values():
        check_enqueue_order(ns.ops)
    assert sim(builds, steps=3).makespan > 0


@pytest.mark.parametrize("sched", ["gpipe", "1f1b"])
def test_ipc_relay_plans_deadlock_free_per_schedule(sched):
    builds = {r: build_ipc(r, 4, 2, 8, 64, 2, 64, sched) for r in range(8)}
    assert sim(builds, steps=3).makespan > 0


@pytest.mark.parametrize("k", [2, 4, 6, "plan"])
def test_relay_stripes_reach_every_row_once(k):
    """Every consumer row of every micro-batch is written by exactly one COPY (direct or
    relayed), for every hop of a pp4 x dp2 mesh with k relays per hop, or the planner's
    per-hop table."""
    pp, dp, nm, mb, width = 4, 2, 4, 64, 64
    if k == "plan":
        k = _plan_table(pp, dp)
    rb = width * 2
    writes = {}
    for r in range(pp * dp):
        ns = build_ipc(r, pp, dp, nm, mb, k, width, "1f1b")
        for o in ns.ops:
            if o["kind"] == nsmod.COPY and (o["b"] >> 32) & 0xff in (1, 2):  # x_in / grad_out
                for row in range(o["count"] // rb):
                    key = (o["b"] >> 32, (o["b"] & 0xffffffff) // rb + row)
                    writes[key] = writes.get(key, 0) + 1
    assert set(writes.values()) == {1}
    # (pp - 1) boundaries x 2 directions x dp replicas x all rows
    assert len(writes) == (pp - 1) * 2 * dp * nm * mb


def test_relay_plan_gives_the_wide_boundary_more_paths():
    """comm.relay_plan: per-hop relay counts from the directed-link load model. At pp4 x dp2 on
    the headline model the 512-column boundary gets more relays than the 128-column one, no
    rank has more duties than allowed, relays never include the hop's own ends, the table is
    deterministic, and the most loaded link carries far less than the un-relayed wide hop."""
    from docker_dist_nn_amd.parallel.comm import relay_link_loads

    hb = [w * 2 * 65536 for w in HEAD_HOPS]
    t = relay_plan(4, 2, hb, max_duties=6)
    assert t == relay_plan(4, 2, hb, max_duties=6)
    k = {h: len(v) for h, v in t.items()}
    assert k[(0, 1, "f")] > k[(2, 3, "f")] and k[(4, 5, "f")] > k[(6, 7, "f")]
    assert max(k.values()) <= 6
    duties = {}
    for (src, dst, _d), rl in t.items():
        assert src not in rl and dst not in rl and len(set(rl)) == len(rl)
        for x in rl:
            duties[x] = duties.get(x, 0) + 1
    assert max(duties.values()) <= 6
    loads = relay_link_loads(4, 2, t, hb)
    assert max(loads.values()) < 0.5 * hb[0]


@pytest.mark.parametrize("pp,dp,k", [(2, 1, 0), (4, 1, 0), (4, 1, 2), (4, 2, 2), (8, 1, 6),
                                     (4, 2, "plan"), (8, 1, "plan"), (2, 4, "plan")])
@pytest.mark.parametrize("sched", ["1f1b", "gpipe", "1f1b_lh"])
def test_ipc_slotted_plans_one_stream_deadlock_free(pp, dp, k, sched):
    """The slotted IPC form (DNN_IPC_PLAN=slotted, the graph-capture form): ONE stream per
    rank in logical-clock order completes -- no wait of a rank precedes, in its own stream,
    the send or relay that another rank's wait needs -- with every relay layout."""
    nm = 2 * pp
    if k == "plan":
        k = _plan_table(pp, dp)
    builds = {r: build_ipc(r, pp, dp, nm, 64, k, 64, sched, mode="slotted")
              for r in range(pp * dp)}
    for ns in builds.values():
        assert ns.mode == "ipc-slotted" and ns.n_streams == 1
        assert {o["stream"] for o in nsmod.flatten(ns.ops)} == {0}
        check_enqueue_order(ns.ops)
    assert sim(builds, steps=3).makespan > 0


def test_ipc_slotted_rows_reach_every_consumer_once():
    """The slotted form moves the same stripes as the streams form."""
    pp, dp, nm, mb, width = 4, 2, 4, 64, 64
    k = _plan_table(pp, dp)
    rb = width * 2
    for mode in ("streams", "slotted"):
        writes = {}
        for r in range(pp * dp):
            for o in build_ipc(r, pp, dp, nm, mb, k, width, "1f1b", mode=mode).ops:
                if o["kind"] == nsmod.COPY and (o["b"] >> 32) & 0xff in (1, 2):
                    for row in range(o["count"] // rb):
                        key = (o["b"] >> 32, (o["b"] & 0xffffffff) // rb + row)
                        writes[key] = writes.get(key, 0) + 1
        assert set(writes.values()) == {1}, mode
        assert len(writes) == (pp - 1) * 2 * dp * nm * mb
