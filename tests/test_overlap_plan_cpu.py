"""Plan transformations of the single-stage overlap plans (parallel/pipeline.py), without a GPU:
overlap mode 5 orders every side wgrad after the dgrad producing its input, and the cross-step
form keeps the waits the next step needs."""
from docker_dist_nn_amd.parallel.pipeline import PipelineExecutor


class _Prog:
    def __init__(self, sizes):
        self.sizes = sizes

    def segment_size(self, name):
        return self.sizes.get(name, 0)


class _Stage:
    def __init__(self, sizes):
        self._prog = _Prog(sizes)


# the headline's shape: the classifier tail already ran the dgrads of layers 3 and 2, so their
# segments are empty
SIZES = {"F0": 4, "B0.L3": 0, "B0.L2": 0, "B0.L1": 1, "W3": 1, "W2": 1, "W1": 1}


def _mode5(sizes, L):
    st = _Stage(sizes)
    return [e[1] for e in PipelineExecutor._mode5_head(st, L)]


def test_mode5_forks_after_each_dgrad_a_side_wgrad_reads():
    """overlap mode 5 put every small wgrad on the side stream behind ONE fork after
    F0, but W_i reads dZ_i, which B0.L{i+1} writes. Every side W_i whose dgrad is real must come
    after that dgrad and a fork on the main stream."""
    L = 6
    sizes = {"F0": 4, **{f"B0.L{i}": 1 for i in range(1, L)}, **{f"W{i}": 1 for i in range(L)}}
    out = _mode5(sizes, L)
    for i in range(2, L - 1):
        b, w = out.index(f"B0.L{i + 1}"), out.index(f"W{i}")
        assert b < w and "@fork" in out[b:w], (i, out)
    # every dgrad exactly once, in order
    assert [s for s in out if s.startswith("B0")] == [f"B0.L{i}" for i in range(L - 1, 0, -1)]
    assert out.index(f"W{L - 1}") > out.index("@fork") > out.index("F0")


def test_mode5_with_tail_keeps_one_fork():
    """The headline's tail already ran the dgrads of layers 3 and 2 (empty segments): their
    wgrads read dZ written by F0, so one fork suffices, as before."""
    out = _mode5(SIZES, 4)
    assert out.count("@fork") == 1
    assert out == ["F0", "@fork", "W3", "B0.L3", "W2", "B0.L2", "B0.L1"]


class _XProg(_Prog):
    def segments(self):
        return ["F0", "F0.L0", "F0.L1", "F0.L2", "F0.L3"]


class _XStage:
    def __init__(self, h0_double):
        self._prog = _XProg({})
        self.geoms = [None] * 4
        self.h0_double = h0_double


def _xplan(h0_double):
    ex = PipelineExecutor.__new__(PipelineExecutor)
    st = _XStage(h0_double)
    ex.stages = [st]
    plan = [(st, "F0", 0), (None, "@fork", 0), (st, "W3", 1), (st, "B0.L3", 0),
            (None, "@fork", 0), (st, "W2", 1), (st, "B0.L2", 0), (None, "@fork", 0),
            (st, "W1", 1), (st, "B0.L1", 0), (None, "@fork", 0), (st, "FINO1-3", 1),
            (st, "W0", 0), (st, "FINO0-0", 0), (None, "@join", 0)]
    first = [e[1] for e in ex._xstep_plan(plan)]
    return first, [e[1] for e in ex._xstep_plan(plan)]


def test_cross_step_plan_waits_for_the_side_wgrads_unless_h0_is_double_buffered():
    """DNN_XSTEP: the next step's layer-0 forward waits for this step's side-stream wgrads
    ("@xwait:w": W1 reads the activation it overwrites) -- unless that activation alternates
    between two buffers (DNN_H0_DOUBLE); the layer-1 forward always waits for the side
    stream's end (the updated W_1). The first step has nothing to wait for."""
    first, steady = _xplan(False)
    assert not any(s.startswith("@xwait") for s in first)
    assert steady[:3] == ["@xwait:w", "F0.L0", "@xwait:end"] and steady[-1] == "@xmark:end"
    assert steady.index("@xmark:w") == steady.index("W1") + 1
    first, steady = _xplan(True)
    assert steady[:2] == ["F0.L0", "@xwait:end"] and "@xmark:w" not in steady
    assert "@join" not in steady and steady[-1] == "@xmark:end"
