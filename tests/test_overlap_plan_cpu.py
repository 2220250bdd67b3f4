"""Plan transformations of the single-stage overlap plans (parallel/pipeline.py), without a GPU:
fork elision keeps every side-stream ordering the plan needs, and the "@rewait" form keeps the
side stream's waits while the main stream records nothing new."""
from docker_dist_nn_amd.parallel.pipeline import PipelineExecutor


class _Prog:
    def __init__(self, sizes):
        self.sizes = sizes

    def segment_size(self, name):
        return self.sizes.get(name, 0)


class _Stage:
    def __init__(self, sizes):
        self._prog = _Prog(sizes)


# the headline's default plan: the classifier tail already ran the dgrads of layers 3 and 2,
# so their segments are empty
PLAN = [("st", "F0", 0), (None, "@fork", 0), ("st", "W3", 1), ("st", "B0.L3", 0),
        (None, "@fork", 0), ("st", "W2", 1), ("st", "B0.L2", 0), (None, "@fork", 0),
        ("st", "W1", 1), ("st", "B0.L1", 0)]
SIZES = {"F0": 4, "B0.L3": 0, "B0.L2": 0, "B0.L1": 1, "W3": 1, "W2": 1, "W1": 1}


def _elide(rewait):
    st = _Stage(SIZES)
    plan = [(st if e[0] == "st" else None, e[1], e[2]) for e in PLAN]
    return [e[1] for e in PipelineExecutor._elide_forks(st, plan, rewait=rewait)]


def test_forks_after_empty_main_segments_are_dropped():
    assert _elide(False) == ["F0", "@fork", "W3", "B0.L3", "W2", "B0.L2", "W1", "B0.L1"]


def test_rewait_keeps_side_waits_without_main_records():
    out = _elide(True)
    assert out.count("@fork") == 1 and out.count("@rewait") == 2
    assert out.index("@rewait") < out.index("W2") < out.index("W1")


def test_fork_after_real_main_work_is_kept():
    st = _Stage(dict(SIZES, **{"B0.L3": 2}))  # a dgrad that really runs between the forks
    plan = [(st if e[0] == "st" else None, e[1], e[2]) for e in PLAN]
    out = [e[1] for e in PipelineExecutor._elide_forks(st, plan)]
    assert out == ["F0", "@fork", "W3", "B0.L3", "@fork", "W2", "B0.L2", "W1", "B0.L1"]
