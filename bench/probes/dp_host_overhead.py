"""Host cost of the data-parallel step path on ONE GPU: the per-op executor with the deferred
DP update (split forward, split optimizer segments, bucketed wgrad+reduce, all-reduce launch
points) but a no-op all-reduce, against the one-call native plan of the plain 1-GPU step. If
the two match, the host issues the DP step faster than the GPU runs it (the comm itself is
RCCL's, measured only on a multi-GPU node)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from docker_dist_nn_amd import NAMED_MODELS  # noqa: E402
from docker_dist_nn_amd.data import DeviceDataset, synthetic_mnist  # noqa: E402
from docker_dist_nn_amd.engine import OptimConfig, Trainer  # noqa: E402
from docker_dist_nn_amd.parallel import pipeline as pl  # noqa: E402


class NoComm:
    world = 2

    def launch(self, flat, a, b):
        return None

    def wait(self):
        pass

    def wait_one(self, w):
        pass


def run(fake_dp: bool, steps=200, warmup=20):
    dev = torch.device("cuda")
    tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=65536, num_micro=1,
                 optim=OptimConfig(lr=0.05), device=dev)
    if fake_dp:
        ex = tr.executor
        ex.grad_sync = NoComm()
        ex.defer = True
        ex._split = {id(st): pl.dp_split(st) for st in tr.stages}
        ex._plan = None  # the one-call plan applies only without a DP group
    x, y = synthetic_mnist(131072, seed=1)
    data = DeviceDataset(x, y, 65536, dev, kp=tr.stages[0].x_in.shape[1])
    for i in range(warmup):
        tr.set_batch(*data.batch(i), zero_copy=True)
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for i in range(steps):
        h0 = time.perf_counter()
        tr.set_batch(*data.batch(i), zero_copy=True)
        tr.step()
        host += time.perf_counter() - h0
    tr.flush()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"path": "deferred-dp (no-op comm)" if fake_dp else "native plan",
            "ms_per_step": round(el / steps * 1e3, 4),
            "host_issue_ms_per_step": round(host / steps * 1e3, 4)}


if __name__ == "__main__":
    for f in (False, True, False, True):
        print(json.dumps(run(f)), flush=True)
