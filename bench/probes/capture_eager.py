"""Capture after eager steps vs all-eager: is the graph step bitwise the eager step, with and
without DNN_XSTEP / DNN_H0_DOUBLE? (diagnosis of tests/test_overlap_gpu.py)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def run(xstep, dbl, capture_after):
    os.environ.update(DNN_BW_OVERLAP_MIN_ROWS="0", DNN_SPLIT_FINO="1", DNN_XSTEP=xstep,
                      DNN_H0_DOUBLE=dbl)
    from docker_dist_nn_amd import NAMED_MODELS
    from docker_dist_nn_amd.data import synthetic_mnist
    from docker_dist_nn_amd.engine import OptimConfig, Trainer

    dev = torch.device("cuda", 0)
    rows = 8192
    x, y = synthetic_mnist(rows, seed=11)
    xb = torch.zeros(rows, 832, dtype=torch.bfloat16)
    xb[:, :784] = torch.from_numpy(x).to(torch.bfloat16)
    xb, yb = xb.to(dev), torch.from_numpy(y).to(dev)
    tr = Trainer(NAMED_MODELS["mnist-fcnn"], micro_batch=rows, num_micro=1, seed=0,
                 optim=OptimConfig(lr=0.1, momentum=0.9), device=dev)
    for k in range(5):
        if capture_after is not None and k == capture_after:
            tr.set_batch(xb, yb)
            tr.capture(warmup=0, copies=1)
            continue
        tr.set_batch(xb, yb)
        tr.step()
    tr.flush()
    torch.cuda.synchronize()
    return tr.stages[0].params.master.clone()


ref = {}
for xs, dbl in (("0", "0"), ("1", "0"), ("1", "1")):
    a = run(xs, dbl, None)
    for cap in (0, 2):
        b = run(xs, dbl, cap)
        print(f"xstep={xs} h0_double={dbl} capture_at={cap}: bitwise={torch.equal(a, b)} "
              f"maxdiff={float((a - b).abs().max()):.3g}", flush=True)
