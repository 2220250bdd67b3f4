"""Cost of L2-uncached operands (utils/devmem.py: the IPC receive buffers) for the GEMMs that
read them: the headline forward / dgrad / wgrad shapes with the A operand in normal vs uncached
memory (and vs fine-grained, if available), one process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from docker_dist_nn_amd.ops.kernels import KMAJ, MNMAJ  # noqa: E402
from docker_dist_nn_amd.utils.devmem import uncached_zeros  # noqa: E402

dev = torch.device("cuda")


def t_us(fn, iters=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(rounds):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return round(statistics.median(ts), 2)


M, K, N = 16384, 512, 256  # a pp4 micro-batch of the headline's 512->256 layer
for where in ("normal", "uncached"):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    if where == "uncached":
        xu = uncached_zeros((M, K), torch.bfloat16, dev)
        xu.copy_(x)
        x = xu
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fwd = t_us(lambda: ops.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=b,
                                act="relu", tiles=(256, 256), stages=9))
    dz = torch.randn(M, N, device=dev).to(torch.bfloat16)
    slabs = torch.empty(16, N, K, device=dev)
    wg = t_us(lambda: ops.gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K, K=0,
                               k_total=M, splits=16, tiles=(128, 128), stages=9))
    cp = torch.empty_like(x)
    copy = t_us(lambda: cp.copy_(x))
    print(json.dumps({"A_in": where, "fwd_us": fwd, "wgrad_us": wg, "copy_us": copy,
                      "bytes": x.numel() * 2}), flush=True)
