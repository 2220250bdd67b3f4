"""hipBLASLt weight-gradient orientation probe: dW = dZ^T X (our [N][K] layout, the library's
slow transposed-A solution) against dW^T = X^T dZ (its [K][N] mirror), bf16 in, fp32 out, and
our split-K MFMA wgrad, for the BASELINE wgrad shapes. One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from docker_dist_nn_amd import ops  # noqa: E402
from stage_sweep import timeit  # noqa: E402

dev = torch.device("cuda")
for (R, K, N) in [(65536, 1024, 1024), (65536, 832, 1024), (65536, 832, 512), (16384, 8192, 8192)]:
    x = torch.randn(R, K, device=dev).to(torch.bfloat16)
    dz = torch.randn(R, N, device=dev).to(torch.bfloat16)
    g = torch.empty(N, K, device=dev)
    gt = torch.empty(K, N, device=dev)
    a = timeit(lambda: ops.blas_gemm(dz, x, g, trans_a=True, trans_b=False, M=N, N=K, K=R), 10)
    b = timeit(lambda: ops.blas_gemm(x, dz, gt, trans_a=True, trans_b=False, M=K, N=N, K=R), 10)
    bm, bn, s = ops.wgrad_config(N, K, R)
    slabs = torch.empty(s, N, K, device=dev)
    c = timeit(lambda: ops.linear_wgrad(dz, x, slabs, splits=s), 10)
    print(json.dumps({"R": R, "K": K, "N": N, "blas_dW_us": round(a, 1),
                      "blas_dWT_us": round(b, 1), "ours_us": round(c, 1), "splits": s}),
          flush=True)
