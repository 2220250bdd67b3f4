"""Kernel names hipBLASLt picks for the step / wide-model shapes (run under rocprofv3)."""
import torch

dev = torch.device("cuda")
for (M, K, N) in [(65536, 832, 512), (65536, 512, 256), (16384, 8192, 8192)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    dz = torch.randn(M, N, device=dev).to(torch.bfloat16)
    for _ in range(3):
        torch.mm(x, w.t())   # fwd
        torch.mm(dz, w)      # dgrad
        torch.mm(dz.t(), x)  # wgrad
    torch.cuda.synchronize()
