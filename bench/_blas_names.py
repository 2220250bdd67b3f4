import torch
d = torch.device("cuda")
for (M, K, N) in [(65536, 832, 512), (65536, 1024, 1024), (65536, 512, 256), (65536, 64, 1024)]:
    x = torch.randn(M, K, device=d).bfloat16(); w = torch.randn(N, K, device=d).bfloat16()
    for _ in range(5): torch.mm(x, w.t())
    dz = torch.randn(M, N, device=d).bfloat16()
    for _ in range(5): torch.mm(dz, w)
torch.cuda.synchronize()
