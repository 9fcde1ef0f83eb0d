"""Which hipBLASLt kernels torch.matmul runs on the bf16 encoder GEMM shapes (for the kernel-name
fields: macro tile, depth, waves, LDS use). Run under rocprofv3 --kernel-trace; comparison only."""
import torch

for M, N, K in ((100864, 3072, 768), (65536, 2304, 768), (100864, 768, 3072)):
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(3):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
