#!/usr/bin/env python3
"""hipBLASLt (torch.matmul, bf16) on the GEMM shapes of the ResNet-50 1x1 convolutions: the library's
achievable TFLOP/s for the same M/N/K, as a yardstick for the implicit-GEMM conv kernels."""
import time

import torch

B = 256
SHAPES = [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (28, 256, 512), (14, 256, 1024),
          (14, 1024, 256), (14, 512, 1024), (7, 512, 2048), (7, 2048, 512), (7, 1024, 2048),
          (28, 1152, 128), (14, 2304, 256), (7, 4608, 512)]  # last three: 3x3 convs as GEMM K=9C


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


for H, C, K in SHAPES:
    M = B * H * H
    a = torch.randn(M, C, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(C, K, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: a @ w)
    print("H%-3d M=%-7d K(red)=%-5d N=%-5d %7.1f us %6.0f TF" % (H, M, C, K, t * 1e6, 2 * M * C * K / t / 1e12), flush=True)
