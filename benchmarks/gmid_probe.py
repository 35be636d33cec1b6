"""Tiny driver for PMC passes over the mid-M GEMM (gemm_mid.hip): a few launches of each variant on
one shape, nothing else on the GPU.  ``python benchmarks/gmid_probe.py --shape 768,4096,4096``."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="768,4096,4096")
    ap.add_argument("--variants", default="0,64,1064")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--g256", action="store_true")
    a = ap.parse_args()
    M, N, K = map(int, a.shape.split(","))
    torch.manual_seed(0)
    A = ((torch.rand((M, K), device="cuda") * 2 - 1)).to(torch.bfloat16)
    W = ops.shuffle_weights(((torch.rand((N, K), device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16))
    out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    for v in map(int, a.variants.split(",")):
        for _ in range(a.iters):
            ops.kernels.gemm_mid(A, W, out=out, variant=v)
    if a.g256 and ops.native().gemm256_ok(M, N, K, K, K):
        for _ in range(a.iters):
            ops.kernels.gemm256(A, W, shuffled=True)
    torch.cuda.synchronize()
    print("done", M, N, K)


if __name__ == "__main__":
    main()
