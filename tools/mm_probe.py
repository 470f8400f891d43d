#!/usr/bin/env python3
"""Library reference for the halo GEMM: torch.matmul (hipBLASLt) on the plain GEMMs with the level-0 /
level-2 conv shapes (M = B*H*W pixels, K = 9*Cin, N = Cout; the im2col matrix is given, i.e. without
the 9x gather, the GroupNorm transform, the epilogue or the statistics the halo kernel fuses) and a
square 8192^3 GEMM.  Random bf16 data, HIP events, median of 10.  Prints one JSON line per shape."""
import json

import torch


def main():
    d = "cuda"
    for (M, K, N, what) in [(4194304, 1152, 128, "level-0 conv 128->128 as a plain GEMM"),
                            (4194304, 2304, 128, "level-0 up-path conv 256->128 as a plain GEMM"),
                            (262144, 2304, 256, "level-2 conv 256->256 as a plain GEMM"),
                            (8192, 8192, 8192, "square")]:
        a = torch.randn(M, K, device=d).bfloat16()
        b = torch.randn(K, N, device=d).bfloat16()
        for _ in range(3):
            c = a @ b
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            c = a @ b
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[len(ts) // 2]
        print(json.dumps({"M": M, "K": K, "N": N, "what": what, "ms": ms, "tflops": 2 * M * K * N / ms / 1e9,
                          "frac_of_2500": 2 * M * K * N / ms / 1e9 / 2500}), flush=True)
        del a, b, c


if __name__ == "__main__":
    main()
