"""Reference point: torch (hipBLASLt) fp16 GEMM throughput at the BERT projection shapes.
Usage: python tools/blas_ref.py [M]"""
import sys

import torch


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    dev = torch.device("cuda", 0)
    for N, K in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        A = torch.randn(M, K, device=dev, dtype=torch.float16)
        W = torch.randn(N, K, device=dev, dtype=torch.float16)
        b = torch.randn(N, device=dev, dtype=torch.float16)
        res = []
        for _ in range(5):
            for _ in range(3):
                torch.nn.functional.linear(A, W, b)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                torch.nn.functional.linear(A, W, b)
            e1.record()
            torch.cuda.synchronize()
            res.append(2.0 * M * N * K / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e12)
        print(f"torch linear fp16 M={M} N={N} K={K}: median {sorted(res)[2]:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
