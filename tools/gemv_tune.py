#!/usr/bin/env python3
"""GEMV (decode rows M ≤ 8) timing with COLD weights: each launch reads a different copy of the matrix (≥ 1 GB of
copies, beyond the 256 MB MALL), as in a real decode step where every layer's weights stream from HBM once.
PATHS: 1 = auto, 3 / 4 / 5 = 1 / 2 / 4 output columns per wave.  Prints µs per launch and HBM GB/s."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = [("qkv", 4096, 2048, 0), ("o", 2048, 2048, 1), ("gu", 12288, 2048, 0), ("down", 2048, 6144, 1),
          ("lm", 151936, 2048, 0)]
PATHS = [int(p) for p in os.environ.get("PATHS", "3,4,5").split(",")]
ROWS = [int(m) for m in os.environ.get("ROWS", "1,2,4,8").split(",")]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    for tag, N, K, epi in SHAPES:
        copies = max(2, math.ceil(1.2e9 / (N * K)))
        wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
        ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
        for M in ROWS:
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            y = torch.zeros(M, N, device=dev)
            out = []
            for path in PATHS:
                def run(i):
                    _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                     ws[i].data_ptr(), N, K, None,
                                                     y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, path,
                                                     None))
                for i in range(copies):
                    run(i)
                torch.cuda.synchronize()
                reps = max(1, 200 // copies)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    for i in range(copies):
                        run(i)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / (reps * copies)
                gbs = N * K * (1 + 2 / 32) / us / 1e3
                out.append(f"{path}: {us:7.2f}us {gbs:6.0f}GB/s")
            print(f"{tag:5s} M={M} N={N:6d} K={K} | " + "  ".join(out), flush=True)
        del wq, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
