#!/usr/bin/env python3
"""Run one Q8 GEMM shape/path N times (for rocprofv3 counter passes): gemm_one.py M N K epi path [iters]."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402


def main():
    M, N, K, epi, path = (int(a) for a in sys.argv[1:6])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
    lib = _lib.load()
    dev = torch.device("cuda:0")
    xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    xd = torch.rand(M, K // 32, device=dev) * 0.01
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
    ws = (torch.rand(N, K // 32, device=dev) * 0.01).half()
    y = torch.zeros(M, N, device=dev)
    for _ in range(iters):
        _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq.data_ptr(), ws.data_ptr(), N, K, None,
                                         y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, path, None))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
