#!/usr/bin/env python3
"""Decode-shape Q8 GEMM timing with COLD weights (tuning aid, GPU).

A decode step streams 28 layers' weights (1.8 GB for 1.7B), so no layer's panel is cache-resident when its GEMM
runs.  Here every launch reads a different copy of the weights from a ring of copies larger than the 256 MiB
Infinity Cache; activations are reused (they are the previous kernel's fresh output in the real loop).
usage: python tools/dec_gemm_tune.py [M ...]      PATHS env: comma list (2 = heuristic, 16+cfg+32·splits forced)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = [("qkv", 4096, 2048, 0), ("o", 2048, 2048, 1), ("gu", 12288, 2048, 3), ("down", 2048, 6144, 1),
          ("lm", 151936, 2048, 0)]
PATHS = [int(p) for p in os.environ.get("PATHS", "2,62,64,65,66,67,68,69,70,71").split(",")]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    Ms = [int(a) for a in sys.argv[1:]] or [32, 64, 128, 160, 256]
    only = os.environ.get("ONLY")
    for tag, N, K, epi in SHAPES:
        if only and tag not in only.split(","):
            continue
        copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
        wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
        ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
        for M in Ms:
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            y = torch.zeros(M, N, device=dev)
            hq = torch.empty(M, N // 2, dtype=torch.int8, device=dev)
            hd = torch.empty(M, N // 64, device=dev)
            flops = 2.0 * M * N * K
            wbytes = N * K * 1.0625
            out = []
            for path in PATHS:
                def run(i):
                    if epi == 3:
                        _lib.check(lib.qasr_op_gemm_swiglu_q8_cfg(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                                  ws[i].data_ptr(), N, K, hq.data_ptr(), hd.data_ptr(),
                                                                  -1 if path == 2 else (path - 16) % 32, None))
                        return
                    _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                     ws[i].data_ptr(), N, K, None,
                                                     y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, path,
                                                     None))
                try:
                    run(0)
                except _lib.QasrError:
                    out.append(f"{path}: n/a")
                    continue
                torch.cuda.synchronize()
                n = copies * max(1, 24 // copies)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(n):
                    run(i % copies)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / n * 1e3
                out.append(f"{path}:{us:6.1f}us {flops / us / 1e6:4.0f}TF {wbytes / us / 1e3:5.2f}TB/s")
            print(f"{tag:5s} M={M:4d} N={N:6d} K={K:5d} | " + " | ".join(out), flush=True)
        del wq, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
