#!/usr/bin/env python3
"""MXFP8 GEMM (block-scaled v_mfma_scale_f32_16x16x128_f8f6f4) vs the Q8 W8A8 GEMM on the engine's shapes:
µs per launch and TFLOP/s (back-to-back launches, random operands).  CFGS: MX configs (-1 auto, 0 128², 1 64², 2
64×128); the Q8 column is gemm_q8's heuristic."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gemm_tune import SHAPES  # noqa: E402
from qasr import _lib  # noqa: E402

CFGS = [int(c) for c in os.environ.get("CFGS", "-1,0,1,2").split(",")]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    only = sys.argv[1:] or None
    for tag, M, N, K, epi in SHAPES:
        if (only and not any(o in tag for o in only)) or epi == 3 or K % 128:
            continue
        x8 = (torch.randint(0, 256, (M, K), dtype=torch.uint8, device=dev) & 0xF7)
        xs = torch.randint(120, 134, (M, K // 32), dtype=torch.uint8, device=dev)
        w8 = (torch.randint(0, 256, (N, K), dtype=torch.uint8, device=dev) & 0xF7)
        ws = torch.randint(120, 134, (N, K // 32), dtype=torch.uint8, device=dev)
        xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        xd = torch.rand(M, K // 32, device=dev) * 0.01
        wq = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wsc = (torch.rand(N, K // 32, device=dev) * 0.01).half()
        y = torch.zeros(M, N, device=dev)
        res = y if epi == 1 else None
        flops = 2.0 * M * N * K
        out = []
        us = timeit(lambda: _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq.data_ptr(),
                                                             wsc.data_ptr(), N, K, None,
                                                             res.data_ptr() if res is not None else None,
                                                             y.data_ptr(), N, epi, 2, None)))
        out.append(f"q8: {us:8.1f}us {flops / us / 1e6:5.0f}TF")
        for cfg in CFGS:
            us = timeit(lambda: _lib.check(lib.qasr_op_gemm_mx(x8.data_ptr(), xs.data_ptr(), M, w8.data_ptr(),
                                                               ws.data_ptr(), N, K, None,
                                                               res.data_ptr() if res is not None else None,
                                                               y.data_ptr(), N, epi, None, None, cfg, None)))
            out.append(f"mx{cfg}: {us:8.1f}us {flops / us / 1e6:5.0f}TF")
        print(f"{tag:14s} M={M:6d} N={N:6d} K={K:5d} | " + "  ".join(out), flush=True)


if __name__ == "__main__":
    main()
