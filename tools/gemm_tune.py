#!/usr/bin/env python3
"""Time the Q8 MFMA GEMM on the engine's shapes for every tile config / split-K choice (tuning aid, GPU)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = [  # (tag, M, N, K, epi)
    ("prefill gu", 27200, 12288, 2048, 0), ("prefill down", 27200, 2048, 6144, 1),
    ("prefill qkv", 27200, 4096, 2048, 0), ("prefill o", 27200, 2048, 2048, 1),
    ("enc fc1", 23360, 4096, 1024, 2), ("enc fc2", 23360, 1024, 4096, 1), ("enc qkv", 23360, 3072, 1024, 0),
    ("dec256 qkv", 256, 4096, 2048, 0), ("dec256 o", 256, 2048, 2048, 1), ("dec256 gu", 256, 12288, 2048, 0),
    ("dec256 down", 256, 2048, 6144, 1), ("dec256 lm", 256, 151936, 2048, 0),
    ("dec64 qkv", 64, 4096, 2048, 0), ("dec64 o", 64, 2048, 2048, 1), ("dec64 gu", 64, 12288, 2048, 0),
    ("dec64 down", 64, 2048, 6144, 1), ("dec64 lm", 64, 151936, 2048, 0),
    ("dec16 gu", 16, 12288, 2048, 0), ("dec16 down", 16, 2048, 6144, 1), ("dec16 lm", 16, 151936, 2048, 0),
    ("dec256 swiglu", 256, 12288, 2048, 3), ("dec128 swiglu", 128, 12288, 2048, 3), ("dec64 swiglu", 64, 12288, 2048, 3),
    ("dec16 swiglu", 16, 12288, 2048, 3), ("prefill swiglu", 27200, 12288, 2048, 3),
]


# 2 = auto; 16 + cfg (+ 32·splits), or 4096 + cfg (+ 256·splits) for any index: kernels_q8.hip kGemmCfgs — 0..3 register-staged {128², 64×128, 64², 32×64},
# 4..7 LDS-DMA K-64 stages {128², 64×128, 64², 128×64}, 8..11 LDS-DMA K-128 stages (same tiles)
PATHS = [int(p) for p in os.environ.get("PATHS", "2,20,21,22,24,25,26,27").split(",")]


def main():
    lib = _lib.load(os.environ.get("QASR_LIB", _lib.LIB_PATH))
    print("lib:", os.environ.get("QASR_LIB", _lib.LIB_PATH))
    dev = torch.device("cuda:0")
    only = sys.argv[1:] if len(sys.argv) > 1 else None
    for tag, M, N, K, epi in SHAPES:
        if only and not any(o in tag for o in only):
            continue
        xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        xd = torch.rand(M, K // 32, device=dev) * 0.01
        wq = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        ws = (torch.rand(N, K // 32, device=dev) * 0.01).half()
        s4 = None
        if os.environ.get("S4", "0") == "1" and K % 128 == 0:   # the regrouped stage scales (Q8Mat::sc4)
            s4 = torch.empty_like(ws)
            _lib.check(lib.qasr_op_stage_scales(ws.data_ptr(), N, K, s4.data_ptr(), None))
            _lib.check(lib.qasr_op_register_stage_scales(ws.data_ptr(), N, K, s4.data_ptr()))
        y = torch.zeros(M, N, device=dev)
        res = y if epi == 1 else None
        hq = torch.empty(M, N // 2, dtype=torch.int8, device=dev)
        hd = torch.empty(M, N // 64, device=dev)
        flops = 2.0 * M * N * K
        out = []
        for path in PATHS:
            def run():
                if epi == 3:   # fused SwiGLU + Q8 epilogue; path → forced config
                    _lib.check(lib.qasr_op_gemm_swiglu_q8_cfg(xq.data_ptr(), xd.data_ptr(), M, wq.data_ptr(),
                                                              ws.data_ptr(), N, K, hq.data_ptr(), hd.data_ptr(),
                                                              -1 if path == 2 else path if path >= 4096 else
                                                              (path - 16) % 32, None))
                    return
                _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq.data_ptr(), ws.data_ptr(), N,
                                                 K, None, res.data_ptr() if res is not None else None,
                                                 y.data_ptr(), N, epi, path, None))
            try:
                run()
            except _lib.QasrError:
                out.append(f"{path}:      n/a")
                continue
            torch.cuda.synchronize()
            iters = max(3, min(50, int(2e12 / flops * 20)))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / iters * 1e3
            out.append(f"{path}:{us:8.1f}us {flops / us / 1e6:6.0f}TF")
        print(f"{tag:14s} M={M:6d} N={N:6d} K={K:5d} | " + " ".join(out), flush=True)
        if s4 is not None:
            _lib.check(lib.qasr_op_register_stage_scales(ws.data_ptr(), N, K, None))


if __name__ == "__main__":
    main()
