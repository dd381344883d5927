#!/usr/bin/env python3
"""Decode-GEMM anatomy probe: time one Q8 GEMM configuration while K (loop length) and N (grid size) vary, with cold
weights (a ring of copies larger than the Infinity Cache) and with warm weights (one copy), to split a launch into
fill / steady-state / tail.  GPU.  usage: CFGS="14:1,12:1" M=256 python tools/dec_gemm_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    M = int(os.environ.get("M", "256"))
    cfgs = [tuple(int(v) for v in c.split(":")) for c in os.environ.get("CFGS", "14:1").split(",")]
    Ks = [int(v) for v in os.environ.get("KS", "512,1024,2048,4096,8192").split(",")]
    Ns = [int(v) for v in os.environ.get("NS", "1024,2048,4096,8192,12288").split(",")]
    epi = int(os.environ.get("EPI", "0"))
    out = []
    for N in Ns:
        for K in Ks:
            copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
            wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
            ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            y = torch.zeros(M, N, device=dev)
            for cfg, sp in cfgs:
                def run(i):
                    _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                     ws[i].data_ptr(), N, K, None,
                                                     y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi,
                                                     2 if cfg < 0 else 16 + cfg + 32 * sp, None))
                rec = {"N": N, "K": K, "cfg": cfg, "splits": sp}
                for tag, cyc in (("cold", copies), ("warm", 1)):
                    run(0)
                    torch.cuda.synchronize()
                    n = max(16, cyc)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(n):
                        run(i % cyc)
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / n * 1e3
                    rec[tag + "_us"] = round(us, 2)
                    rec[tag + "_tf"] = round(2.0 * M * N * K / us / 1e6, 1)
                print(json.dumps(rec), flush=True)
                out.append(rec)
            del wq, ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
