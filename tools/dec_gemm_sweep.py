#!/usr/bin/env python3
"""Sweep every Q8 GEMM configuration × split-K count on the decode shapes with COLD weights (a ring of weight copies
larger than the Infinity Cache, as in a decode step that streams 28 layers) and print the best few per (shape, M)
next to the heuristic.  Tuning aid for gemm_q8's decode table (kernels_q8.hip).  GPU.
usage: python tools/dec_gemm_sweep.py [out.json]
env: SHAPES (qkv,o,down,gu), MS (row counts), CFGS (configuration indices; ≥ 32 use the wide path code
4096 + cfg + 256·splits), S4=1 registers the regrouped stage scales of every weight copy (Q8Mat::sc4: the K-128
tiles stage their scales by 16-byte DMA), FIX (split-K fix-up workspace, default 1)."""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = [("qkv", 4096, 2048, 0), ("o", 2048, 2048, 1), ("down", 2048, 6144, 1), ("gu", 12288, 2048, 3),
          ("lmhead", 151936, 2048, 0)]   # the decode steps' vocabulary projection (SHAPES=lmhead)
MS = [int(x) for x in os.environ.get("MS", "16,32,64,96,128,160,192,224,256").split(",")]
CFGS = list(range(4, 31)) + list(range(36, 40))   # 32..35 and 40..48 removed in round 5
SPLITS = [1, 2, 3, 4, 6, 8]
SWIGLU_CFGS = [4, 5, 8, 9, 12, 13, 15, 20, 22, 23, 28, 29, 30, 38, 39]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    result = {}
    fix = os.environ.get("FIX", "1") == "1"   # split-K through the fix-up workspace (FIX=0: f32 atomics)
    if fix:
        part = torch.empty(256 * 12288 * 8, dtype=torch.float32, device=dev)
        cnt = torch.zeros(8192, dtype=torch.int32, device=dev)
        _lib.check(lib.qasr_op_set_gemm_fixup(part.data_ptr(), part.numel() * 4, cnt.data_ptr(), cnt.numel()))
    det = C.c_int32(0)
    _lib.check(lib.qasr_get_deterministic(C.byref(det)))
    det = det.value == 1   # the default: split-K only through the fix-up (wave-64 tiles), the rest unsplit
    wave64 = {12, 15, 20, 22, 23, 33, 35}
    print(f"deterministic={det} fix-up={fix}", flush=True)
    shapes = [s for s in SHAPES if s[0] in os.environ.get("SHAPES", "qkv,o,down,gu").split(",")]
    cfgs = [int(c) for c in os.environ["CFGS"].split(",")] if "CFGS" in os.environ else CFGS
    for tag, N, K, epi in shapes:
        copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
        wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
        ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
        s4 = []
        if os.environ.get("S4", "0") == "1":
            for w in ws:
                o = torch.empty_like(w)
                _lib.check(lib.qasr_op_stage_scales(w.data_ptr(), N, K, o.data_ptr(), None))
                _lib.check(lib.qasr_op_register_stage_scales(w.data_ptr(), N, K, o.data_ptr()))
                s4.append(o)
        for M in MS:
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            y = torch.zeros(M, N, device=dev)
            hq = torch.empty(M, N // 2, dtype=torch.int8, device=dev)
            hd = torch.empty(M, N // 64, device=dev)
            def splits(c):
                if 24 <= c <= 30:
                    return [0]
                if det and not (fix and c in wave64):
                    return [1]
                return SPLITS if (fix or epi != 3) else [0]
            combos = [(-1, 0)] + ([(c, s) for c in SWIGLU_CFGS if c in cfgs or "CFGS" not in os.environ
                                   for s in splits(c)]
                                  if epi == 3 else [(c, s) for c in cfgs for s in splits(c)])
            times = []
            for cfg, sp in combos:
                def run(i):
                    if epi == 3:
                        code = cfg if cfg < 0 else 4096 + cfg + 256 * sp
                        _lib.check(lib.qasr_op_gemm_swiglu_q8_cfg(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                                  ws[i].data_ptr(), N, K, hq.data_ptr(), hd.data_ptr(),
                                                                  code, None))
                        return
                    path = 2 if cfg < 0 else 4096 + cfg + 256 * sp
                    # a store GEMM with split-K clears y inside gemm_q8 (hipMemsetAsync): timed as part of it
                    _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                     ws[i].data_ptr(), N, K, None,
                                                     y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, path,
                                                     None))
                try:
                    run(0)
                except _lib.QasrError:
                    continue
                torch.cuda.synchronize()
                n = copies * max(1, 16 // copies)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(n):
                    run(i % copies)
                e1.record()
                torch.cuda.synchronize()
                times.append((round(e0.elapsed_time(e1) / n * 1e3, 2), cfg, sp))
            heur = next(t for t in times if t[1] < 0)
            best = sorted(times)[:6]
            result[f"{tag}:{M}"] = {"heuristic_us": heur[0], "best": best, "all": sorted(times)}
            print(f"{tag:5s} M={M:4d} heuristic {heur[0]:7.1f}us | best " +
                  "  ".join(f"{t:6.1f}us c{c}s{s}" for t, c, s in best), flush=True)
        for w in ws:
            if s4:
                _lib.check(lib.qasr_op_register_stage_scales(w.data_ptr(), N, K, None))
        del wq, ws, s4
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(result, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
