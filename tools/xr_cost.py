#!/usr/bin/env python3
"""≤ 32-row decode linears: the per-phase exact launches (qasr_op_xr_linear / qasr_op_xr_gu_swiglu, kernels_xr.hip)
against the exact-row MFMA kernel (qasr_op_gemm_exact_rows [+ swiglu]) and the batched table GEMM (qasr_op_linear_q8
path 2 / qasr_op_gemm_swiglu_q8), 1.7B decoder shapes, COLD weights (a ring of copies larger than the Infinity Cache).
The norm is a separate launch in every column (folded variants: fold_*).  GPU.  usage: python tools/xr_cost.py [out.json]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = [("qkv", 4096, 2048, 0), ("o", 2048, 2048, 1), ("gu", 12288, 2048, 3), ("down", 2048, 6144, 1)]
MS = [int(v) for v in os.environ.get("XR_COST_MS", "1,2,4,8,12,16,24,32").split(",")]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    part = torch.empty(256 * 12288 * 8, dtype=torch.float32, device=dev)
    cnt = torch.zeros(8192, dtype=torch.int32, device=dev)
    _lib.check(lib.qasr_op_set_gemm_fixup(part.data_ptr(), part.numel() * 4, cnt.data_ptr(), cnt.numel()))
    out = {}
    for tag, N, K, epi in SHAPES:
        copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
        wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
        ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
        s4 = []
        for w in ws:
            o = torch.empty_like(w)
            _lib.check(lib.qasr_op_stage_scales(w.data_ptr(), N, K, o.data_ptr(), None))
            _lib.check(lib.qasr_op_register_stage_scales(w.data_ptr(), N, K, o.data_ptr()))
            s4.append(o)
        for M in MS:
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            src = torch.randn(M, K, device=dev)
            nw = torch.ones(K, device=dev)
            y = torch.zeros(M, N, device=dev)
            hq = torch.empty(M, max(N // 2, 1), dtype=torch.int8, device=dev)
            hd = torch.empty(M, max(N // 64, 1), device=dev)
            p = lambda t: t.data_ptr()  # noqa: E731

            def table(i):
                if M < 5:
                    return None
                if epi == 3:
                    _lib.check(lib.qasr_op_gemm_swiglu_q8(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K, p(hq), p(hd),
                                                          None))
                else:
                    _lib.check(lib.qasr_op_linear_q8(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K, None,
                                                     p(y) if epi == 1 else None, p(y), N, epi, 2, None))
                return True

            def exact(i):
                _lib.check(lib.qasr_op_gemm_exact_rows(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K,
                                                       p(y) if epi == 1 else None, p(y), N, 1 if epi == 1 else 0,
                                                       None))
                if epi == 3:
                    _lib.check(lib.qasr_op_swiglu_q8_interleaved(p(y), M, N // 2, p(hq), p(hd), None))
                return True

            def xr(i, fold=False):
                if fold and (M > 8 or epi == 1):
                    return None
                a = (None, None, p(src), p(nw)) if fold else (p(xq), p(xd), None, None)
                if epi == 3:
                    _lib.check(lib.qasr_op_xr_gu_swiglu(*a, 1e-6, M, p(wq[i]), p(ws[i]), N, K, p(hq), p(hd), None))
                else:
                    _lib.check(lib.qasr_op_xr_linear(*a, 1e-6, M, p(wq[i]), p(ws[i]), N, K, p(y), N,
                                                     1 if epi == 1 else 0, None))
                return True

            def tile(i):
                # the multi-fragment exact tile (qasr_op_xr_tile, round 5's measured-negative build 6d57de9 only;
                # gate/up: + swiglu_q8_interleaved)
                if not hasattr(lib, "qasr_op_xr_tile"):
                    return None
                _lib.check(lib.qasr_op_xr_tile(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K, p(y), N,
                                               1 if epi == 1 else 0, None))
                if epi == 3:
                    _lib.check(lib.qasr_op_swiglu_q8_interleaved(p(y), M, N // 2, p(hq), p(hd), None))
                return True

            row = {}
            big = M > 32
            for name, fn in (("table", table), ("exact", exact), ("xr", None if big else xr), ("tile", tile),
                             ("xr_fold", None if big else (lambda i: xr(i, True)))):
                if fn is None or fn(0) is None:
                    continue
                torch.cuda.synchronize()
                n = copies * max(1, 16 // copies)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(n):
                    fn(i % copies)
                e1.record()
                torch.cuda.synchronize()
                row[name] = round(e0.elapsed_time(e1) / n * 1e3, 2)
            out[f"{tag}:{M}"] = row
            print(f"{tag:5s} M={M:3d} " + "  ".join(f"{k} {v:7.2f}us" for k, v in row.items()), flush=True)
        for w in ws:
            _lib.check(lib.qasr_op_register_stage_scales(w.data_ptr(), N, K, None))
        del wq, ws, s4
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
