#!/usr/bin/env python3
"""In-graph cost of one launch of each batch-1 decode op (SURVEY §8(d) C2 shapes): a chain of R launches of the op is
captured into a hipGraph (torch.cuda.graph, the C ABI ops on its stream) and replayed; the replay time ÷ R is the
op's marginal cost inside a decode step graph, boundary included.  GEMV chains read a distinct weight copy per
launch, with enough copies (> 600 MB) that every launch streams from HBM as in a 28-layer step.  GPU.
usage: python tools/graph_cost.py [arch ...]   (default qwen3-asr-1.7b)"""
import ctypes as C
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = {"qwen3-asr-1.7b": dict(H=2048, F=6144, nh=16, nkv=8, V=151936),
          "qwen3-asr-0.6b": dict(H=1024, F=3072, nh=16, nkv=8, V=151936)}
HD = 128
KEYS = 150   # a 5 s clip's prompt (~75 audio + ~15 text tokens) plus ~40 generated


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()   # warm: allocations, first-launch setup outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # µs per replay


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    archs = sys.argv[1:] or ["qwen3-asr-1.7b"]
    out = {}
    for arch in archs:
        sh = SHAPES[arch]
        H, F, nh, nkv, V = sh["H"], sh["F"], sh["nh"], sh["nkv"], sh["V"]
        QKV = (nh + 2 * nkv) * HD
        res = {}
        x = torch.randn(1, max(H, F, nh * HD), device=dev)
        nw = torch.rand(max(H, F), device=dev) + 0.5
        xq = torch.randint(-127, 128, (1, max(H, F, nh * HD)), dtype=torch.int8, device=dev)
        xd = torch.rand(1, max(H, F, nh * HD) // 32, device=dev) * 0.01
        y = torch.zeros(1, max(QKV, 2 * F, V), device=dev)
        gu = torch.randn(1, 2 * F, device=dev)

        R = 56
        res["rmsnorm_q8"] = timed(lambda: [_lib.check(lib.qasr_op_rmsnorm_q8(
            x.data_ptr(), 1, H, nw.data_ptr(), C.c_float(1e-6), xq.data_ptr(), xd.data_ptr(), stream()))
            for _ in range(R)]) / R
        res["swiglu_q8"] = timed(lambda: [_lib.check(lib.qasr_op_swiglu_q8_interleaved(
            gu.data_ptr(), 1, F, xq.data_ptr(), xd.data_ptr(), stream())) for _ in range(R)]) / R
        res["quant_rows_32 (floor)"] = timed(lambda: [_lib.check(lib.qasr_op_quant_rows(
            x.data_ptr(), 1, 32, 32, xq.data_ptr(), xd.data_ptr(), stream())) for _ in range(R)]) / R

        # fused decode attention over KEYS cached keys (q/k norm + RoPE + KV write + attention + Q8 output); each
        # launch of the chain on its own layer's cache (28 layers, as in a step)
        kvd = nkv * HD
        for keys in [int(k) for k in os.environ.get("ATTN_KEYS", str(KEYS)).split(",")]:
            kc = [torch.randn(keys + 1, kvd, device=dev).half() for _ in range(28)]
            vc = [torch.randn(keys + 1, kvd, device=dev).half() for _ in range(28)]
            qkv = torch.randn(1, QKV, device=dev)
            pos = torch.tensor([keys], dtype=torch.int32, device=dev)
            kvs = torch.tensor([0], dtype=torch.int32, device=dev)
            kvl = torch.tensor([keys + 1], dtype=torch.int32, device=dev)
            rope = torch.randn(keys + 1, HD // 2, 2, device=dev)
            qn = torch.rand(HD, device=dev) + 0.5
            res["attention_decode_fused" + ("" if keys == KEYS else f"@{keys}")] = timed(lambda: [_lib.check(
                lib.qasr_op_attention_decode_fused(
                    qkv.data_ptr(), 1, nh, nkv, HD, pos.data_ptr(), pos.data_ptr(), qn.data_ptr(), qn.data_ptr(),
                    rope.data_ptr(), C.c_float(1e-6), kc[i % 28].data_ptr(), vc[i % 28].data_ptr(), kvs.data_ptr(),
                    kvl.data_ptr(), C.c_float(HD ** -0.5), xq.data_ptr(), xd.data_ptr(), stream()))
                for i in range(R)]) / R
            # the session's default for ≤ 4 rows: ranges over 512 keys split over up to 8 workgroups
            part = torch.empty(4 * nkv * 16 * (nh // nkv) * 130, device=dev)
            cnt = torch.zeros(4 * nkv, dtype=torch.int32, device=dev)
            res["attention_decode_split" + ("" if keys == KEYS else f"@{keys}")] = timed(lambda: [_lib.check(
                lib.qasr_op_attention_decode_split(
                    qkv.data_ptr(), 1, nh, nkv, HD, pos.data_ptr(), pos.data_ptr(), qn.data_ptr(), qn.data_ptr(),
                    rope.data_ptr(), C.c_float(1e-6), kc[i % 28].data_ptr(), vc[i % 28].data_ptr(), kvs.data_ptr(),
                    kvl.data_ptr(), C.c_float(HD ** -0.5), xq.data_ptr(), xd.data_ptr(), part.data_ptr(),
                    cnt.data_ptr(), stream()))
                for i in range(R)]) / R
        if os.environ.get("ATTN_ONLY"):
            out[arch] = {k: round(v, 2) for k, v in res.items()}
            print(json.dumps({arch: out[arch]}), flush=True)
            continue

        src = torch.randn(1, 2 * max(H, F), device=dev)
        hq = torch.empty(1, F, dtype=torch.int8, device=dev)
        hd = torch.empty(1, F // 32, device=dev)
        # pro: 0 the stand-alone GEMV (separate norm / SwiGLU launches), 1 the per-CU GEMV on Q8 rows, 2 with the
        # norm prologue, 3 with the norm prologue and the SwiGLU epilogue
        for tag, N, K, epi, pro in (("gemv_qkv", QKV, H, 0, 0), ("gemv_qkv+rms", QKV, H, 0, 2),
                                    ("gemv_o", H, nh * HD, 1, 0), ("gemv_o_wide", H, nh * HD, 1, 1),
                                    ("gemv_gu", 2 * F, H, 0, 0), ("gemv_gu+rms+swiglu", 2 * F, H, 3, 3),
                                    ("gemv_down", H, F, 1, 0), ("gemv_down_wide", H, F, 1, 1),
                                    ("gemv_lm_head", V, H, 0, 0)):
            nbytes = N * K * 1.0625
            n = max(28 if "lm_head" not in tag else 4, math.ceil(600e6 / nbytes))
            # WARM=1: one weight copy re-read by every launch (Infinity-Cache / L2 resident), the cold chain's contrast
            ncopy = 1 if os.environ.get("WARM") else n
            wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(ncopy)]
            ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(ncopy)]

            def chain():
                for i in range(n):
                    if pro:
                        _lib.check(lib.qasr_op_gemv_fused(
                            0 if pro == 1 else 1, src.data_ptr(), K, nw.data_ptr(), 1e-6, 1, xq.data_ptr(),
                            xd.data_ptr(), wq[i % ncopy].data_ptr(), ws[i % ncopy].data_ptr(), N, K,
                            y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, hq.data_ptr(), hd.data_ptr(),
                            stream()))
                        continue
                    _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), 1, wq[i % ncopy].data_ptr(),
                                                     ws[i % ncopy].data_ptr(), N, K, None,
                                                     y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, 1,
                                                     stream()))
            us = timed(chain) / n
            res[tag] = us
            res[tag + "_TBps"] = round(nbytes / us / 1e6, 2)
            del wq, ws
            torch.cuda.empty_cache()
        out[arch] = {k: round(v, 2) for k, v in res.items()}
        print(json.dumps({arch: out[arch]}), flush=True)


if __name__ == "__main__":
    main()
