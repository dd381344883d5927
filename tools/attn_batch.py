#!/usr/bin/env python3
"""Batched decode attention (SURVEY §8(d) C4 decode steps): the fused kernel (q/k norm + RoPE + KV write + attention +
Q8 output) at M rows whose KV lengths follow the bench workload (prompt 13·s+16 audio/text tokens, s ~ U[2,12], plus
the tokens generated so far), one KV cache per layer (28, cold as in a step), a chain of 28 launches captured in a
hipGraph.  Prints µs per launch and the KV stream rate.  GPU.  usage: python tools/attn_batch.py"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

HD, NH, NKV = 128, 16, 8


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    secs = rng.uniform(2, 12, 256)
    prompt = (13 * secs + 16).astype(int)
    out = []
    for M, frac in [(256, 0.1), (224, 0.4), (150, 0.6), (64, 0.85)]:
        idx = np.argsort(-secs)[:M]                        # the longest utterances are the last to finish
        lens = (prompt[idx] + (frac * 8 * secs[idx]).astype(int) + 1).astype(np.int32)
        starts = np.concatenate([[0], np.cumsum(lens + 100)[:-1]]).astype(np.int32)
        slots = int((starts + lens).max()) + 8
        kvd = NKV * HD
        L = 28
        kc = [torch.randn(slots, kvd, device=dev).half() for _ in range(L)]
        vc = [torch.randn(slots, kvd, device=dev).half() for _ in range(L)]
        qkv = torch.randn(M, (NH + 2 * NKV) * HD, device=dev)
        pos = torch.from_numpy(lens - 1).to(dev)
        slot = torch.from_numpy(starts + lens - 1).to(dev)
        kvs, kvl = torch.from_numpy(starts).to(dev), torch.from_numpy(lens).to(dev)
        rope = torch.randn(int(lens.max()) + 1, HD // 2, 2, device=dev)
        qn = torch.rand(HD, device=dev) + 0.5
        oq = torch.empty(M, NH * HD, dtype=torch.int8, device=dev)
        od = torch.empty(M, NH * HD // 32, device=dev)

        def chain():
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            for i in range(L):
                _lib.check(lib.qasr_op_attention_decode_fused(
                    qkv.data_ptr(), M, NH, NKV, HD, pos.data_ptr(), slot.data_ptr(), qn.data_ptr(), qn.data_ptr(),
                    rope.data_ptr(), C.c_float(1e-6), kc[i].data_ptr(), vc[i].data_ptr(), kvs.data_ptr(),
                    kvl.data_ptr(), C.c_float(HD ** -0.5), oq.data_ptr(), od.data_ptr(), st))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            chain()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps / L * 1e3
        kv = float(lens.sum()) * kvd * 2 * 2
        rec = {"rows": M, "mean_keys": round(float(lens.mean()), 1), "us": round(us, 2),
               "kv_MB": round(kv / 1e6, 1), "TBps": round(kv / us / 1e6, 2),
               "variant": os.environ.get("QASR_ATTN_VARIANT", "0")}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del kc, vc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
