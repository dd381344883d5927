#!/usr/bin/env python3
"""The one-wave decode attention (k_attn_wave) against the 4-wave kernel (k_attention) on the C4 mix with cold KV
(buffers rotated over > 256 MB, the MALL size), unfused launches (qasr_op_attention_dense, dense = 0) with Q8 output,
per row count.  usage: attn_wave_probe.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    hd, nh, nkv = 128, 16, 8
    for M, extra in [(256, 1), (256, 40), (192, 50), (128, 70), (96, 80), (64, 85), (33, 90)]:
        secs = rng.uniform(2, 12, M)
        lens = ((13 * secs + 16).astype(int) + extra).astype(np.int32)
        kv_bytes = float(lens.sum()) * nkv * hd * 2 * 2
        copies = max(3, int(np.ceil(600e6 / kv_bytes)))
        starts = np.concatenate([[0], np.cumsum(lens + 16)[:-1]]).astype(np.int32)
        slots = int((starts + lens).max()) + 8
        ks = [torch.randn(slots, nkv * hd, device=dev).half() for _ in range(copies)]
        vs = [torch.randn(slots, nkv * hd, device=dev).half() for _ in range(copies)]
        q = torch.randn(M, nh * hd, device=dev).half()
        s_t, l_t = torch.from_numpy(starts).to(dev), torch.from_numpy(lens).to(dev)
        oq = torch.empty(M, nh * hd, dtype=torch.int8, device=dev)
        od = torch.empty(M, nh * hd // 32, device=dev)
        res = {}
        for wave in (0, 1):
            _lib.check(lib.qasr_op_set_attn_wave_rows(wave))

            def run(i):
                _lib.check(lib.qasr_op_attention_dense(q.data_ptr(), nh * hd, ks[i].data_ptr(), vs[i].data_ptr(),
                                                       nkv * hd, s_t.data_ptr(), l_t.data_ptr(), M, nh, nkv, hd,
                                                       1 / np.sqrt(hd), None, oq.data_ptr(), od.data_ptr(), 0, None))
            for i in range(copies):
                run(i)
            torch.cuda.synchronize()
            n = 6 * copies
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(n):
                run(i % copies)
            e1.record()
            torch.cuda.synchronize()
            res[wave] = e0.elapsed_time(e1) / n * 1e3
        _lib.check(lib.qasr_op_set_attn_wave_rows(0))
        print(f"M={M:3d} keys~{int(lens.mean()):3d} max {int(lens.max()):3d}: 4-wave {res[0]:7.1f} us "
              f"({kv_bytes / res[0] / 1e3:5.0f} GB/s)  one-wave {res[1]:7.1f} us ({kv_bytes / res[1] / 1e3:5.0f} GB/s)",
              flush=True)
        del ks, vs
        torch.cuda.empty_cache()

if __name__ == "__main__":
    main()
