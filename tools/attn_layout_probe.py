#!/usr/bin/env python3
"""Does the KV cache layout bound the decode attention?  Times the decode-row attention (unfused k_attention) on the
C4 mix at 256 rows with cold KV (buffers rotated over > 256 MB, the MALL size) in two layouts of the same bytes:
  slot-major (today): K[slot][kvh][hd], a (row, KV head)'s keys are 256-B pieces 2 KB apart;
  head-major (probe): K[kvh][slot][hd], emulated as rows·nkv single-KV-head rows with contiguous key ranges.
usage: attn_layout_probe.py"""
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
    G = nh // nkv
    for M, extra in [(256, 1), (256, 40), (128, 70)]:
        secs = rng.uniform(2, 12, M)
        lens = ((13 * secs + 16).astype(int) + extra).astype(np.int32)
        kv_bytes = float(lens.sum()) * nkv * hd * 2 * 2
        copies = max(3, int(np.ceil(600e6 / kv_bytes)))
        for layout in ("slot-major", "head-major"):
            if layout == "slot-major":
                rows, h, kvh_n, ld = M, nh, nkv, nkv * hd
                l_r = lens
            else:
                rows, h, kvh_n, ld = M * nkv, G, 1, hd
                l_r = np.repeat(lens, nkv)
            starts = np.concatenate([[0], np.cumsum(l_r + 16)[:-1]]).astype(np.int32)
            slots = int((starts + l_r).max()) + 8
            ks = [torch.randn(slots, kvh_n * hd, device=dev).half() for _ in range(copies)]
            vs = [torch.randn(slots, kvh_n * hd, device=dev).half() for _ in range(copies)]
            q = torch.randn(rows, h * hd, device=dev).half()
            s_t, l_t = torch.from_numpy(starts).to(dev), torch.from_numpy(l_r.astype(np.int32)).to(dev)
            oq = torch.empty(rows, h * hd, dtype=torch.int8, device=dev)
            od = torch.empty(rows, h * hd // 32, device=dev)

            def run(i):
                _lib.check(lib.qasr_op_attention_dense(q.data_ptr(), h * hd, ks[i].data_ptr(), vs[i].data_ptr(), ld,
                                                       s_t.data_ptr(), l_t.data_ptr(), rows, h, kvh_n, hd,
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
            us = e0.elapsed_time(e1) / n * 1e3
            print(f"M={M} keys~{int(lens.mean())} {layout:10s} {us:8.1f} us  {kv_bytes / us / 1e3:7.0f} GB/s "
                  f"(cold: {copies} copies)", flush=True)
            del ks, vs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
