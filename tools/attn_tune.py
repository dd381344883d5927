#!/usr/bin/env python3
"""Time the attention kernels on the engine's shapes (GPU): decode rows (one utterance each, ranges scattered over
the KV cache) and prefill rows (causal runs per utterance).  QASR_ATTN_SINGLE=1 runs decode rows as single-row MFMA tiles (A/B)."""
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
    secs = rng.uniform(2, 12, 256)
    prompt = (13 * secs + 16).astype(int)
    cases = []
    for M, extra in [(256, 1), (256, 40), (128, 70), (32, 90)]:
        lens = (prompt[:M] + extra).astype(np.int32)
        starts = np.concatenate([[0], np.cumsum(lens + 100)[:-1]]).astype(np.int32)
        cases.append((f"decode M={M} ctx~{int(lens.mean())}", starts, lens, False))
    st, ln = [], []
    base = 0
    for p in prompt:
        st += [base] * p
        ln += list(range(1, p + 1))
        base += p + 100
    cases.append((f"prefill rows={len(st)}", np.array(st, np.int32), np.array(ln, np.int32), True))
    for name, starts, lens, dense in cases:
        rows = len(starts)
        slots = int((starts + lens).max()) + 8
        k = torch.randn(slots, nkv * hd, device=dev).half()
        v = torch.randn(slots, nkv * hd, device=dev).half()
        q = torch.randn(rows, nh * hd, device=dev).half()
        s_t, l_t = torch.from_numpy(starts).to(dev), torch.from_numpy(lens).to(dev)
        oq = torch.empty(rows, nh * hd, dtype=torch.int8, device=dev)
        od = torch.empty(rows, nh * hd // 32, device=dev)

        def run():
            _lib.check(lib.qasr_op_attention_dense(q.data_ptr(), nh * hd, k.data_ptr(), v.data_ptr(), nkv * hd,
                                                   s_t.data_ptr(), l_t.data_ptr(), rows, nh, nkv, hd,
                                                   1 / np.sqrt(hd), None, oq.data_ptr(), od.data_ptr(), int(dense),
                                                   None))
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        kv_bytes = float(lens.sum()) * nkv * hd * 2 * 2 if not dense else float((starts + lens).max()) * 0
        print(f"{name:28s} {us:9.1f} us   KV stream {kv_bytes / us / 1e3 if kv_bytes else 0:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
