#!/usr/bin/env python3
"""Cost of one draft verify pass by row count (GPU): a 1.7B session, a 10 s prompt, then teacher-forced continuations
fed as ONE verify pass of n rows (Session.forced_logits(one_pass=True)), timed end to end minus the same call with
n = 1; run under rocprofv3 --kernel-trace --stats to see which kernels a pass spends its time in.
usage: python tools/verify_cost.py [arch] [n1,n2,…]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from bench import speech_like  # noqa: E402


def main():
    from qasr.transcribe_cpp import Model

    arch = sys.argv[1] if len(sys.argv) > 1 else "qwen3-asr-1.7b"
    ns = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8, 16, 32]
    m = Model.synthetic(arch, seed=7)
    s = m.session(kv_type="f16", n_ctx=4096)
    audio = speech_like(np.random.default_rng(5), 160000)
    base = None
    for n in ns:
        f = np.array([1000 + 37 * i for i in range(n)], np.int32)
        s.forced_logits(audio, f, one_pass=True)   # warm (graphs, scratch)
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            s.forced_logits(audio, f, one_pass=True)
            t.append(time.perf_counter() - t0)
        ms = 1e3 * float(np.median(t))
        base = ms if base is None else base
        print(f"{arch} verify pass n={n:2d}: call {ms:7.2f} ms (vs n={ns[0]}: +{ms - base:6.2f} ms)", flush=True)


if __name__ == "__main__":
    main()
