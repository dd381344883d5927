#!/usr/bin/env python3
"""Diagnostic for the C4-scale batch test (tests/test_model_real_gpu.py::test_real_batch_c4_scale): the same 64
segments as a batch twice, in a fresh session, and as single runs; prints every batch/batch and batch/single
divergence (segment, first token index) instead of stopping at the first.  QASR_* env switches apply as usual."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, ROOT)
from bench import speech_like  # noqa: E402
from qasr.transcribe_cpp import Model  # noqa: E402


def main():
    m = Model.synthetic("qwen3-asr-1.7b", seed=7)
    s = m.session(kv_type="f16", n_ctx=4096)
    rng = np.random.default_rng(11)
    secs = rng.uniform(2.0, 12.0, size=64)
    clips = [speech_like(np.random.default_rng(500 + i), int(float(x) * 16000)) for i, x in enumerate(secs)]
    b1 = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
    b2 = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
    singles = [s.run(c, force_tokens_per_s=8).tokens for c in clips]
    s2 = m.session(kv_type="f16", n_ctx=4096)
    b3 = [r.tokens for r in s2.run_batch(clips, force_tokens_per_s=8)]

    def divs(a, b):
        out = []
        for i in range(64):
            d = next((j for j in range(len(a[i])) if a[i][j] != b[i][j]), None)
            if d is not None:
                out.append((i, d))
        return out
    print("batch1 vs batch2 (same session):", divs(b1, b2), flush=True)
    print("batch1 vs batch3 (fresh session):", divs(b1, b3), flush=True)
    print("batch1 vs singles:", divs(b1, singles), flush=True)
    print("batch3 vs singles:", divs(b3, singles), flush=True)
    for i, d in divs(b1, singles)[:6]:
        lg = s.forced_logits(clips[i], np.asarray(singles[i][:d], np.int32))[d]
        rng_ = float(lg.max() - lg.min())
        tb, ts = b1[i][d], singles[i][d]
        print(f"seg {i} tok {d}: single picks {ts} ({lg[ts]:.3f}), batch picks {tb} ({lg[tb]:.3f}); gap "
              f"{lg[ts] - lg[tb]:.3f} = {100 * (lg[ts] - lg[tb]) / rng_:.2f} % of the range {rng_:.1f}", flush=True)


if __name__ == "__main__":
    main()
