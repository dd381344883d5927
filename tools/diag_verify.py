#!/usr/bin/env python3
"""Diagnosis (GPU): a forced continuation as ONE draft verify pass vs one decode step per token at the real shapes,
long prompt (split decode attention), with the attention split / the fused q-k prologue switched off, and repeats.
usage: python tools/diag_verify.py [arch] [seconds] [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from bench import speech_like  # noqa: E402


def main():
    from qasr.transcribe_cpp import Model

    arch = sys.argv[1] if len(sys.argv) > 1 else "qwen3-asr-1.7b"
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 17
    m = Model.synthetic(arch, seed=7)
    audio = speech_like(np.random.default_rng(32), int(secs * 16000))
    forced = np.array([1000 + 37 * i for i in range(n)], np.int32)

    def show(tag, a, b):
        d = np.abs(a - b).max(1)
        first = next((i for i in range(len(d)) if d[i] > 0), None)
        print(f"{arch} {secs:g}s n={n} {tag:34s} first differing row {first}  max " + " ".join(f"{x:.2g}" for x in d),
              flush=True)

    s = m.session(kv_type="f16", n_ctx=4096)
    ref = s.forced_logits(audio, forced)
    if "--mr-child" in sys.argv:
        show(f"QASR_EXACT_MR={os.environ.get('QASR_EXACT_MR')}: verify vs steps", ref,
             s.forced_logits(audio, forced, one_pass=True))
        return
    v1 = s.forced_logits(audio, forced, one_pass=True)
    v2 = s.forced_logits(audio, forced, one_pass=True)
    show("verify vs steps", ref, v1)
    show("verify vs verify", v1, v2)
    show("steps vs steps", ref, s.forced_logits(audio, forced))
    os.environ["QASR_NO_ATTN_SPLIT"] = "1"
    s2 = m.session(kv_type="f16", n_ctx=4096)
    del os.environ["QASR_NO_ATTN_SPLIT"]
    show("no split: verify vs steps", s2.forced_logits(audio, forced), s2.forced_logits(audio, forced, one_pass=True))
    os.environ["QASR_NO_QK_FUSE"] = "1"
    show("no qk fuse: verify vs steps", s.forced_logits(audio, forced), s.forced_logits(audio, forced, one_pass=True))
    del os.environ["QASR_NO_QK_FUSE"]
    import subprocess

    for mr in ("4", "2", "1"):   # QASR_EXACT_MR is read once per process: a child process per setting
        subprocess.run([sys.executable, os.path.abspath(__file__), arch, str(secs), str(n), "--mr-child"],
                       env=dict(os.environ, QASR_EXACT_MR=mr), check=False)
    for k in (2, 4, 8, 9, 16):
        f = forced[:k]
        show(f"k={k} verify vs steps", s.forced_logits(audio, f), s.forced_logits(audio, f, one_pass=True))


if __name__ == "__main__":
    main()
