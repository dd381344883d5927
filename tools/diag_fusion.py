#!/usr/bin/env python3
"""Diagnosis (GPU): the 1-row decode with fused GEMV prologues vs the separate launches (QASR_NO_DEC_FUSE=1), fresh
sessions, repeats.  Prints the largest logit difference per forced row.  QASR_LIB selects the library build.
usage: python tools/diag_fusion.py [arch]"""
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
    m = Model.synthetic(arch, seed=7)
    audio = speech_like(np.random.default_rng(16), 80000)
    forced = np.array([900 + 41 * i for i in range(5)], np.int32)
    sess = {}
    sess["fused"] = m.session(kv_type="f16", n_ctx=4096)
    os.environ["QASR_NO_DEC_FUSE"] = "1"
    sess["unfused"] = m.session(kv_type="f16", n_ctx=4096)
    del os.environ["QASR_NO_DEC_FUSE"]
    sess["fused2"] = m.session(kv_type="f16", n_ctx=4096)
    out = {k: s.forced_logits(audio, forced) for k, s in sess.items()}
    out["fused_again"] = sess["fused"].forced_logits(audio, forced)
    out["unfused_again"] = sess["unfused"].forced_logits(audio, forced)
    for k in out:
        d = np.abs(out[k] - out["fused"]).max(1)
        print(f"{os.environ.get('QASR_LIB', 'current')[-30:]:30s} {k:14s} vs fused: " + " ".join(f"{x:.3g}" for x in d),
              flush=True)


if __name__ == "__main__":
    main()
