#!/usr/bin/env python3
"""Single-utterance latency of the server path (SURVEY §8(d) C2/C3 shapes): one `session.run` per request on a
seeded speech-like clip, synthetic weights, forced 8 tokens per audio-second so the work is deterministic.
Prints one JSON line per (arch, clip length)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from bench import speech_like  # noqa: E402
from qasr.transcribe_cpp import Model  # noqa: E402


def main():
    archs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["qwen3-asr-0.6b", "qwen3-asr-1.7b"]
    lengths = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1.0, 5.0, 12.0]
    for arch in archs:
        m = Model.synthetic(arch, seed=0)
        s = m.session(kv_type="f16", n_ctx=32768)
        for secs in lengths:
            audio = speech_like(np.random.default_rng(0), int(secs * 16000))
            for _ in range(2):
                s.run(audio, force_tokens_per_s=8)
            times, stages = [], None
            for _ in range(10):
                t0 = time.perf_counter()
                r = s.run(audio, force_tokens_per_s=8)
                times.append(time.perf_counter() - t0)
                stages = r
            ms = np.array(times) * 1e3
            print(json.dumps({"arch": arch, "audio_s": secs, "tokens": len(stages.tokens),
                              "p50_ms": round(float(np.median(ms)), 2), "p95_ms": round(float(np.percentile(ms, 95)), 2),
                              "rtf_inv": round(secs / (np.median(ms) / 1e3), 1),
                              "stage_ms": {k: round(v, 2) for k, v in stages.timings_ms.items()}}), flush=True)
        s.close()
        m.close()


if __name__ == "__main__":
    main()
