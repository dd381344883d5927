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
    import ctypes as C

    from qasr import _lib

    prof = "--prof" in sys.argv
    # --device: the clip uploaded once and run from HBM (run_batch_device, the bench's convention); the host path
    # stages pageable audio, which rocprofv3's tracing does not survive
    device = "--device" in sys.argv
    argv = [a for a in sys.argv if a not in ("--prof", "--device")]
    archs = argv[1].split(",") if len(argv) > 1 else ["qwen3-asr-0.6b", "qwen3-asr-1.7b"]
    lengths = [float(x) for x in argv[2].split(",")] if len(argv) > 2 else [1.0, 5.0, 12.0]
    for arch in archs:
        m = Model.synthetic(arch, seed=0)
        s = m.session(kv_type="f16", n_ctx=32768)
        for secs in lengths:
            audio = speech_like(np.random.default_rng(0), int(secs * 16000))
            if device:
                import torch
                dev = torch.from_numpy(audio).cuda()
                torch.cuda.synchronize()

                def one():
                    return s.run_batch_device(dev.data_ptr(), [0], [audio.size], force_tokens_per_s=8)[0]
            else:
                def one():
                    return s.run(audio, force_tokens_per_s=8)
            for _ in range(2):
                one()
            times, stages = [], None
            for _ in range(10):
                t0 = time.perf_counter()
                r = one()
                times.append(time.perf_counter() - t0)
                stages = r
            ms = np.array(times) * 1e3
            breakdown = None
            if prof:   # one extra eager run with HIP events around every launch: per-kernel-class time
                lib = _lib.load()
                _lib.check(lib.qasr_prof_reset())
                _lib.check(lib.qasr_prof_enable(1))
                one()
                _lib.check(lib.qasr_prof_enable(0))
                need = C.c_size_t()
                lib.qasr_prof_report(None, 0, C.byref(need))
                buf = C.create_string_buffer(need.value)
                _lib.check(lib.qasr_prof_report(buf, need.value, C.byref(need)))
                breakdown = {k: {"count": v["count"], "ms": round(v["ms"], 3)}
                             for k, v in sorted(json.loads(buf.value.decode()).items(), key=lambda kv: -kv[1]["ms"])}
            print(json.dumps({"arch": arch, "audio_s": secs, "tokens": len(stages.tokens),
                              "p50_ms": round(float(np.median(ms)), 2), "p95_ms": round(float(np.percentile(ms, 95)), 2),
                              "rtf_inv": round(secs / (np.median(ms) / 1e3), 1),
                              "stage_ms": {k: round(v, 2) for k, v in stages.timings_ms.items()},
                              **({"eager_kernel_ms": breakdown} if breakdown else {})}), flush=True)
        s.close()
        m.close()


if __name__ == "__main__":
    main()
