"""Persistent decode (kernels_persist.hip) against the launch chain, 1.7B synthetic weights: tokens of single runs and
of batches (batch-invariant mode: exact lm_head too) must be equal bit for bit; prints timings.
usage: python tools/persist_check.py [arch] [n_batch]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, ROOT)
from bench import speech_like  # noqa: E402


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "qwen3-asr-1.7b"
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from qasr.transcribe_cpp import Model

    m = Model.synthetic(arch, seed=7)
    os.environ["QASR_PERSIST"] = "0"
    s0 = m.session(kv_type="f16", n_ctx=4096)
    os.environ["QASR_PERSIST"] = "1"
    s1 = m.session(kv_type="f16", n_ctx=4096)
    rng = np.random.default_rng(3)
    secs = rng.uniform(2.0, 12.0, size=nb)
    secs[0] = 12.0
    clips = [speech_like(np.random.default_rng(100 + i), int(x * 16000)) for i, x in enumerate(secs)]
    for name, s in (("chain", s0), ("persist", s1)):
        s.run(clips[1], force_tokens_per_s=8)
        t = time.perf_counter()
        r = s.run(clips[1], force_tokens_per_s=8)
        print(f"{name}: single {secs[1]:.1f}s {len(r.tokens)} tokens {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
    a = s0.run(clips[0], force_tokens_per_s=8).tokens
    b = s1.run(clips[0], force_tokens_per_s=8).tokens
    print("single 12 s equal:", a == b, len(a), flush=True)
    singles = [s0.run(c, force_tokens_per_s=8).tokens for c in clips]
    p1 = [s1.run(c, force_tokens_per_s=8).tokens for c in clips]
    print("singles persist == chain:", sum(x == y for x, y in zip(singles, p1)), "/", nb, flush=True)
    for s in (s0, s1):
        s.set_batch_invariant(True)
    for name, s in (("chain", s0), ("persist", s1)):
        s.run_batch(clips, force_tokens_per_s=8)
        t = time.perf_counter()
        bt = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
        dt = time.perf_counter() - t
        eq = sum(x == y for x, y in zip(bt, singles))
        print(f"{name}: batch-invariant batch of {nb}: {1e3 * dt:.1f} ms, {secs.sum() / dt:.0f} audio-s/s, "
              f"equal to singles {eq}/{nb}", flush=True)
    for s in (s0, s1):
        s.set_batch_invariant(False)
    for name, s in (("chain", s0), ("persist", s1)):
        s.run_batch(clips, force_tokens_per_s=8)
        t = time.perf_counter()
        bt = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
        dt = time.perf_counter() - t
        eq = sum(x == y for x, y in zip(bt, singles))
        print(f"{name}: default batch of {nb}: {1e3 * dt:.1f} ms, {secs.sum() / dt:.0f} audio-s/s, "
              f"equal to singles {eq}/{nb}", flush=True)
    s0.close()
    s1.close()
    m.close()


if __name__ == "__main__":
    main()
