#!/usr/bin/env python3
"""Diagnosis (GPU): where a draft verify pass first departs from one decode step per token.  Runs a forced
continuation both ways with QASR_DUMP_DIR set (engine.cpp dump_rows: every decode-sized stage's output rows per
layer) and prints, per layer and stage, the rows whose bytes differ and the largest difference.
usage: python tools/diag_layers.py [arch] [seconds] [n] [audio seed] [prior runs: n1,n2,…]"""
import os
import re
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
TMP = tempfile.mkdtemp(prefix="qasr_dump_")
os.environ["QASR_DUMP_DIR"] = TMP   # read when the library loads
os.environ["QASR_NO_GRAPH"] = "1"   # dumps synchronise the stream: eager passes only (engine.cpp dump_rows)
from bench import speech_like  # noqa: E402

STAGES = {"x_in": np.float32, "qkv": np.float32, "att_q": np.int8, "att_d": np.float32, "x_mid": np.float32,
          "h_q": np.int8, "h_d": np.float32}


def load(d):
    out = []
    for f in sorted(os.listdir(d)):
        m = re.match(r"(\d+)_(\w+?)_L(\d+)_r(\d+)\.bin", f)
        what, l, rows = m.group(2), int(m.group(3)), int(m.group(4))
        a = np.fromfile(os.path.join(d, f), STAGES[what]).reshape(rows, -1)
        out.append((what, l, rows, a))
    return out


def main():
    from qasr.transcribe_cpp import Model

    arch = sys.argv[1] if len(sys.argv) > 1 else "qwen3-asr-1.7b"
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 17
    aseed = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    prior = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else []
    m = Model.synthetic(arch, seed=7)
    s = m.session(kv_type="f16", n_ctx=4096)
    audio = speech_like(np.random.default_rng(aseed), int(secs * 16000))
    for p in prior:   # earlier forced runs in the same session (the test's order)
        f = np.array([1000 + 37 * i for i in range(p)], np.int32)
        same = np.array_equal(s.forced_logits(audio, f), s.forced_logits(audio, f, one_pass=True))
        print(f"prior n={p}: {'identical' if same else 'DIFFER'}", flush=True)
    forced = np.array([1000 + 37 * i for i in range(n)], np.int32)
    da, db = os.path.join(TMP, "steps"), os.path.join(TMP, "verify")
    os.makedirs(da)
    os.makedirs(db)
    os.environ["QASR_DUMP_DIR"] = da
    ref = s.forced_logits(audio, forced)
    os.environ["QASR_DUMP_DIR"] = db
    got = s.forced_logits(audio, forced, one_pass=True)
    os.environ["QASR_DUMP_DIR"] = TMP
    d = np.abs(ref - got).max(1)
    print(f"{arch} {secs:g}s n={n} logits max diff per row: " + " ".join(f"{x:.2g}" for x in d), flush=True)
    steps = [x for x in load(da) if x[2] == 1]
    verify = [x for x in load(db) if x[2] == n]
    per_call = len(steps) // n
    assert per_call * n == len(steps) and per_call == len(verify), (len(steps), len(verify))
    shown = 0
    for j, (what, l, rows, b) in enumerate(verify):
        bad, mx = [], 0.0
        for i in range(n):
            w2, l2, _, a = steps[i * per_call + j]
            assert (w2, l2) == (what, l)
            if not np.array_equal(a[0], b[i]):
                bad.append(i)
                mx = max(mx, float(np.abs(a[0].astype(np.float64) - b[i].astype(np.float64)).max()))
        if bad:
            print(f"L{l:02d} {what:6s} rows differing {bad}  max {mx:.3g}", flush=True)
            shown += 1
            if shown >= 24:
                break
    if not shown:
        print("every dumped stage identical", flush=True)


if __name__ == "__main__":
    main()
