#!/usr/bin/env python3
"""C4 at full size (bench.py's 256-segment workload, seed 1, 1.7B synthetic, 8 forced tokens/s): the batch's token
streams against the 256 single runs; every divergence with the single path's teacher-forced logit margin (the
single run's own arithmetic: stable-order prefill, 1-row decode steps) in % of the row's range.  GPU."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, ROOT)
from bench import make_workload  # noqa: E402
from qasr.transcribe_cpp import Model  # noqa: E402


def main():
    m = Model.synthetic("qwen3-asr-1.7b", seed=7)
    s = m.session(kv_type="f16", n_ctx=4096)
    clips = make_workload(1, 0, seed=1, total=256)
    batch = [r.tokens for r in s.run_batch(clips, force_tokens_per_s=8)]
    singles = [s.run(c, force_tokens_per_s=8).tokens for c in clips]
    divs = []
    for i in range(len(clips)):
        d = next((j for j in range(len(batch[i])) if batch[i][j] != singles[i][j]), None)
        if d is None:
            continue
        lg = s.forced_logits(clips[i], np.asarray(singles[i][:d], np.int32))[d]
        rng = float(lg.max() - lg.min())
        top = np.sort(lg)[-2:]
        divs.append({"segment": i, "token": d, "of": len(batch[i]), "single_tok": int(singles[i][d]),
                     "batch_tok": int(batch[i][d]), "forced_argmax": int(lg.argmax()),
                     "margin_pct_of_range": round(100 * float(lg[singles[i][d]] - lg[batch[i][d]]) / rng, 3),
                     "top2_gap_pct": round(100 * float(top[1] - top[0]) / rng, 3)})
    out = {"segments": len(clips), "tokens": int(sum(len(b) for b in batch)),
           "first_tokens_equal": all(b[0] == x[0] for b, x in zip(batch, singles)),
           "diverging_segments": len(divs), "divergences": divs}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
