"""Phase timing of the persistent decode from its grid-wait stamps (QASR_PERSIST_STAMPS, kernels_persist.hip):
runs one single-utterance request (and one batch) with stamps on, prints per phase kind the critical work time
(last arrival − first release of the previous wait) and the wait latency (first release − last arrival), in µs.
usage: python tools/persist_stamps.py [arch] [rows]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, ROOT)
from bench import speech_like  # noqa: E402

NAMES7 = ["N1", "QKV", "ATT", "O", "N2", "GU", "D"]   # norms as phases
NAMES5 = ["QKV", "ATT", "O", "GU", "D"]               # norms folded into QKV / GU
MAXW = 512


def analyse(fn, grid):
    st = np.fromfile(fn, dtype=np.uint64).reshape(-1, MAXW, 2)[:grid].astype(np.int64)
    used = int(np.max(np.nonzero(st[0, :, 1])[0])) + 1
    arr, rel = st[:, :used, 0], st[:, :used, 1]
    last_arr = arr.max(0)
    first_rel = rel.min(0)
    last_rel = rel.max(0)
    work = np.empty(used)
    work[0] = np.nan
    work[1:] = (last_arr[1:] - first_rel[:-1]) / 100.0    # 100 MHz ticks → µs
    lat = (first_rel - last_arr) / 100.0
    skew = (last_rel - first_rel) / 100.0
    total = (last_rel[-1] - first_rel[0]) / 100.0
    print(f"waits {used}, total {total:.1f} µs between the first and the last wait")
    per = 5 if (used + 1) % 5 == 0 and (used + 1) % 7 != 0 else 7
    names = NAMES5 if per == 5 else NAMES7
    for k, nm in enumerate(names):
        idx = [w for w in range(1, used) if w % per == k]
        if not idx:
            continue
        print(f"  {nm:4s} work {np.nanmean(work[idx]):7.2f} µs   wait latency {lat[idx].mean():5.2f}   release skew {skew[idx].mean():5.2f}")


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "qwen3-asr-1.7b"
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    fn = os.path.join(ROOT, "gpurun_out", "persist_stamps.bin")
    os.environ["QASR_PERSIST"] = "1"
    os.environ["QASR_PERSIST_STAMPS"] = fn
    from qasr.transcribe_cpp import Model

    m = Model.synthetic(arch, seed=7)
    s = m.session(kv_type="f16", n_ctx=4096)
    clips = [speech_like(np.random.default_rng(100 + i), int(3.0 * 16000)) for i in range(rows)]
    if rows == 1:
        s.run(clips[0], force_tokens_per_s=8)
    else:
        s.run_batch(clips, force_tokens_per_s=8)
    st = np.fromfile(fn, dtype=np.uint64).reshape(-1, MAXW, 2)
    grid = int((st[:, 0, 1] != 0).sum())
    print(f"{arch} rows {rows} grid {grid}")
    analyse(fn, grid)
    s.close()
    m.close()


if __name__ == "__main__":
    main()
