#!/usr/bin/env python3
"""Experiment: the C4 bench workload split into P sub-batches run concurrently by P sessions (one host thread and
one HIP stream each) on one GPU — does overlapping independent decode loops fill the latency-bound GEMM / norm /
attention kernels?  usage: python tools/par_bench.py [P ...]"""
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from bench import FORCE_TPS, lpt_shard, make_workload  # noqa: E402
from qasr.transcribe_cpp import Model  # noqa: E402


def main():
    ps = [int(a) for a in sys.argv[1:]] or [1, 2, 3]
    audio = make_workload(1, 0)
    lens = [a.size for a in audio]
    total_s = sum(lens) / 16000.0
    dev = torch.from_numpy(np.concatenate(audio)).cuda()
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    model = Model.synthetic("qwen3-asr-1.7b", seed=0)
    sessions = [model.session(kv_type="f16", n_ctx=32768) for _ in range(max(ps))]
    for P in ps:
        shards = lpt_shard(lens, P)

        def work(i):
            idx = sorted(shards[i])
            sessions[i].run_batch_device(dev.data_ptr(), [offs[j] for j in idx], [lens[j] for j in idx],
                                         force_tokens_per_s=FORCE_TPS, want_results=False)

        def step():
            th = [threading.Thread(target=work, args=(i,)) for i in range(P)]
            for t in th:
                t.start()
            for t in th:
                t.join()

        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        print(f"P={P}: {dt * 1e3:.1f} ms/step, {total_s / dt:.1f} audio-s/s", flush=True)


if __name__ == "__main__":
    main()
