#!/usr/bin/env python3
"""conv 3×3 s2 + GELU timing at the C4 step's sizes (the encoder's two conv3x3 launches over ~1,900 one-second
chunks: 64×50 → 32×25 f16 out, 32×25 → 16×13 f32 out, 480 channels), plus a hash of each output so A/B builds
(QASR_LIB=…) can be checked for identical bits.  GPU.
usage: QASR_LIB=light-whisper_amd/libqasr.so python tools/conv_probe.py [chunks]"""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1900
    C = 480
    g = torch.Generator(device=dev).manual_seed(7)
    res = {"lib": os.path.basename(_lib.LIB_PATH), "chunks": n}
    for tag, hi, wi, mode in (("conv2", 64, 50, 0), ("conv3", 32, 25, 1)):
        x = (torch.randn(n, hi, wi, C, device=dev, generator=g) * 0.5).half()
        w = (torch.randn(C, 9, C, device=dev, generator=g) / (9 * C) ** 0.5).half()
        b = torch.randn(C, device=dev, generator=g) * 0.1
        ho, wo = (hi + 1) // 2, (wi + 1) // 2
        out = torch.empty(n * ho * wo * C, dtype=torch.float16 if mode == 0 else torch.float32, device=dev)

        def run():
            _lib.check(lib.qasr_op_conv3x3_gelu(x.data_ptr(), n, hi, wi, w.data_ptr(), b.data_ptr(), C,
                                                out.data_ptr(), mode, None))

        run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 5
        ev[0].record()
        for _ in range(reps):
            run()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        flops = 2.0 * n * ho * wo * C * 9 * C
        res[tag] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1),
                    "sha16": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]}
        del x, w, out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
