#!/usr/bin/env python3
"""Write assets/warmup_noise.f32: the reference server's warm-up signal, np.random.default_rng(0).standard_normal(16000)
as float32 × 0.002 (qwen3_asr_server.py:139-140), 16,000 little-endian f32.  engine_main.cpp's warm-up reads it."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    audio = np.random.default_rng(0).standard_normal(16_000).astype(np.float32) * 0.002
    assert audio.dtype == np.float32
    audio.astype("<f4").tofile(os.path.join(ROOT, "assets", "warmup_noise.f32"))
