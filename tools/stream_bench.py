#!/usr/bin/env python3
"""C3 streaming workload: a 60 s recording (seed 3) replayed in simulated real time through the
native `engine serve` process over the reference stdio/JSON protocol, the way the app's interim loop drives the
sidecar (src-tauri/src/services/audio_service/interim.rs:95-195, constants in audio_service/mod.rs:10-20):

  * a tick every `interval` ms (220 to start; adjust_interval: −24 ms after a request ≤ 180 ms, +42 ms after one
    ≥ 420 ms, clamped to [140, 460]); a tick sends a request once ≥ 0.2 s of audio exist and ≥ 1024 new samples
    arrived since the last one;
  * each request carries the last ≤ 12 s as inline pcm_s16le base64 plus 100 hot words (accepted and ignored,
    as by the reference server);
  * requests are serial (the app holds a mutex across write + read); the simulated clock advances by the measured
    round-trip time;
  * a final request with the whole recording once the recording ends.

Model: QASR_SYNTHETIC=1 (seeded synthetic 1.7B weights — no checkpoint in the container) with
QASR_FORCE_TOKENS_PER_S=8 so every request does a deterministic amount of decode work.  Prints one JSON line:
per-request p50 / p95 round-trip latency, the engine's own inference / VAD times and RTF⁻¹ of the final request.
Usage: stream_bench.py [--seconds 60] [--engine qwen3-asr-1.7b]"""
import argparse
import base64
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import recording, speech_like  # noqa: E402

SR = 16000
MIN_INTERIM_S, MIN_GROWTH, WINDOW_S = 0.2, 1024, 12.0
I_MIN, I_BASE, I_MAX, I_DOWN, I_UP, HEAVY, LIGHT = 140, 220, 460, 24, 42, 420, 180


def adjust_interval(cur, elapsed_ms):   # interim.rs adjust_interval, executed = true
    if elapsed_ms >= HEAVY:
        return min(cur + I_UP, I_MAX)
    if elapsed_ms <= LIGHT:
        return max(cur - I_DOWN, I_MIN)
    if cur > I_BASE:
        return max(cur - 8, I_BASE)
    if cur < I_BASE:
        return min(cur + 4, I_BASE)
    return cur


class Engine:
    def __init__(self, engine, env_extra):
        env = dict(os.environ)
        env.update(env_extra)
        self.p = subprocess.Popen([os.path.join(ROOT, "light-whisper_amd", "engine"), "serve", "--engine", engine],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env)
        self.init = json.loads(self.p.stdout.readline())
        self.rid = 0

    def request(self, obj):
        """-> (reply, round-trip seconds from the first byte written to the reply line read; the client's own
        JSON/base64 encoding — the Rust caller's work — is done before the clock starts)"""
        self.rid += 1
        obj["request_id"] = self.rid
        line = (json.dumps(obj, ensure_ascii=False) + "\n").encode()
        t0 = time.perf_counter()
        self.p.stdin.write(line)
        self.p.stdin.flush()
        raw = self.p.stdout.readline()
        dt = time.perf_counter() - t0
        reply = json.loads(raw)
        assert reply.get("request_id") == self.rid, reply
        return reply, dt

    def close(self):
        try:
            self.request({"action": "exit"})
        finally:
            self.p.wait(timeout=30)


def transcribe_req(pcm, hot_words):
    b = (np.clip(pcm, -1.0, 1.0) * 32767.0).astype("<i2").tobytes()
    return {"action": "transcribe", "audio_base64": base64.b64encode(b).decode(), "audio_format": "pcm_s16le",
            "sample_rate": SR, "hot_words": hot_words}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--engine", default="qwen3-asr-1.7b")
    ap.add_argument("--speech-only", action="store_true",
                    help="continuous speech-like audio (no pauses): every window is ~12 s of speech the VAD keeps, "
                         "the full-load case (the default recording's pauses let the VAD trim windows)")
    ap.add_argument("--draft", type=int, default=1, help="QASR_STREAM_DRAFT (prompt-lookup drafts, 1 = default on)")
    ap.add_argument("--enc-cache", type=int, default=1,
                    help="QASR_STREAM_ENC_CACHE (encoder windows of growing interim windows reused, 1 = default on)")
    ap.add_argument("--draft-noise", type=float, default=0.0,
                    help="QASR_DRAFT_NOISE: replace each proposed draft token by a random id with this probability "
                         "(acceptance below the degenerate 100 %% of synthetic transcripts; the output is unchanged)")
    a = ap.parse_args()
    audio = (speech_like(np.random.default_rng(3), int(a.seconds * SR)) if a.speech_only else
             recording(a.seconds, seed=3))
    hot = [f"热词{i:03d}" for i in range(100)]
    with tempfile.TemporaryDirectory() as tmp:
        eng = Engine(a.engine, {"QASR_SYNTHETIC": "1", "QASR_FORCE_TOKENS_PER_S": "8", "HF_HUB_CACHE": tmp,
                                "LIGHT_WHISPER_DATA_DIR": tmp, "QASR_STREAM_DRAFT": str(a.draft),
                                "QASR_STREAM_ENC_CACHE": str(a.enc_cache), "QASR_DRAFT_NOISE": str(a.draft_noise)})
        assert eng.init.get("success"), eng.init
        eng.request(transcribe_req(audio[: 2 * SR], hot))   # first-request warm-up (graphs, buffers)
        clock, interval, last, lat, inf, vad, sizes, speech = 0.0, I_BASE, 0, [], [], [], [], []
        while True:
            clock += interval / 1e3
            if clock >= a.seconds:
                break
            avail = int(clock * SR)
            if avail < MIN_INTERIM_S * SR or avail - last < MIN_GROWTH:
                interval = min(max(interval - 8, I_MIN), I_BASE)   # adjust_interval, executed = false
                continue
            window = audio[max(0, avail - int(WINDOW_S * SR)): avail]
            r, dt = eng.request(transcribe_req(window, hot))
            assert r.get("success"), r
            last = avail
            lat.append(dt * 1e3)
            inf.append(r.get("inference_ms", 0.0))
            vad.append(r.get("vad_ms", 0.0))
            sizes.append(window.size / SR)
            speech.append(r.get("speech_duration", 0.0))
            clock += dt
            interval = adjust_interval(interval, dt * 1e3)
        fin, fin_s = eng.request(transcribe_req(audio, hot))
        fin_ms = fin_s * 1e3
        stats, _ = eng.request({"action": "stats"})
        eng.close()
    lat = np.array(lat)
    out = {"workload": f"C3 streaming: {a.seconds:g} s " + ("continuous speech-like audio" if a.speech_only else
                                                               "recording (seed 3)")
                       + ", interim ticks (interim.rs policy), ≤12 s windows, 100 hot words, + final request",
           "draft": bool(a.draft), "draft_noise": a.draft_noise, "encoder_cache": bool(a.enc_cache),
           "engine": a.engine, "weights": "synthetic (QASR_SYNTHETIC=1), 8 forced tokens/audio-s",
           "requests": int(lat.size), "mean_window_s": round(float(np.mean(sizes)), 2),
           "p50_ms": round(float(np.median(lat)), 2), "p95_ms": round(float(np.percentile(lat, 95)), 2),
           "max_ms": round(float(lat.max()), 2), "engine_inference_p50_ms": round(float(np.median(inf)), 2),
           "engine_vad_p50_ms": round(float(np.median(vad)), 2),
           "speech_s_p50": round(float(np.median(speech)), 2), "vad_rejected": int(sum(1 for x in speech if x == 0)),
           "interim_rtf_inv": round(float(np.sum(sizes) / (lat.sum() / 1e3)), 1),
           "final": {"audio_s": round(audio.size / SR, 1), "round_trip_ms": round(fin_ms, 1),
                     "inference_ms": fin.get("inference_ms"), "vad_ms": fin.get("vad_ms"),
                     "speech_duration": fin.get("speech_duration"),
                     "rtf_inv": round(audio.size / SR / (fin_ms / 1e3), 1)},
           "prompt_lookup": stats.get("stats", {}).get("prompt_lookup"),
           "encoder_cache_stats": stats.get("stats", {}).get("encoder_cache")}
    print(json.dumps(out, ensure_ascii=False), flush=True)


if __name__ == "__main__":
    main()
