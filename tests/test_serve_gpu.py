"""`engine serve` with the real HIP backend (the process the Rust app spawns: funasr_service.rs:917-972 →
engine.py:45-57 → server_common.BaseASRServer.run :339-437 → Qwen3ASRServer.transcribe_audio, qwen3_asr_server.py:
269-353).  QASR_SYNTHETIC=1 gives the seeded 0.6B weights (no GGUF is provisioned); FireRedVAD, the crop, the
decode and the reply are the production code.

Checked: the init line; a transcribe whose speech FireRedVAD accepts → vad_segments > 0 and the reply's text equal
to Session.run on the same cropped samples (the in-process C ABI, qwen3_asr_server.py:321,326); hot_words accepted
and ignored (the reference ignores them); stats; a short interim replay (interim.rs:135-156: the last
≤12 s re-sent each tick) followed by the final request; exit.  The interim replay runs at both model sizes — C3 is
quoted on qwen3-asr-1.7b — with the engine's defaults (prompt-lookup drafts and the encoder cache ON): every reply
equals the plain in-process Session.run (no drafts, no cache) bit for bit, the final request repeated gives the same
reply, and its first tokens match the oracle up to a clear-margin rule.
"""
import base64
import json
import os
import subprocess

import numpy as np
import pytest

from bench import recording

pytestmark = pytest.mark.gpu

ENGINE = "qwen3-asr-0.6b"
MAX_NEW = 48


class Engine:
    def __init__(self, tmp_path, extra=None, engine=ENGINE):
        from qasr import _lib

        env = {k: v for k, v in os.environ.items() if k not in ("QASR_PROTOCOL_TEST_FAKE",)}
        # synthetic weights rarely emit EOS: cap the natural decode (the reference decodes to EOS or n_ctx)
        env.update(QASR_SYNTHETIC="1", QASR_MAX_NEW_TOKENS=str(MAX_NEW), LIGHT_WHISPER_DATA_DIR=str(tmp_path),
                   HF_HUB_CACHE=str(tmp_path / "hf"), **(extra or {}))
        self.p = subprocess.Popen([_lib.ENGINE_PATH, "serve", "--engine", engine], stdin=subprocess.PIPE,
                                  stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env)
        self.init = json.loads(self.p.stdout.readline())

    def ask(self, obj):
        self.p.stdin.write(json.dumps(obj) + "\n")
        self.p.stdin.flush()
        line = self.p.stdout.readline()
        assert line, "engine closed stdout"
        return line, json.loads(line)

    def close(self):
        if self.p.poll() is None:
            try:
                self.ask({"action": "exit", "request_id": 99})
            finally:
                self.p.wait(timeout=30)


def pcm_request(audio_i16, rid, hot_words=None):
    req = {"action": "transcribe", "audio_base64": base64.b64encode(audio_i16.astype("<i2").tobytes()).decode(),
           "audio_format": "pcm_s16le", "sample_rate": 16000, "request_id": rid}
    if hot_words is not None:
        req["hot_words"] = hot_words
    return req


def _ref(engine):
    """in-process engine pieces on the same weights: the synthetic model (seed 0, as QASR_SYNTHETIC) + VAD; the
    session has no drafts and no encoder cache (the plain decode the served transcripts must equal bit for bit)"""
    from qasr.firered_vad import FireRedVad
    from qasr.transcribe_cpp import Model

    m = Model.synthetic(engine, seed=0)
    s = m.session(kv_type="f16", n_ctx=32768)
    v = FireRedVad()
    return m, s, v


@pytest.fixture(scope="module")
def ref(torch_dev):
    m, s, v = _ref(ENGINE)
    yield s, v
    v.close()
    s.close()
    m.close()


def crop(ref, audio_i16):
    """FireRedVAD crop of transcribe_audio (qwen3_asr_server.py:152-173): (samples, segments) or (None, 0)"""
    _, v = ref
    a = audio_i16.astype(np.float32) / 32768.0
    segs = v.speech_timestamps(a)
    if not segs:
        return None, 0
    st, en = max(0, segs[0]["start"]), min(a.size, segs[-1]["end"])
    return a[st:en], len(segs)


def expected(ref, audio_i16):
    """what transcribe_audio replies for this PCM: FireRedVAD crop → session.run → .strip()"""
    a, n = crop(ref, audio_i16)
    if a is None:
        return None, 0
    return ref[0].run(a, max_new_tokens=MAX_NEW).text.strip(), n


def speech_clip(seconds, seed):
    return np.clip(np.round(recording(seconds, seed) * 32768.0), -32768, 32767).astype(np.int16)


def test_serve_real_backend(ref, tmp_path):
    e = Engine(tmp_path)
    try:
        init = e.init
        assert init["success"] is True and init["model_loaded"] is True
        # qwen3_asr_server.py:208-223 key order; gpu_name / gpu_memory_total from hipGetDeviceProperties
        assert list(init) == ["success", "message", "model_loaded", "engine", "backend", "device", "gpu_name",
                              "gpu_memory_total"]
        assert init["engine"] == ENGINE and init["backend"] == "hip" and init["gpu_name"]
        assert init["gpu_memory_total"] > 0
        audio = speech_clip(4.0, 3)
        want, nseg = expected(ref, audio)
        assert nseg > 0, "FireRedVAD must accept the test clip"
        _, r = e.ask(pcm_request(audio, 1))
        assert r["success"] is True and r["request_id"] == 1
        assert r["vad_segments"] == nseg and r["input_mode"] == "memory" and r["backend"] == "hip"
        assert r["text"] == want and r["raw_text"] == want
        assert 0 < r["speech_duration"] <= 4.0 and r["duration"] == 4.0
        # hot_words are accepted and ignored: the same reply (timings aside)
        _, r2 = e.ask(pcm_request(audio, 2, hot_words=["Kubernetes", "张三", "ROCm"] * 30))
        assert r2["text"] == want and r2["vad_segments"] == nseg
        _, st = e.ask({"action": "stats", "request_id": 3})
        assert st["stats"]["transcription_count"] == 2 and st["stats"]["vad_calls"] == 2
        assert st["stats"]["backend"] == "hip" and st["request_id"] == 3
        # silence: VAD-rejected, Qwen not run
        _, r3 = e.ask(pcm_request(np.zeros(16000, np.int16), 4))
        assert r3["vad_segments"] == 0 and r3["text"] == "" and r3["inference_ms"] == 0.0
        _, st = e.ask({"action": "stats", "request_id": 5})
        assert st["stats"]["vad_rejected"] == 1 and st["stats"]["transcription_count"] == 2
    finally:
        e.close()
    assert e.p.returncode == 0


@pytest.fixture(scope="module", params=["qwen3-asr-0.6b", "qwen3-asr-1.7b"])
def ref_arch(request, torch_dev):
    m, s, v = _ref(request.param)
    yield request.param, (s, v)
    v.close()
    s.close()
    m.close()


def test_serve_interim_replay(ref_arch, tmp_path):
    """C3 (interim.rs:135-146): a recording growing in steps, each tick re-sends the last ≤12 s — growing
    windows, then sliding ones past 12 s — then the final request, sent twice.  The engine runs with its defaults
    (drafts + encoder cache on); every reply's text equals the plain in-process Session.run on the same crop (bit-
    identical transcripts: the drafts and the cache change the speed, not the tokens), and the repeated final request
    gives the same reply.  The final crop's first tokens match the oracle's greedy tokens up to a clear-margin rule."""
    import oracle

    engine, ref = ref_arch
    e = Engine(tmp_path, engine=engine)
    try:
        full = speech_clip(15.0, 4)
        ticks = [int(t * 16000) for t in (0.7, 1.4, 2.1, 5.6, 9.8, 11.2, 11.9, 12.6, 13.3, 14.0, 15.0)]
        for i, end in enumerate(ticks):
            win = full[max(0, end - 12 * 16000):end]
            line, r = e.ask(pcm_request(win, 100 + i, hot_words=["热词"]))
            assert r["success"] is True and r["request_id"] == 100 + i, line
            if win.size < 8000:
                assert r["text"] == "" and "vad_segments" not in r
                continue
            want, nseg = expected(ref, win)
            assert r["vad_segments"] == nseg
            assert r["text"] == (want or ""), (engine, i)
        finals = [e.ask(pcm_request(full, 200 + k))[1] for k in range(2)]
        want, nseg = expected(ref, full)
        assert nseg > 0 and all(f["vad_segments"] == nseg and f["text"] == want for f in finals), engine
        _, st = e.ask({"action": "stats", "request_id": 300})
        # (windows the VAD rejects or shorter than 0.5 s do not count: qwen3_asr_server.py:290-315)
        assert 2 <= st["stats"]["transcription_count"] <= len(ticks) + 2
    finally:
        e.close()
    # the final crop against the oracle (same seeded weights): first tokens equal up to a near-tie of the oracle logits
    a, _ = crop(ref, full)
    got = ref[0].run(a, max_new_tokens=12).tokens
    oracle.set_mode(engine=True)
    o = oracle.Model(oracle.arch_config(engine), seed=0)
    rmel, rtv = oracle.mel(a)
    remb = o.encode(rmel, rtv)
    sp = oracle.QWEN_SPECIAL
    ids = np.array(oracle.chat_prompt(remb.shape[0]), np.int32)
    toks, lg = oracle.KV(o, len(ids) + 16).generate(ids, sp["tok_audio_pad"], remb, eos=(sp["tok_eos0"], sp["tok_eos1"]),
                                                    max_new=12, want_logits=True)
    n = min(len(got), len(toks))
    div = next((j for j in range(n) if got[j] != toks[j]), n)
    if div < n:
        top2 = np.sort(lg[div])[-2:]
        # the near-tie rule of every parity test: top-2 gap below 0.5 % of the row's range
        assert top2[1] - top2[0] < 0.005 * (lg[div].max() - lg[div].min()), (engine, div, got, list(toks))
    assert div >= min(4, n), (engine, got, list(toks))


def _write_f32_wav(path, audio):
    """IEEE-float mono 16 kHz WAV (format 3): the samples round-trip bit for bit through qasr_audio_load_path"""
    data = np.asarray(audio, dtype="<f4").tobytes()
    fmt = (3).to_bytes(2, "little") + (1).to_bytes(2, "little") + (16000).to_bytes(4, "little") + \
        (64000).to_bytes(4, "little") + (4).to_bytes(2, "little") + (32).to_bytes(2, "little")
    body = b"WAVE" + b"fmt " + len(fmt).to_bytes(4, "little") + fmt + b"data" + len(data).to_bytes(4, "little") + data
    with open(path, "wb") as f:
        f.write(b"RIFF" + len(body).to_bytes(4, "little") + body)


def test_engine_longform_matches_python_pipeline(ref, tmp_path):
    """`engine longform` — the native C5 host path (no PyTorch: file unique-id hand-off, halo-sharded VAD, segmenter,
    LPT, one ASR batch, token gather; world 1 here) — gives the segments and token streams of the Python pipeline
    (qasr.longform + Session.run_batch) on the same 60 s recording and weights, and the parsed text of each"""
    from qasr import _lib, longform

    s, v = ref
    audio = recording(60.0, 5)
    wav = tmp_path / "rec.wav"
    _write_f32_wav(wav, audio)
    env = {k: val for k, val in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(QASR_SYNTHETIC="1", HF_HUB_CACHE=str(tmp_path / "hf"))
    out = subprocess.run([_lib.ENGINE_PATH, "longform", "--engine", ENGINE, "--force-tps", "8", str(wav)],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout)
    probs = longform.shard_probabilities(v, audio, 0, 1)
    segs = longform.segments(probs, audio.size)
    assert len(segs) >= 2 and got["segments_total"] == len(segs) and got["world"] == 1
    assert [(d["start"], d["end"]) for d in got["segments"]] == segs
    res = s.run_batch([audio[a:b] for a, b in segs], force_tokens_per_s=8)
    assert [d["tokens"] for d in got["segments"]] == [r.tokens for r in res]
    assert [d["text"] for d in got["segments"]] == [r.text for r in res]
    assert [d["language"] for d in got["segments"]] == [r.language or "" for r in res]


@pytest.mark.parametrize("stage", ["model", "vad", "asr"])
def test_engine_longform_failure_is_agreed(stage, tmp_path):
    """`engine longform` with an injected stage failure (QASR_FAIL_STAGE) at world 1 through the agreement path
    (QASR_LONGFORM_COMM=1: a one-rank communicator, qasr_dist_agree before each collective): the engine exits
    non-zero with the stage's reason and prints no result (the N-rank protocol itself: tests/test_shard_cpu.py::
    test_longform_stage_agreement_gloo); and with the communicator but no failure it still succeeds"""
    from qasr import _lib

    audio = recording(8.0, 6)
    wav = tmp_path / "rec.wav"
    _write_f32_wav(wav, audio)
    env = {k: val for k, val in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(QASR_SYNTHETIC="1", HF_HUB_CACHE=str(tmp_path / "hf"), QASR_LONGFORM_COMM="1",
               QASR_RDV_KEY=f"t{os.getpid()}_{stage}", QASR_RDV_DIR=str(tmp_path), QASR_FAIL_STAGE=stage)
    args = [_lib.ENGINE_PATH, "longform", "--engine", "qwen3-asr-0.6b", "--force-tps", "8", str(wav)]
    out = subprocess.run(args, capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 1 and out.stdout == "", (out.returncode, out.stdout[:200], out.stderr[-2000:])
    assert f"injected failure (QASR_FAIL_STAGE={stage})" in out.stderr, out.stderr[-2000:]
    if stage == "asr":
        env.pop("QASR_FAIL_STAGE")
        ok = subprocess.run(args, capture_output=True, text=True, env=env, timeout=300)
        assert ok.returncode == 0, ok.stderr[-2000:]
        assert json.loads(ok.stdout)["world"] == 1


def test_engine_longform_rank_never_joins(tmp_path):
    """`engine longform` at world 2 where rank 1 fails before it joins the communicator (QASR_FAIL_STAGE=init,
    QASR_FAIL_RANK=1): rank 1 exits with the injected reason, and rank 0 — blocked in the communicator init — exits
    non-zero at the communicator's deadline (QASR_DIST_TIMEOUT_MS) instead of hanging (the
    reference's expectation is a process that exits, funasr_service.rs:1367-1385).  Only rank 0 ever opens RCCL on the
    card, so one GPU serves both ranks."""
    import time

    from qasr import _lib

    audio = recording(4.0, 3)
    wav = tmp_path / "rec.wav"
    _write_f32_wav(wav, audio)
    base = {k: val for k, val in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    base.update(QASR_SYNTHETIC="1", HF_HUB_CACHE=str(tmp_path / "hf"), QASR_RDV_KEY=f"nj{os.getpid()}",
                QASR_RDV_DIR=str(tmp_path), QASR_FAIL_STAGE="init", QASR_FAIL_RANK="1", QASR_DIST_TIMEOUT_MS="6000",
                WORLD_SIZE="2", LOCAL_RANK="0")
    args = [_lib.ENGINE_PATH, "longform", "--engine", "qwen3-asr-0.6b", "--force-tps", "8", str(wav)]
    t0 = time.monotonic()
    p0 = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env={**base, "RANK": "0"})
    p1 = subprocess.run(args, capture_output=True, text=True, env={**base, "RANK": "1"}, timeout=120)
    try:
        out0, err0 = p0.communicate(timeout=90)
    except subprocess.TimeoutExpired:
        p0.kill()
        out0, err0 = p0.communicate()
        raise AssertionError("rank 0 still blocked 90 s after start: " + err0[-2000:])
    took = time.monotonic() - t0
    assert p1.returncode == 1 and "injected failure (QASR_FAIL_STAGE=init)" in p1.stderr, p1.stderr[-2000:]
    assert p0.returncode == 1 and out0 == "", (p0.returncode, out0[:200], err0[-2000:])
    assert "timed out" in err0, err0[-2000:]
    print(f"rank 0 failed after {took:.1f} s: {err0.strip().splitlines()[-1][:300]}")
    assert took < 120
