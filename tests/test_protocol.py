"""The native `engine` speaks the reference's stdio JSON protocol byte-for-byte.

Golden: the reference server loop (server_common.py:339-437 + qwen3_asr_server.py) driven with the reference
tests' fake engine/VAD (test_qwen3_asr_server.py:15-57) — tests/golden/protocol.json.  The native engine is
run with the same fakes (QASR_PROTOCOL_TEST_FAKE=1, no GPU needed); wall-clock fields are normalised.
"""
import json
import os
import re
import subprocess

import pytest

from qasr import _lib

G = os.path.join(os.path.dirname(__file__), "golden", "protocol.json")
TIMING_KEYS = {"vad_ms", "inference_ms", "average_inference_ms", "average_vad_ms"}


def _norm(obj):
    if isinstance(obj, dict):
        return {k: (type(v).__name__ if k in TIMING_KEYS else _norm(v)) for k, v in obj.items()}
    if isinstance(obj, str):
        return re.sub(r"耗时: [0-9.]+秒", "耗时: <t>秒", obj)
    return obj


def _run_engine(lines, env_extra, args=("serve", "--engine", "qwen3-asr-1.7b")):
    env = dict(os.environ, QASR_PROTOCOL_TEST_FAKE="1", **env_extra)
    return subprocess.run([_lib.ENGINE_PATH, *args], input="\n".join(lines) + "\n", capture_output=True, text=True,
                          env=env, timeout=60)


@pytest.fixture(scope="module")
def golden():
    return json.load(open(G, encoding="utf-8"))


def test_transcript_matches_reference(golden, tmp_path):
    res = _run_engine(golden["requests"], {"LIGHT_WHISPER_DATA_DIR": str(tmp_path), "HF_HUB_CACHE": str(tmp_path)})
    assert res.returncode == 0, res.stderr
    got = [ln for ln in res.stdout.splitlines() if ln.strip()]
    want = golden["replies"]
    # the reply after "exit" is never produced (the server stops reading)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        gj, wj = json.loads(g), json.loads(w)
        assert _norm(gj) == _norm(wj), (g, w)
        # key order and separators are part of the wire format (json.dumps(ensure_ascii=False))
        assert list(gj) == list(wj)
        if not (TIMING_KEYS & set(gj)) and "耗时" not in g and "stats" not in gj:
            assert g == w
    assert os.path.exists(os.path.join(tmp_path, "logs", "qwen3_asr_server.log"))


def test_stdout_is_protocol_only(golden, tmp_path):
    res = _run_engine(['{"action": "status", "request_id": 7}', '{"action": "exit"}'],
                      {"LIGHT_WHISPER_DATA_DIR": str(tmp_path)})
    lines = res.stdout.splitlines()
    assert all(json.loads(ln) is not None for ln in lines)
    assert json.loads(lines[1])["request_id"] == 7


def test_eof_exits_cleanly(tmp_path):
    res = _run_engine([], {"LIGHT_WHISPER_DATA_DIR": str(tmp_path)})
    assert res.returncode == 0
    assert json.loads(res.stdout.splitlines()[0])["success"] is True


def test_cli_rejects_unknown_engine(tmp_path):
    res = _run_engine([], {"LIGHT_WHISPER_DATA_DIR": str(tmp_path)}, args=("serve", "--engine", "whisper-large"))
    assert res.returncode == 2


def test_models_not_downloaded_without_fake(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("QASR_PROTOCOL_TEST_FAKE", "QASR_SYNTHETIC")}
    env.update(LIGHT_WHISPER_DATA_DIR=str(tmp_path), HF_HUB_CACHE=str(tmp_path))
    res = subprocess.run([_lib.ENGINE_PATH, "serve", "--engine", "qwen3-asr-0.6b"], input="", capture_output=True,
                         text=True, env=env, timeout=60)
    first = json.loads(res.stdout.splitlines()[0])
    assert first == {"success": False, "error": "Qwen3-ASR Q8 模型未下载: Qwen3-ASR-0.6B-Q8_0.gguf",
                     "type": "models_not_downloaded", "engine": "qwen3-asr-0.6b"}


def test_longform_cli_arguments(tmp_path):
    """`engine longform` (the native C5 host path): no recording → usage (2); no GGUF and no QASR_SYNTHETIC → the
    reference's not-downloaded message (1); a bad RANK / WORLD_SIZE → an error before any GPU work (1)"""
    env = {k: v for k, v in os.environ.items() if k not in ("QASR_SYNTHETIC", "RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(LIGHT_WHISPER_DATA_DIR=str(tmp_path), HF_HUB_CACHE=str(tmp_path))
    run = lambda *a, **e: subprocess.run([_lib.ENGINE_PATH, "longform", "--engine", "qwen3-asr-0.6b", *a],
                                         capture_output=True, text=True, env={**env, **e}, timeout=60)
    res = run()
    assert res.returncode == 1 and "Qwen3-ASR-0.6B-Q8_0.gguf" in res.stderr
    res = run(QASR_SYNTHETIC="1")
    assert res.returncode == 2 and "usage: engine longform" in res.stderr
    res = run(str(tmp_path / "x.wav"), QASR_SYNTHETIC="1", RANK="3", WORLD_SIZE="2")
    assert res.returncode == 1 and "bad RANK / WORLD_SIZE" in res.stderr


def test_path_mode_requests(tmp_path):
    """audio_path requests (qwen3_asr_server.py:256-267, the app's WAV fallback funasr_service.rs:1296-1323): the reply
    carries input_mode "path" and the duration of the decoded 16 kHz audio; an undecodable file is a
    transcription_error reply and the server keeps serving."""
    import numpy as np

    gdir = os.path.join(os.path.dirname(__file__), "golden")
    exp = np.load(os.path.join(gdir, "wav_expected.npz"))
    names = sorted({k.split("__")[0] for k in exp.files})
    reqs = [json.dumps({"action": "transcribe", "audio_path": os.path.join(gdir, "wav", n), "request_id": i})
            for i, n in enumerate(names)]
    reqs.append(json.dumps({"action": "transcribe", "audio_path": os.path.join(gdir, "wav", "adpcm4_mono_16k.wav"),
                            "request_id": 50}))
    reqs.append(json.dumps({"action": "status", "request_id": 51}))
    res = _run_engine(reqs + ['{"action": "exit"}'], {"LIGHT_WHISPER_DATA_DIR": str(tmp_path)})
    lines = [json.loads(ln) for ln in res.stdout.splitlines() if ln.strip()]
    replies = {r.get("request_id"): r for r in lines[1:]}
    for i, n in enumerate(names):
        r = replies[i]
        assert r["success"] is True and r["input_mode"] == "path", r
        assert r["duration"] == float(exp[n + "__duration"])
    bad = replies[50]
    assert bad["success"] is False and bad["type"] == "transcription_error" and bad["input_mode"] == "path"
    assert "Unsupported WAV sample format" in bad["error"]
    assert replies[51]["success"] is True


def test_fractional_sample_rate(tmp_path):
    """a float sample_rate is used as given (decode_inline_audio duration, `_resample` target length), not truncated"""
    import base64

    import numpy as np

    pcm = (np.arange(16000) % 200 - 100).astype("<i2")
    b64 = base64.b64encode(pcm.tobytes()).decode()
    req = json.dumps({"action": "transcribe", "audio_base64": b64, "audio_format": "pcm_s16le",
                      "sample_rate": 16000.5, "request_id": 1})
    res = _run_engine([req, '{"action": "exit"}'], {"LIGHT_WHISPER_DATA_DIR": str(tmp_path)})
    r = json.loads(res.stdout.splitlines()[1])
    assert r["success"] is True and r["duration"] == 16000 / 16000.5
