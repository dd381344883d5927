"""Host-side logic of libqasr (no GPU needed) against the reference's own behaviour.

  * the C ABI loads and exports every symbol include/qasr.h declares;
  * the segmenter (qasr_vad_timestamps_from_probabilities) vs FireRedVad._timestamps_from_probabilities
    outputs (firered_vad.py:121-191, golden vad_post.json);
  * pcm_s16le base64 decoding (server_common.py:145-187) and the linear resampler
    (qwen3_asr_server.py:230-243) vs the reference's outputs (golden audio_io.json);
  * the Python mirror of the FireRedVad post-processing API.
"""
import base64
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

from qasr import _lib
from qasr.firered_vad import FireRedVadOptions, timestamps_from_probabilities

G = os.path.join(os.path.dirname(__file__), "golden")
HDR = os.path.join(os.path.dirname(__file__), "..", "include", "qasr.h")


def test_header_symbols_exported():
    declared = set(re.findall(r"QASR_API\s+[^;(]*?\b(qasr_\w+)\s*\(", open(HDR).read()))
    assert len(declared) >= 40
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    missing = declared - _lib.exported_symbols()
    assert not missing, missing


def test_version_and_backend_errors():
    lib = _lib.load()
    assert b"gfx950" in lib.qasr_version()
    h = C.c_void_p()
    for be in (b"cuda", b"vulkan", b"cpu"):
        rc = lib.qasr_model_open(b"/nonexistent.gguf", be, C.byref(h))
        assert rc == 4  # QASR_E_BACKEND — no non-HIP backend exists
        assert be.decode() in lib.qasr_last_error().decode()


def test_segmenter_matches_reference():
    cases = json.load(open(os.path.join(G, "vad_post.json")))
    for c in cases:
        o = c["options"]
        opts = FireRedVadOptions(**o)
        assert timestamps_from_probabilities(c["probs"], c["audio_len"], opts) == c["expected"], o


def test_decode_pcm_matches_reference():
    d = json.load(open(os.path.join(G, "audio_io.json")))
    lib = _lib.load()
    for case in d["decode"]:
        b = case["payload"].encode()
        n = C.c_size_t()
        out = np.empty(len(b), np.float32)
        _lib.check(lib.qasr_decode_pcm_s16le(b, len(b), out.ctypes.data_as(C.c_void_p), out.size, C.byref(n)))
        ref = np.asarray(case["audio"], np.float32)
        assert n.value == ref.size and np.array_equal(out[: n.value], ref)
        assert n.value / case["sample_rate"] == case["duration"]
    for case in d["decode_errors"]:
        if case["format"] != "pcm_s16le" or not case["payload"] or case["sample_rate"] == 0:
            continue  # format / rate checks live in the server loop (tests/test_protocol.py)
        b = case["payload"].encode()
        n = C.c_size_t()
        rc = lib.qasr_decode_pcm_s16le(b, len(b), None, 0, C.byref(n))
        assert rc != 0
        msg = lib.qasr_last_error().decode()
        assert msg in case["error"], (msg, case["error"])


def test_resample_matches_reference():
    d = json.load(open(os.path.join(G, "audio_io.json")))
    lib = _lib.load()
    for case in d["resample"]:
        x = np.asarray(case["x"], np.float32)
        ref = np.asarray(case["y"], np.float32)
        n = C.c_size_t()
        out = np.empty(max(ref.size, 1), np.float32)
        _lib.check(lib.qasr_resample_linear(x.ctypes.data_as(C.c_void_p), x.size, case["sr"],
                                            out.ctypes.data_as(C.c_void_p), out.size, C.byref(n)))
        assert n.value == ref.size
        assert np.array_equal(out[: n.value], ref), (case["sr"], np.abs(out[: n.value] - ref).max())


def test_base64_edge_cases():
    lib = _lib.load()
    n = C.c_size_t()
    pcm = np.arange(-5, 5, dtype="<i2")
    b = base64.b64encode(pcm.tobytes())
    out = np.empty(10, np.float32)
    _lib.check(lib.qasr_decode_pcm_s16le(b, len(b), out.ctypes.data_as(C.c_void_p), 10, C.byref(n)))
    assert np.array_equal(out, pcm.astype(np.float32) / 32768.0)
    assert lib.qasr_decode_pcm_s16le(b"AAE", 3, None, 0, C.byref(n)) == 3           # Incorrect padding
    assert lib.qasr_decode_pcm_s16le(b"AAAA", 4, None, 0, C.byref(n)) == 1          # odd byte count (3 bytes)
    assert lib.qasr_decode_pcm_s16le(b"!!!!", 4, None, 0, C.byref(n)) == 3          # Non-base64 digit found


def test_utf8_replace_matches_python():
    """transcript bytes → UTF-8 exactly as bytes.decode("utf-8", "replace") (the Qwen2 tokenizer's decode)"""
    lib = _lib.load()
    rng = np.random.default_rng(3)
    pool = [bytes([b]) for b in range(256)] + [c.encode() for c in "aé中😀ß€"] + [b"\xe4\xb8", b"\xf0\x9f\x98",
                                                                               b"\xed\xa0\x80", b"\xc0\xaf"]
    cases = [b"", b"plain ascii", "中文 text".encode(), b"\xff\xfe", b"\xe4\xb8\x41", b"\xf4\x90\x80\x80"]
    cases += [b"".join(pool[i] for i in rng.integers(0, len(pool), int(rng.integers(1, 40)))) for _ in range(3000)]
    buf = C.create_string_buffer(512)
    n = C.c_size_t()
    for b in cases:
        _lib.check(lib.qasr_utf8_replace_invalid(b, len(b), buf, 512, C.byref(n)))
        assert buf.raw[: n.value] == b.decode("utf-8", "replace").encode(), b
