"""FireRedVAD on the GPU through the C ABI vs the golden ONNX-graph interpretation and the reference KAT.

Pinned by: test_firered_vad.py:53-59 (1 s of zeros → 98 probabilities, no speech) and the DFSMN outputs of
the reference ONNX graph interpreted in numpy (tests/golden/dfsmn.npz).  Fbank tolerance is in the log
domain (FFT rounding differs from the numpy float64 restatement).
"""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
D = np.load(os.path.join(os.path.dirname(__file__), "golden", "dfsmn.npz"))
NAMES = ["zeros_1s", "tone_bursts_3s", "noise_0p7s", "short_399", "one_frame_400"]


@pytest.fixture(scope="module")
def vad(torch_dev):
    from qasr.firered_vad import FireRedVad

    v = FireRedVad()
    yield v
    v.close()


@pytest.mark.parametrize("name", NAMES)
def test_fbank(vad, name):
    f = vad.features(np.clip(D[f"{name}__audio"] * 32768.0, -32768, 32767) / 32768.0)
    ref = D[f"{name}__feats"]
    assert f.shape == ref.shape
    if f.size:
        assert np.abs(f - ref).max() < 2e-3


@pytest.mark.parametrize("name", NAMES)
def test_probabilities(vad, name):
    p = vad.probabilities(D[f"{name}__audio"])
    ref = D[f"{name}__probs"]
    assert p.shape == ref.shape
    if p.size:
        assert np.abs(p - ref).max() < 1e-4


def test_reference_kat_one_second_of_zeros(vad):
    z = np.zeros(16000, np.float32)
    assert vad.probabilities(z).shape == (98,)
    assert vad.speech_timestamps(z) == []


def _smoothed(p, win=5):
    """the segmenter's smoothed probabilities (firered_vad.py:121-191: moving mean, prefix mean for the first frames)"""
    c = np.cumsum(np.concatenate([[0.0], p.astype(np.float64)]))
    t = np.arange(p.size)
    lo = np.maximum(0, t - win + 1)
    return (c[t + 1] - c[lo]) / (t + 1 - lo)


def _burst_signal():
    rng = np.random.default_rng(11)
    t = np.arange(16000 * 6) / 16000.0
    env = (np.sin(2 * np.pi * 0.4 * t) > 0).astype(np.float32)
    voiced = sum(np.sin(2 * np.pi * 140 * k * t + rng.uniform(0, 6)) / k for k in range(1, 9))
    audio = (0.25 * env * voiced * (1 + 0.5 * np.sin(2 * np.pi * 4 * t)) + 0.003 * rng.standard_normal(t.size))
    return audio.astype(np.float32)


@pytest.mark.parametrize("case", ["bursts", "rec9s", "rec12s", "rec15s", "rec30s"])
def test_speech_timestamps_match_oracle_pipeline(vad, case):
    """integer segments (sample offsets) from INDEPENDENT probabilities: the GPU pipeline (HIP fbank → DFSMN → host
    segmenter) against the oracle's own fbank → DFSMN → segmenter on the same PCM, bit-exact.  The probabilities agree
    within 1e-3; each case's oracle smoothed probabilities stay > 2e-3 from the 0.5 threshold (checked here, on the
    CPU numbers), so that tolerance cannot move a speech/silence decision and the segments must be equal."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from bench import recording
    from convert_vad import read_qvad

    audio = _burst_signal() if case == "bursts" else \
        recording(*{"rec9s": (9.0, 3), "rec12s": (12.0, 4), "rec15s": (15.0, 7), "rec30s": (30.0, 6)}[case])
    audio = audio.astype(np.float32)
    w = read_qvad(os.path.join(os.path.dirname(__file__), "..", "assets", "fireredvad_dfsmn.qvad"))
    pcm = np.clip(audio * 32768.0, -32768, 32767).astype(np.float32)
    pr = oracle.vad_probabilities(oracle.fbank(pcm), w)
    assert np.abs(_smoothed(pr) - 0.5).min() > 2e-3, "case too close to the threshold for an exact comparison"
    want = oracle.vad_segments(pr, audio.size)
    assert want, "each case has speech"
    p = vad.probabilities(audio)
    assert np.abs(p - pr).max() < 1e-3
    assert vad.speech_timestamps(audio) == want


def test_sharded_long_form_probabilities_bit_identical(vad):
    """SURVEY §8(e) long-form VAD: each rank's halo-extended frame range gives exactly the single-pass
    probabilities of its core frames, for any number of ranks (here 1, 2, 3 and 7 simulated in one process)"""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from bench import recording
    from qasr import longform

    audio = recording(45.0, seed=2)
    full = vad.probabilities(audio)
    assert full.size == longform.n_frames(audio.size)
    for world in (1, 2, 3, 7):
        parts = [longform.shard_probabilities(vad, audio, r, world) for r in range(world)]
        assert np.array_equal(np.concatenate(parts), full), world
    assert longform.segments(full, audio.size) == [(s["start"], s["end"]) for s in vad.speech_timestamps(audio)]
