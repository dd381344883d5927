"""The CPU oracle pinned against the committed golden fixtures (runs without a GPU).

  * VAD segmenter vs the reference's own FireRedVad._timestamps_from_probabilities outputs (vad_post.json),
    including the two cases of the reference test test_firered_vad.py:25-50;
  * kaldi fbank + DFSMN vs the ONNX graph interpreted in numpy (dfsmn.npz) and the reference KAT
    (1 s of zeros → 98 frames, no speech; test_firered_vad.py:53-59);
  * log-mel, encoder, projector, decoder logits vs transformers' qwen3_asr in FLOAT mode (hf_tiny.npz).
"""
import json
import os

import numpy as np
import pytest

import oracle
from convert_vad import read_qvad

G = os.path.join(os.path.dirname(__file__), "golden")
VAD = os.path.join(os.path.dirname(__file__), "..", "assets", "fireredvad_dfsmn.qvad")


def _opts(o):
    return dict(threshold=o.get("threshold", 0.5), smooth_window=o.get("smooth_window_frames", 5),
                min_speech_ms=o.get("min_speech_duration_ms", 150), min_silence_ms=o.get("min_silence_duration_ms", 300),
                pad_ms=o.get("speech_pad_ms", 120))


def test_vad_segmenter_matches_reference():
    cases = json.load(open(os.path.join(G, "vad_post.json")))
    assert len(cases) >= 40
    for c in cases:
        got = oracle.vad_segments(np.array(c["probs"], np.float32), c["audio_len"], **_opts(c["options"]))
        assert got == c["expected"], c["options"]


def test_reference_postprocessing_cases():
    # test_firered_vad.py:25-50 verbatim inputs/expectations
    small = dict(smooth_window=1, min_speech_ms=100, min_silence_ms=200, pad_ms=0)
    p = np.concatenate([np.zeros(10), np.ones(9), np.zeros(30)]).astype(np.float32)
    assert oracle.vad_segments(p, 8000, **small) == []
    p = np.concatenate([np.zeros(20), np.ones(15), np.zeros(20), np.ones(15), np.zeros(30)]).astype(np.float32)
    assert oracle.vad_segments(p, 16000, **dict(small, pad_ms=120)) == [{"start": 1280, "end": 13120}]


@pytest.fixture(scope="module")
def dfsmn():
    return np.load(os.path.join(G, "dfsmn.npz")), read_qvad(VAD)


@pytest.mark.parametrize("name", ["zeros_1s", "tone_bursts_3s", "noise_0p7s", "short_399", "one_frame_400"])
def test_fbank_and_dfsmn(dfsmn, name):
    d, w = dfsmn
    audio = d[f"{name}__audio"]
    pcm = np.clip(audio * 32768.0, -32768.0, 32767.0).astype(np.float32)  # firered_vad.py:89
    feats = oracle.fbank(pcm)
    assert feats.shape == d[f"{name}__feats"].shape
    if feats.size:
        assert np.abs(feats - d[f"{name}__feats"]).max() < 1e-3
    probs = oracle.vad_probabilities(feats, w)
    assert probs.shape == d[f"{name}__probs"].shape
    if probs.size:
        assert np.abs(probs - d[f"{name}__probs"]).max() < 1e-5


def test_reference_kat_zeros(dfsmn):
    _, w = dfsmn
    z = np.zeros(16000, np.float32)
    probs = oracle.vad_probabilities(oracle.fbank(z), w)
    assert probs.shape == (98,)
    assert oracle.vad_segments(probs, z.size) == []


@pytest.mark.parametrize("t", [1, 2, 25, 333])
def test_dfsmn_graph_on_random_features(dfsmn, t):
    d, w = dfsmn
    f = d[f"randfeat{t}__cmvn_feats"]
    raw = f / w["istd"] + w["mean"]
    assert np.abs(oracle.vad_probabilities(raw, w) - d[f"randfeat{t}__probs"]).max() < 1e-5


@pytest.fixture(scope="module")
def hf():
    return np.load(os.path.join(G, "hf_tiny.npz"))


@pytest.fixture(scope="module")
def float_model():
    from make_golden import TINY, TINY_SEED

    oracle.set_mode(engine=False)
    m = oracle.Model(TINY, seed=TINY_SEED)
    yield m
    oracle.set_mode(engine=True)


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_mel_matches_transformers(hf, tag):
    mel, tv = oracle.mel(hf[f"{tag}__audio"])
    assert tv == int(hf[f"{tag}__t_valid"])
    assert np.abs(mel - hf[f"{tag}__mel"]).max() < 1e-4


def test_mel_filters_match_transformers():
    from transformers.audio_utils import mel_filter_bank

    ref = mel_filter_bank(num_frequency_bins=201, num_mel_filters=128, min_frequency=0.0, max_frequency=8000.0,
                          sampling_rate=16000, norm="slaney", mel_scale="slaney").astype(np.float32)
    assert np.abs(oracle.mel_filters(128) - ref).max() < 1e-7


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_encoder_matches_transformers(float_model, hf, tag):
    proj, enc = float_model.encode(hf[f"{tag}__mel"], int(hf[f"{tag}__t_valid"]), want_enc=True)
    assert np.abs(enc - hf[f"{tag}__enc"]).max() < 1e-4
    assert np.abs(proj - hf[f"{tag}__proj"]).max() < 1e-4


def test_decoder_matches_transformers(float_model, hf):
    ids = hf["dec__ids"]
    kv = oracle.KV(float_model, 128)
    x = kv.embed(ids)
    x[ids == 4000] = hf["b__proj"]
    lg = kv.forward(x, all_logits=True)
    ref = hf["dec__logits"]
    assert np.abs(lg - ref).max() < 1e-3 * np.abs(ref).max()
    assert (lg.argmax(1) == ref.argmax(1)).all()


def test_q8_roundtrip_and_block_dots():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((4, 256)).astype(np.float32)
    q = oracle.quantize_q8(x)
    y = oracle.dequantize_q8(q, 256)
    assert np.abs(y - x).max() <= np.abs(x).max() / 127 * 0.5 + 1e-6
    assert q.shape == (4, 8 * 34)


@pytest.mark.parametrize("arch,fixture", [("qwen3-asr-0.6b", "hf_06b.npz"), ("qwen3-asr-1.7b", "hf_17b.npz")])
def test_oracle_matches_transformers_at_real_dims(arch, fixture):
    """the oracle pinned at the real qwen3-asr-0.6b dimensions (18 encoder layers of d 896 / 14 heads
    with 104-token windows; 28 decoder layers, GQA 16/8, the 151,936-row tied vocabulary) against transformers'
    qwen3_asr on the same seeded synthetic weights (tests/golden/hf_06b.npz, make_golden.py make_hf_06b): log-mel,
    encoder / projector rows and float64 row sums, and the chat prompt's last 8 logit rows (top-64 entries + float64
    sums).  Oracle in float mode (dequantised weights, f32 activations: HF's own arithmetic, f32 summation order
    aside).  Round 6: the same at qwen3-asr-1.7b (24 encoder layers of d 1,024 / 16 heads, decoder d 2,048 / FFN 6,144:
    tests/golden/hf_17b.npz, make_hf_17b) — the model C4 / C5 are quoted on."""
    import os

    hf = np.load(os.path.join(os.path.dirname(__file__), "golden", fixture))
    cfg = oracle.arch_config(arch)
    oracle.set_mode(engine=False)
    try:
        m = oracle.Model(cfg, seed=7)
        mel, tv = oracle.mel(hf["audio"])
        assert tv == int(hf["t_valid"]) == 1000
        assert np.abs(mel - hf["mel"]).max() < 1e-4
        proj, enc = m.encode(hf["mel"], tv, want_enc=True)
        assert proj.shape == (130, cfg["proj_out"]) and enc.shape == (130, cfg["enc_d"])
        rows = hf["enc_rows"]
        e_enc = np.abs(enc[rows] - hf["enc_sel"]).max() / np.abs(hf["enc_sel"]).max()
        e_proj = np.abs(proj[rows] - hf["proj_sel"]).max() / np.abs(hf["proj_sel"]).max()
        e_sum = np.abs(proj.astype(np.float64).sum(1) - hf["proj_sum"]).max() / np.abs(proj).max()
        ids = hf["ids"]
        kv = oracle.KV(m, 160)
        x = kv.embed(ids)
        x[ids == oracle.QWEN_SPECIAL["tok_audio_pad"]] = proj
        kv.forward(x[:-8])
        lg = np.concatenate([kv.forward(x[i:i + 1]) for i in range(len(ids) - 8, len(ids))])
        top_i, top_v = hf["logit_top_idx"], hf["logit_top_val"]
        span = np.abs(top_v).max()
        e_lg = np.abs(np.take_along_axis(lg, top_i, 1) - top_v).max() / span
        e_lsum = np.abs(lg.astype(np.float64).sum(1) - hf["logit_sum"]).max() / np.abs(hf["logit_abs_sum"]).max()
        print(f"{arch} dims vs HF: enc {e_enc:.2e} proj {e_proj:.2e} proj-sum {e_sum:.2e} logits {e_lg:.2e} "
              f"logit-sum {e_lsum:.2e}")
        # observed (r3): enc 6.9e-7, proj 7.8e-7, proj row sums 1.7e-5, logits 2.3e-7 of the span, logit sums 1.2e-8
        # (f32 summation order through 18 + 28 layers); bounds ≈ 10x
        assert e_enc < 1e-5 and e_proj < 1e-5 and e_sum < 2e-4
        assert e_lg < 3e-6 and e_lsum < 2e-7
        assert (lg.argmax(1) == top_i[:, 0]).all()
        # the top-64 set agrees wherever the 64th and 65th entries of HF's row are not within the error
        assert all(len(set(np.argsort(-lg[r])[:16]) ^ set(top_i[r, :16])) <= 2 for r in range(8))
    finally:
        oracle.set_mode(engine=True)
