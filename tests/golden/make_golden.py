"""Generate the committed golden fixtures under tests/golden/ (run in the build container only).

Sources — every fixture is data (inputs + expected outputs); no reference source is copied:
  * vad_post.json      — outputs of the reference's own FireRedVad._timestamps_from_probabilities
                         (src-tauri/resources/firered_vad.py:121-191), imported from /root/reference, on the
                         two cases of test_firered_vad.py:25-50 plus seeded random probability tracks.
  * audio_io.json      — reference decode_inline_audio (server_common.py:145-187) and
                         Qwen3ASRServer._resample (qwen3_asr_server.py:230-243) outputs.
  * protocol.json      — stdin/stdout transcript of the reference server loop (server_common.py:339-437 +
                         qwen3_asr_server.py) driven with the reference tests' fake engine/VAD pattern
                         (test_qwen3_asr_server.py:15-57).
  * dfsmn.npz          — FireRedVAD DFSMN probabilities computed by interpreting the reference ONNX graph
                         node by node in numpy (independent of the C oracle), on kaldi-fbank features from a
                         numpy restatement of kaldi-native-fbank's defaults.  Includes the reference KAT input
                         (1 s of zeros, test_firered_vad.py:53-59).
  * hf_tiny.npz        — transformers 5.15 qwen3_asr (the in-container restatement of the model math, NOT the
                         reference engine) on a tiny seeded config: log-mel, encoder/projector outputs and
                         decoder logits, with weights from the shared synthetic generator (Q8_0 dequantised).
  * parse.json         — (language, transcription) from transformers' Qwen3-ASR output parser
                         (processing_qwen3_asr.py:159-196, the in-container restatement; transcribe.cpp's own
                         parser is absent, so parity with it stays unpinned) on hand-written and seeded cases.
  * wav/*.wav + wav_expected.npz — path-mode inputs (qwen3_asr_server.py:256-267): the reference's own
                         Qwen3ASRServer._load_audio run on these files with soundfile (absent here) replaced by a
                         stub that restates libsndfile's WAV decoding (integer PCM / 2^(bits-1), u8 − 128, float32
                         as is); the channel mean and _resample are the reference's code.

Usage: python tests/golden/make_golden.py   (needs /root/reference + transformers; not run on the GPU box)
"""
from __future__ import annotations

import base64
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
REF_RES = "/root/reference/src-tauri/resources"
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


# ---------------------------------------------------------------------------------------------- VAD post
def make_vad_post():
    sys.path.insert(0, REF_RES)
    from firered_vad import FireRedVad, FireRedVadOptions  # noqa: E402  (module import only; no knf/ort)

    def vad(**opts):
        v = object.__new__(FireRedVad)
        v.options = FireRedVadOptions(**opts)
        return v

    cases = []
    small = {"smooth_window_frames": 1, "min_speech_duration_ms": 100, "min_silence_duration_ms": 200,
             "speech_pad_ms": 0}
    p1 = np.concatenate([np.zeros(10), np.ones(9), np.zeros(30)]).astype(np.float32)
    cases.append({"probs": p1.tolist(), "audio_len": 8000, "options": small})
    p2 = np.concatenate([np.zeros(20), np.ones(15), np.zeros(20), np.ones(15), np.zeros(30)]).astype(np.float32)
    cases.append({"probs": p2.tolist(), "audio_len": 16000, "options": dict(small, speech_pad_ms=120)})
    rng = np.random.default_rng(1234)
    for i in range(40):
        t = int(rng.integers(1, 700))
        # bursty tracks: alternating speech/silence runs with noise, to exercise every state transition
        p = np.zeros(t, np.float32)
        pos = 0
        sp = bool(rng.integers(0, 2))
        while pos < t:
            run = int(rng.integers(1, 60))
            base = 0.8 if sp else 0.15
            p[pos:pos + run] = np.clip(base + rng.normal(0, 0.25, size=min(run, t - pos)), 0, 1)
            pos += run
            sp = not sp
        opts = {}
        if i % 3 == 1:
            opts = {"smooth_window_frames": int(rng.integers(1, 9)), "min_speech_duration_ms": int(rng.integers(0, 300)),
                    "min_silence_duration_ms": int(rng.integers(0, 500)), "speech_pad_ms": int(rng.integers(0, 300))}
        if i % 3 == 2:
            opts = {"threshold": float(rng.uniform(0.3, 0.7))}
        audio_len = int(t * 160 + rng.integers(-300, 400))
        cases.append({"probs": p.tolist(), "audio_len": max(audio_len, 0), "options": opts})
    cases.append({"probs": [], "audio_len": 0, "options": {}})
    for c in cases:
        c["expected"] = vad(**c["options"])._timestamps_from_probabilities(np.asarray(c["probs"], np.float32),
                                                                          c["audio_len"])
    json.dump(cases, open(os.path.join(HERE, "vad_post.json"), "w"))
    print("vad_post.json", len(cases))


# ---------------------------------------------------------------------------------------------- audio io
def make_audio_io():
    env = dict(os.environ, LIGHT_WHISPER_DATA_DIR=tempfile.mkdtemp())
    code = r"""
import base64, json, sys
import numpy as np
sys.path.insert(0, %r)
import server_common, qwen3_asr_server
rng = np.random.default_rng(7)
out = {"decode": [], "resample": []}
for n, sr in [(1, 16000), (160, 16000), (3201, 8000), (16000, 44100), (480, 16000.5)]:
    pcm = rng.integers(-32768, 32768, size=n).astype("<i2")
    payload = base64.b64encode(pcm.tobytes()).decode()
    audio, dur = server_common.decode_inline_audio(payload, "pcm_s16le", sr)
    out["decode"].append({"payload": payload, "sample_rate": sr, "duration": dur, "audio": audio.astype(float).tolist()})
errs = []
for payload, fmt, sr in [("", "pcm_s16le", 16000), ("AAE=", "pcm_s16le", 0), ("AAEC", "pcm_s16le", 16000),
                         ("!!!!", "pcm_s16le", 16000), ("AAA=", "mp3", 16000)]:
    try:
        server_common.decode_inline_audio(payload, fmt, sr)
        errs.append({"payload": payload, "format": fmt, "sample_rate": sr, "error": None})
    except Exception as e:
        errs.append({"payload": payload, "format": fmt, "sample_rate": sr, "error": str(e)})
out["decode_errors"] = errs
for n, sr in [(100, 8000), (441, 44100), (1000, 22050), (16000, 48000), (5, 16000), (0, 8000), (7, 96000),
              (1000, 16000.5), (441, 44100.7), (800, 8000.25), (3, 15999.9)]:
    x = rng.standard_normal(n).astype(np.float32)
    y = qwen3_asr_server.Qwen3ASRServer._resample(x, sr)
    out["resample"].append({"x": x.astype(float).tolist(), "sr": sr, "y": np.asarray(y, np.float32).astype(float).tolist()})
print(json.dumps(out))
""" % REF_RES
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, check=True)
    data = json.loads(res.stdout.strip().splitlines()[-1])
    json.dump(data, open(os.path.join(HERE, "audio_io.json"), "w"))
    print("audio_io.json", {k: len(v) for k, v in data.items()})


# ---------------------------------------------------------------------------------------------- protocol
def make_protocol():
    env = dict(os.environ, LIGHT_WHISPER_DATA_DIR=tempfile.mkdtemp(), HF_HUB_CACHE=tempfile.mkdtemp())
    pcm_silence = base64.b64encode(np.zeros(16000, "<i2").tobytes()).decode()
    pcm_ramp = base64.b64encode(np.arange(16000, dtype="<i2").tobytes()).decode()
    pcm_short = base64.b64encode(np.zeros(4000, "<i2").tobytes()).decode()
    lines = [
        json.dumps({"action": "status", "request_id": 1}),
        json.dumps({"action": "transcribe", "audio_base64": pcm_ramp, "audio_format": "pcm_s16le",
                    "sample_rate": 16000, "hot_words": ["光速", "ROCm"], "request_id": 2}, ensure_ascii=False),
        json.dumps({"action": "transcribe", "audio_base64": pcm_short, "audio_format": "pcm_s16le",
                    "sample_rate": 16000, "request_id": 3}),
        "this is not json",
        json.dumps({"action": "bogus", "request_id": 4}),
        json.dumps({"action": "stats", "request_id": 5}),
        json.dumps({"action": "transcribe", "audio_base64": "AAE", "audio_format": "pcm_s16le",
                    "sample_rate": 16000, "request_id": 6}),
        json.dumps({"action": "transcribe", "audio_path": "/nonexistent/file.wav", "request_id": 7}),
        json.dumps({"action": "transcribe", "audio_base64": pcm_silence, "audio_format": "pcm_s16le",
                    "sample_rate": 16000, "request_id": 8}),
        json.dumps({"action": "cleanup", "request_id": 9}),
        json.dumps({"action": "stats"}),
        json.dumps({"action": "exit", "request_id": 10}),
        json.dumps({"action": "status", "request_id": 11}),
    ]
    driver = r"""
import sys, types
from unittest import mock
import numpy as np
sys.path.insert(0, %r)
import qwen3_asr_server as q
class FakeSession:
    def run(self, audio, **kw):
        return types.SimpleNamespace(text="  测试文本 ", language="Chinese")
    def close(self): pass
class FakeModel:
    def __init__(self, path, backend): pass
    def session(self, **kw): return FakeSession()
    def close(self): pass
class FakeVad:
    calls = 0
    def warmup(self): pass
    def speech_timestamps(self, audio):
        # speech only where the input is not all zeros: [1600, 14400) like test_qwen3_asr_server.py:420
        return [] if not np.any(audio) else [{"start": 1600, "end": 6400}, {"start": 9600, "end": 14400}]
sys.modules["transcribe_cpp"] = types.SimpleNamespace(Model=FakeModel)
with mock.patch.object(q.Qwen3ASRServer, "_detect_device", return_value="cpu"), \
     mock.patch.object(q.Qwen3ASRServer, "_resolve_model_path", return_value="model.gguf"), \
     mock.patch.object(q.Qwen3ASRServer, "_warmup_inference"), \
     mock.patch.object(q, "FireRedVad", return_value=FakeVad()), \
     mock.patch("importlib.metadata.version", return_value="0.1.3"):
    q.Qwen3ASRServer(engine="qwen3-asr-1.7b").run()
""" % REF_RES
    res = subprocess.run([sys.executable, "-c", driver], input="\n".join(lines) + "\n", capture_output=True,
                         text=True, env=env, check=True)
    replies = [ln for ln in res.stdout.splitlines() if ln.strip()]
    json.dump({"engine": "qwen3-asr-1.7b", "requests": lines, "replies": replies},
              open(os.path.join(HERE, "protocol.json"), "w"), ensure_ascii=False, indent=0)
    print("protocol.json", len(lines), "requests", len(replies), "replies")


# ---------------------------------------------------------------------------------------------- DFSMN
def kaldi_fbank_numpy(pcm: np.ndarray) -> np.ndarray:
    """numpy restatement of kaldi-native-fbank 1.22.3 Fbank with firered_vad.py:65-72 options."""
    n = pcm.size
    if n < 400:
        return np.zeros((0, 80), np.float32)
    t = 1 + (n - 400) // 160
    idx = np.arange(t)[:, None] * 160 + np.arange(400)[None, :]
    fr = pcm.astype(np.float32)[idx]
    fr = fr - fr.mean(axis=1, keepdims=True, dtype=np.float32)
    pre = fr.copy()
    pre[:, 1:] = fr[:, 1:] - np.float32(0.97) * fr[:, :-1]
    pre[:, 0] = fr[:, 0] - np.float32(0.97) * fr[:, 0]
    win = np.power(0.5 - 0.5 * np.cos(2 * np.pi * np.arange(400) / 399.0), 0.85).astype(np.float32)
    x = np.zeros((t, 512), np.float64)
    x[:, :400] = pre * win
    spec = np.fft.rfft(x, axis=1)[:, :256]
    pw = (spec.real ** 2 + spec.imag ** 2).astype(np.float32)
    mel = lambda f: 1127.0 * np.log(1.0 + f / 700.0)  # noqa: E731
    lo, hi = mel(20.0), mel(8000.0)
    delta = (hi - lo) / 81
    fm = mel(31.25 * np.arange(256))
    banks = np.zeros((80, 256), np.float32)
    for b in range(80):
        left, center, right = lo + b * delta, lo + (b + 1) * delta, lo + (b + 2) * delta
        m = (fm > left) & (fm < right)
        banks[b, m] = np.where(fm[m] <= center, (fm[m] - left) / (center - left), (right - fm[m]) / (right - center))
    e = pw @ banks.T
    return np.log(np.maximum(e, np.finfo(np.float32).eps)).astype(np.float32)


def run_onnx_graph(model, feat: np.ndarray) -> np.ndarray:
    """Interpret the FireRedVAD ONNX graph (ops: MatMul Add Relu Transpose Conv Slice Pad Sigmoid) in numpy."""
    env = dict(model["initializers"])
    env["feat"] = feat.astype(np.float32)
    for n in model["nodes"]:
        ins = [env[i] if i else None for i in n["inputs"]]
        op, a = n["op"], n["attrs"]
        if op == "MatMul":
            r = np.matmul(ins[0], ins[1])
        elif op == "Add":
            r = ins[0] + ins[1]
        elif op == "Relu":
            r = np.maximum(ins[0], 0)
        elif op == "Sigmoid":
            r = 1.0 / (1.0 + np.exp(-ins[0]))
        elif op == "Transpose":
            r = np.transpose(ins[0], a["perm"])
        elif op == "Conv":  # depthwise 1-D, group == channels
            x, w = ins[0], ins[1]
            k = a["kernel_shape"][0]
            p0, p1 = a["pads"]
            xp = np.pad(x, ((0, 0), (0, 0), (p0, p1)))
            tout = xp.shape[2] - k + 1
            r = np.zeros((x.shape[0], x.shape[1], tout), np.float32)
            for j in range(k):
                r += w[None, :, 0, j:j + 1] * xp[:, :, j:j + tout]
        elif op == "Slice":
            data, st, en, ax, stp = ins
            sl = [slice(None)] * data.ndim
            sl[int(ax[0])] = slice(int(st[0]), int(en[0]) if en[0] < 2 ** 62 else None, int(stp[0]))
            r = data[tuple(sl)]
        elif op == "Pad":
            pads = ins[1]
            nd = ins[0].ndim
            r = np.pad(ins[0], [(int(pads[i]), int(pads[i + nd])) for i in range(nd)])
        else:
            raise NotImplementedError(op)
        env[n["outputs"][0]] = r.astype(np.float32)
    return env[model["outputs"][0]].reshape(-1)


def make_dfsmn():
    from convert_vad import load_reference_vad

    w, graph = load_reference_vad()
    rng = np.random.default_rng(99)
    inputs = {}
    inputs["zeros_1s"] = np.zeros(16000, np.float32)
    t = np.arange(48000) / 16000.0
    tone = 0.3 * np.sin(2 * np.pi * 220 * t) * (np.sin(2 * np.pi * 1.5 * t) > 0)
    inputs["tone_bursts_3s"] = (tone + 0.01 * rng.standard_normal(t.size)).astype(np.float32)
    inputs["noise_0p7s"] = (0.05 * rng.standard_normal(11200)).astype(np.float32)
    inputs["short_399"] = (0.1 * rng.standard_normal(399)).astype(np.float32)
    inputs["one_frame_400"] = (0.1 * rng.standard_normal(400)).astype(np.float32)
    out = {}
    for name, audio in inputs.items():
        pcm = np.clip(audio * 32768.0, -32768.0, 32767.0).astype(np.float32)  # firered_vad.py:89
        feats = kaldi_fbank_numpy(pcm)
        cm = (feats - w["mean"]) * w["istd"]
        probs = run_onnx_graph(graph, cm[None]) if feats.shape[0] else np.zeros(0, np.float32)
        out[f"{name}__audio"] = audio
        out[f"{name}__feats"] = feats
        out[f"{name}__probs"] = probs.astype(np.float32)
    # graph-only check on random CMVN'd features (no fbank dependency), incl. T=1 and T=2 edge cases
    for tt in (1, 2, 25, 333):
        f = rng.standard_normal((tt, 80)).astype(np.float32)
        out[f"randfeat{tt}__cmvn_feats"] = f
        out[f"randfeat{tt}__probs"] = run_onnx_graph(graph, f[None]).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "dfsmn.npz"), **out)
    print("dfsmn.npz", len(out), "arrays; KAT zeros frames:", out["zeros_1s__probs"].shape)


# ---------------------------------------------------------------------------------------------- HF tiny
TINY = dict(n_mels=128, conv_ch=64, enc_d=128, enc_layers=2, enc_heads=2, enc_ffn=256, n_window=50,
            n_window_infer=800, proj_out=256, txt_h=256, txt_layers=2, txt_heads=2, txt_kv_heads=1, head_dim=128,
            txt_ffn=512, vocab=4096, rope_theta=1000000.0, rms_eps=1e-6, ln_eps=1e-5)
TINY_SEED = 20260821


def tiny_tensors(cfg=TINY, seed=TINY_SEED):
    """Synthetic GGUF-style tensors from the oracle's generator (orc_model_synth) — the same values the
    product's on-device generator produces (checked by tests/test_model_gpu.py)."""
    import oracle

    return oracle.Model(cfg, seed=seed).export()


def hf_model(c, tens, audio_token_id):
    """transformers' Qwen3ASRForConditionalGeneration (the in-container stand-in for the model math) at
    config c, loaded with the synthetic GGUF-style tensors `tens` dequantised (Q8_0 → f32, f16 → f32)"""
    import torch
    from transformers import Qwen3ASRConfig, Qwen3ASRForConditionalGeneration

    import oracle

    torch.manual_seed(0)
    cfg = Qwen3ASRConfig(
        audio_config=dict(num_mel_bins=128, encoder_layers=c["enc_layers"], encoder_attention_heads=c["enc_heads"],
                          encoder_ffn_dim=c["enc_ffn"], d_model=c["enc_d"], n_window=50, output_dim=c["proj_out"],
                          n_window_infer=800, downsample_hidden_size=c["conv_ch"]),
        text_config=dict(model_type="qwen3", hidden_size=c["txt_h"], intermediate_size=c["txt_ffn"],
                         num_hidden_layers=c["txt_layers"], num_attention_heads=c["txt_heads"],
                         num_key_value_heads=c["txt_kv_heads"], head_dim=c["head_dim"], vocab_size=c["vocab"],
                         rms_norm_eps=c["rms_eps"], max_position_embeddings=4096, tie_word_embeddings=True,
                         rope_parameters={"rope_type": "default", "rope_theta": c["rope_theta"]}),
        audio_token_id=audio_token_id,
    )
    model = Qwen3ASRForConditionalGeneration(cfg).eval()

    def dq(name, k):
        return torch.from_numpy(oracle.dequantize_q8(tens[name], k))

    def f16(name):
        return torch.from_numpy(oracle.lib and tens[name].view(np.float16).astype(np.float32))

    sd = {}
    at = "model.audio_tower."
    for i in (1, 2, 3):
        sd[f"{at}conv2d{i}.weight"] = f16(f"a.conv{i}.weight")
        sd[f"{at}conv2d{i}.bias"] = torch.from_numpy(tens[f"a.conv{i}.bias"])
    sd[f"{at}conv_out.weight"] = dq("a.conv_out.weight", c["conv_ch"] * 16)
    for l in range(c["enc_layers"]):
        p = f"{at}layers.{l}."
        for hf, me in (("q_proj", "attn_q"), ("k_proj", "attn_k"), ("v_proj", "attn_v"), ("out_proj", "attn_out")):
            sd[p + f"self_attn.{hf}.weight"] = dq(f"a.blk.{l}.{me}.weight", c["enc_d"])
            sd[p + f"self_attn.{hf}.bias"] = torch.from_numpy(tens[f"a.blk.{l}.{me}.bias"])
        sd[p + "fc1.weight"] = dq(f"a.blk.{l}.ffn_up.weight", c["enc_d"])
        sd[p + "fc1.bias"] = torch.from_numpy(tens[f"a.blk.{l}.ffn_up.bias"])
        sd[p + "fc2.weight"] = dq(f"a.blk.{l}.ffn_down.weight", c["enc_ffn"])
        sd[p + "fc2.bias"] = torch.from_numpy(tens[f"a.blk.{l}.ffn_down.bias"])
        sd[p + "self_attn_layer_norm.weight"] = torch.from_numpy(tens[f"a.blk.{l}.ln1.weight"])
        sd[p + "self_attn_layer_norm.bias"] = torch.from_numpy(tens[f"a.blk.{l}.ln1.bias"])
        sd[p + "final_layer_norm.weight"] = torch.from_numpy(tens[f"a.blk.{l}.ln2.weight"])
        sd[p + "final_layer_norm.bias"] = torch.from_numpy(tens[f"a.blk.{l}.ln2.bias"])
    sd[f"{at}ln_post.weight"] = torch.from_numpy(tens["a.ln_post.weight"])
    sd[f"{at}ln_post.bias"] = torch.from_numpy(tens["a.ln_post.bias"])
    mp = "model.multi_modal_projector."
    sd[mp + "linear_1.weight"] = dq("a.proj1.weight", c["enc_d"])
    sd[mp + "linear_1.bias"] = torch.from_numpy(tens["a.proj1.bias"])
    sd[mp + "linear_2.weight"] = dq("a.proj2.weight", c["enc_d"])
    sd[mp + "linear_2.bias"] = torch.from_numpy(tens["a.proj2.bias"])
    lm = "model.language_model."
    sd[lm + "embed_tokens.weight"] = dq("token_embd.weight", c["txt_h"])
    sd[lm + "norm.weight"] = torch.from_numpy(tens["output_norm.weight"])
    for l in range(c["txt_layers"]):
        p = f"{lm}layers.{l}."
        sd[p + "input_layernorm.weight"] = torch.from_numpy(tens[f"blk.{l}.attn_norm.weight"])
        sd[p + "post_attention_layernorm.weight"] = torch.from_numpy(tens[f"blk.{l}.ffn_norm.weight"])
        sd[p + "self_attn.q_norm.weight"] = torch.from_numpy(tens[f"blk.{l}.attn_q_norm.weight"])
        sd[p + "self_attn.k_norm.weight"] = torch.from_numpy(tens[f"blk.{l}.attn_k_norm.weight"])
        for hf, me, k in (("q_proj", "attn_q", c["txt_h"]), ("k_proj", "attn_k", c["txt_h"]),
                          ("v_proj", "attn_v", c["txt_h"]), ("o_proj", "attn_output", c["txt_heads"] * c["head_dim"])):
            sd[p + f"self_attn.{hf}.weight"] = dq(f"blk.{l}.{me}.weight", k)
        sd[p + "mlp.gate_proj.weight"] = dq(f"blk.{l}.ffn_gate.weight", c["txt_h"])
        sd[p + "mlp.up_proj.weight"] = dq(f"blk.{l}.ffn_up.weight", c["txt_h"])
        sd[p + "mlp.down_proj.weight"] = dq(f"blk.{l}.ffn_down.weight", c["txt_ffn"])
    sd["lm_head.weight"] = sd[lm + "embed_tokens.weight"]
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if "positional_embedding" not in m]
    assert not missing and not unexpected, (missing, unexpected)
    return model


def make_hf_tiny():
    import torch
    from transformers.models.qwen3_asr.feature_extraction_qwen3_asr import Qwen3ASRFeatureExtractor

    model = hf_model(TINY, tiny_tensors(), 4000)
    fe = Qwen3ASRFeatureExtractor()
    rng = np.random.default_rng(5)
    out = {}
    # audio lengths: < min_length (0.3 s), partial chunk (2.37 s), > 8 s attention window (10.46 s)
    for tag, n in (("a", 4800), ("b", 37920), ("c", 167360)):
        tt = np.arange(n) / 16000.0
        audio = (0.2 * np.sin(2 * np.pi * 180 * tt) * (1 + np.sin(2 * np.pi * 3 * tt)) +
                 0.02 * rng.standard_normal(n)).astype(np.float32)
        feats = fe(audio, sampling_rate=16000, return_tensors="pt", return_attention_mask=True)
        x = feats["input_features"]
        mask = feats["attention_mask"]
        t_valid = int(mask.sum())
        t_pad = (t_valid + 99) // 100 * 100
        with torch.no_grad():
            a = model.model.get_audio_features(x, mask, return_dict=True)
        out[f"{tag}__audio"] = audio
        out[f"{tag}__mel"] = x[0, :, :t_pad].numpy().astype(np.float32)
        out[f"{tag}__t_valid"] = np.array(t_valid)
        out[f"{tag}__enc"] = a.last_hidden_state.numpy().astype(np.float32)
        out[f"{tag}__proj"] = a.pooler_output.numpy().astype(np.float32)
    # decoder: prompt with audio placeholders spliced from clip b, full-sequence logits
    n_audio = out["b__proj"].shape[0]
    ids = [3990, 5, 6, 3991, 7] + [4000] * n_audio + [3992, 3991, 8, 3990, 9]
    ids_t = torch.tensor([ids])
    with torch.no_grad():
        emb = model.model.language_model.embed_tokens(ids_t)
        pos = (ids_t == 4000)[0]
        emb[0, pos] = torch.from_numpy(out["b__proj"])
        o = model.model.language_model(inputs_embeds=emb)
        logits = model.lm_head(o.last_hidden_state)[0]
    out["dec__ids"] = np.array(ids, np.int32)
    out["dec__logits"] = logits.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "hf_tiny.npz"), **out)
    print("hf_tiny.npz", {k: v.shape for k, v in out.items()})


# ---------------------------------------------------------------------------------------------- HF at 0.6B dims
REAL_SEED = 7   # tests/test_model_real_gpu.py's synthetic-weight seed


def make_hf_06b(arch="qwen3-asr-0.6b", fname="hf_06b.npz"):
    """the oracle pinned at the real qwen3-asr-0.6b dimensions (18 encoder layers, d 896, 14 heads; 28
    decoder layers, GQA 16/8, head 128, the 151,936-row tied vocabulary).  transformers' qwen3_asr on the oracle's
    seeded synthetic weights (Q8_0 dequantised), 10 s of speech-like audio: the log-mel, the encoder / projector rows
    (a row subset + float64 sums) and the decoder logits of the chat prompt's last 8 rows, stored compactly (top-64
    values and indices per row + float64 checksums).  tests/test_oracle_cpu.py checks the oracle (float mode) against
    it.  (make_hf_17b: the same at qwen3-asr-1.7b — the benchmarked model — round 6.)"""
    import torch
    from transformers.models.qwen3_asr.feature_extraction_qwen3_asr import Qwen3ASRFeatureExtractor

    import oracle
    from bench import speech_like

    c = oracle.arch_config(arch)
    sp = oracle.QWEN_SPECIAL
    model = hf_model(c, oracle.Model(c, seed=REAL_SEED).export(), sp["tok_audio_pad"])
    audio = speech_like(np.random.default_rng(505), 160000)
    fe = Qwen3ASRFeatureExtractor()
    feats = fe(audio, sampling_rate=16000, return_tensors="pt", return_attention_mask=True)
    x, mask = feats["input_features"], feats["attention_mask"]
    t_valid = int(mask.sum())
    t_pad = (t_valid + 99) // 100 * 100
    with torch.no_grad():
        a = model.model.get_audio_features(x, mask, return_dict=True)
    enc = a.last_hidden_state.numpy().astype(np.float32)
    proj = a.pooler_output.numpy().astype(np.float32)
    rows = np.array([0, 1, 12, 13, 51, 103, 104, 117, enc.shape[0] - 1], np.int32)
    ids = oracle.chat_prompt(proj.shape[0])
    ids_t = torch.tensor([ids])
    with torch.no_grad():
        emb = model.model.language_model.embed_tokens(ids_t)
        emb[0, (ids_t == sp["tok_audio_pad"])[0]] = torch.from_numpy(proj)
        h = model.model.language_model(inputs_embeds=emb).last_hidden_state
        logits = model.lm_head(h[:, -8:])[0].numpy().astype(np.float32)
    top = np.argsort(-logits, axis=1, kind="stable")[:, :64]
    out = {"audio": audio, "mel": x[0, :, :t_pad].numpy().astype(np.float32), "t_valid": np.array(t_valid),
           "enc_rows": rows, "enc_sel": enc[rows], "proj_sel": proj[rows],
           "enc_sum": enc.astype(np.float64).sum(1), "proj_sum": proj.astype(np.float64).sum(1),
           "ids": np.array(ids, np.int32), "logit_top_idx": top.astype(np.int32),
           "logit_top_val": np.take_along_axis(logits, top, 1),
           "logit_sum": logits.astype(np.float64).sum(1), "logit_abs_sum": np.abs(logits.astype(np.float64)).sum(1)}
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(fname, {k: v.shape for k, v in out.items()})


def make_hf_17b():
    """the oracle pinned at the real qwen3-asr-1.7b dimensions (24 encoder layers of d 1,024 / 16 heads; 28 decoder
    layers of d 2,048, GQA 16/8, FFN 6,144, the tied 151,936-row vocabulary): make_hf_06b's fixture for the model C4
    and C5 are quoted on"""
    make_hf_06b("qwen3-asr-1.7b", "hf_17b.npz")


# ---------------------------------------------------------------------------------------------- BPE encode
BPE_CASES = ["Kubernetes", "张三", "ROCm 7.2", "light-whisper", "I'm here", "don't STOP", "They'LL go", "hello world",
             "  leading spaces", "trailing spaces   ", "tab\tseparated", "line\nbreak", "crlf\r\nline",
             "multi\n\n\nblank", "   ", "\n", "", "a", "1234567", "3.14159", "v2.0-rc1", "x86_64", "C++17",
             "email@example.com", "https://example.com/a?b=c", "深度学习", "语音识别模型", "東京タワー", "カタカナ",
             "ひらがな", "한국어 음성", "Привет мир", "Ελληνικά", "mixed中文English混合", "数字123和letters",
             "emoji 😀 test", "(括号)", "「引用」", "full，width。", "€100", "naïve café", "Straße", "ÀÉÎÕÜ",
             "hot-word, another; third", "Qwen3-ASR", "MI355X", "GPT-4o", "O'Brien", "rock'n'roll", "   x   ",
             "\u3000全角空格", "a\u00a0b", "end.\r\n", "...!!!???", "#hashtag @mention", "1,000,000",
             "pi=3.1415926535", "ＡＢＣ１２３", "日本語とEnglishの混在", "word" * 8]


def make_bpe():
    """byte-level BPE encoding of hot-word context (Qwen2 / Qwen3 tokenizer semantics: NFC, the
    Qwen2 pre-tokenizer regex, GPT-2 byte↔unicode map, BPE merges by rank).  A synthetic vocabulary + merge list is
    trained here (tokenizers BpeTrainer on a seeded multilingual corpus — no download) and the expected ids of
    BPE_CASES come from transformers.Qwen2Tokenizer built on it (tests/test_host_cpu.py pins the engine's encoder)."""
    from tokenizers import Regex, Tokenizer, models, pre_tokenizers, trainers
    from transformers import Qwen2Tokenizer
    from transformers.models.qwen2.tokenization_qwen2 import PRETOKENIZE_REGEX

    rng = np.random.default_rng(17)
    words = ("the quick brown fox jumps over lazy dog speech recognition model audio stream token hot word "
             "kubernetes cluster deploy gpu kernel memory bandwidth latency throughput english chinese japanese "
             "don't I'm you're we've they'll she'd it's hello world light whisper").split()
    han = [chr(c) for c in range(0x4E00, 0x4E00 + 400)] + list("张三深度学习语音识别模型中文混合数字和括号引用全角空格東京")
    kana = [chr(c) for c in range(0x3041, 0x3097)] + [chr(c) for c in range(0x30A1, 0x30FB)]
    lines = []
    for _ in range(4000):
        k = rng.integers(0, 5)
        if k == 0:
            lines.append(" ".join(rng.choice(words, rng.integers(3, 12))))
        elif k == 1:
            lines.append("".join(rng.choice(han, rng.integers(2, 20))))
        elif k == 2:
            lines.append("".join(rng.choice(kana, rng.integers(2, 12))) + "。")
        elif k == 3:
            lines.append(f"{rng.integers(0, 100000)} items, v{rng.integers(0, 9)}.{rng.integers(0, 9)} ok!")
        else:
            lines.append(" ".join(rng.choice(words, 3)) + " " + "".join(rng.choice(han, 4)) + "\n\n")
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.Sequence([pre_tokenizers.Split(Regex(PRETOKENIZE_REGEX), behavior="isolated"),
                                                pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tk.train_from_iterator(lines, trainers.BpeTrainer(vocab_size=1500, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                                      show_progress=False))
    model = json.loads(tk.to_str())["model"]
    vocab = model["vocab"]
    merges = [m if isinstance(m, str) else " ".join(m) for m in model["merges"]]
    vocab = {k: v for k, v in sorted(vocab.items(), key=lambda kv: kv[1])}
    ref = Qwen2Tokenizer(vocab=dict(vocab), merges=[tuple(m.split(" ")) for m in merges])
    cases = [{"text": t, "ids": ref.encode(t, add_special_tokens=False)} for t in BPE_CASES]
    bdir = os.path.join(HERE, "bpe")
    os.makedirs(bdir, exist_ok=True)
    json.dump(vocab, open(os.path.join(bdir, "vocab.json"), "w"), ensure_ascii=False)
    open(os.path.join(bdir, "merges.txt"), "w").write("#version: 0.2\n" + "\n".join(merges) + "\n")
    json.dump(cases, open(os.path.join(bdir, "cases.json"), "w"), ensure_ascii=False, indent=0)
    print("bpe:", len(vocab), "pieces,", len(merges), "merges,", len(cases), "cases")


# ---------------------------------------------------------------------------------------------- transcript parse
def make_parse():
    from transformers.models.qwen3_asr.processing_qwen3_asr import _parse_single_output

    cases = ["language English<asr_text>Hello world.", "language None<asr_text>", "LANGUAGE NONE<asr_text> tail ",
             "language Chinese<asr_text>你好，世界。", "\n\n  language Japanese\nsecond line<asr_text> こんにちは ",
             "no tag at all  ", "Chinese<asr_text>text", "language <asr_text>abc", "language  <asr_text>x",
             "system\nassistant\nlanguage English<asr_text>after assistant", "", "   \n\t ", "<asr_text>only text",
             "language German<asr_text>a<asr_text>b", "Language French\r\nfoo<asr_text> bar",
             "language English<asr_text>" + "a" * 25 + "b", "language English<asr_text>" + "哈" * 21 + "结束",
             "x" * 20 + "y", "language English<asr_text>" + "ab" * 25 + "c",
             "language English<asr_text>pre " + "la " * 30 + "post",
             "language Chinese<asr_text>" + "我们" * 20 + "然后" + "好" * 30,
             "　language Korean　<asr_text>　텍스트　", "language English x<asr_text>y"]
    rng = np.random.default_rng(3)
    alpha = ["a", "b", " ", "\n", "language ", "<asr_text>", "None", "你", "assistant\n", "ab", "ABC"]
    for _ in range(150):
        k = int(rng.integers(1, 12))
        parts = [alpha[int(i)] for i in rng.integers(0, len(alpha), size=k)]
        reps = int(rng.integers(0, 3))
        if reps:
            parts.append(alpha[int(rng.integers(0, len(alpha)))] * int(rng.integers(15, 45)))
        cases.append("".join(parts))
    out = []
    for c in cases:
        r = _parse_single_output(c)
        out.append({"raw": c, "language": r["language"] or "", "text": r["transcription"]})
    json.dump(out, open(os.path.join(HERE, "parse.json"), "w"), ensure_ascii=False)
    print("parse.json", len(out))


# ---------------------------------------------------------------------------------------------- path-mode WAV
def _wav_bytes(frames: np.ndarray, rate: int, fmt: int, bits: int, extensible=False) -> bytes:
    """RIFF/WAVE: frames [n][ch] already in the sample type's integer/float domain"""
    import struct

    ch = frames.shape[1]
    if bits == 24:
        v = frames.astype("<i4").reshape(-1)
        data = np.stack([(v & 0xFF), (v >> 8) & 0xFF, (v >> 16) & 0xFF], 1).astype(np.uint8).tobytes()
    else:
        dt = {8: np.uint8, 16: "<i2", 32: "<f4" if fmt == 3 else "<i4", 64: "<f8"}[bits]
        data = frames.astype(dt).tobytes()
    ba = ch * bits // 8
    if extensible:
        sub = struct.pack("<HII", bits, (1 << ch) - 1, fmt) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        fmt_chunk = struct.pack("<HHIIHHH", 0xFFFE, ch, rate, rate * ba, ba, bits, 22) + sub
    else:
        fmt_chunk = struct.pack("<HHIIHH", fmt, ch, rate, rate * ba, ba, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt_chunk)) + fmt_chunk
    body += b"LIST" + struct.pack("<I", 4) + b"INFO"   # an unrelated chunk before the data
    body += b"data" + struct.pack("<I", len(data)) + data + (b"\x00" if len(data) % 2 else b"")
    return b"RIFF" + struct.pack("<I", len(body)) + body


def make_wav():
    rng = np.random.default_rng(11)
    wdir = os.path.join(HERE, "wav")
    os.makedirs(wdir, exist_ok=True)
    specs = [  # name, rate, channels, fmt, bits, seconds, extensible
        ("pcm16_stereo_44k1", 44100, 2, 1, 16, 0.6, False),
        ("pcm24_mono_48k", 48000, 1, 1, 24, 0.55, False),
        ("float32_mono_16k", 16000, 1, 3, 32, 0.7, False),
        ("pcm8_mono_8k", 8000, 1, 1, 8, 0.8, False),
        ("pcm32_stereo_22k05", 22050, 2, 1, 32, 0.6, False),
        ("pcm16_ext_3ch_16k", 16000, 3, 1, 16, 0.3, True),
        # float64 and G.711 (fmt 7 µ-law, fmt 6 A-law) — libsndfile decodes them too
        ("float64_mono_16k", 16000, 1, 3, 64, 0.5, False),
        ("ulaw_mono_8k", 8000, 1, 7, 8, 0.5, False),
        ("alaw_stereo_8k", 8000, 2, 6, 8, 0.4, False),
    ]
    for name, rate, ch, fmt, bits, secs, ext in specs:
        n = int(rate * secs)
        x = (0.4 * np.sin(2 * np.pi * 220 * np.arange(n)[:, None] / rate + np.arange(ch)) +
             0.05 * rng.standard_normal((n, ch)))
        if fmt == 3:
            fr = x.astype(np.float32 if bits == 32 else np.float64)
        elif fmt in (6, 7):   # 8-bit G.711 codes of the companded signal (every byte is a valid code)
            fr = np.clip(np.round(127.5 + 127.5 * np.sign(x) * np.log1p(255 * np.abs(x)) / np.log(256)), 0, 255)
        elif bits == 8:
            fr = np.clip(np.round(x * 127 + 128), 0, 255)
        else:
            fr = np.clip(np.round(x * (2 ** (bits - 1) - 1)), -(2 ** (bits - 1)), 2 ** (bits - 1) - 1)
        open(os.path.join(wdir, name + ".wav"), "wb").write(_wav_bytes(fr, rate, fmt, bits, ext))
    # a 4-bit IMA ADPCM header: refused (an error reply), never a division by zero
    import struct

    adpcm = struct.pack("<HHIIHHHH", 0x11, 1, 16000, 8000, 256, 4, 2, 505)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(adpcm)) + adpcm + b"data" + struct.pack("<I", 512) + bytes(512)
    open(os.path.join(wdir, "adpcm4_mono_16k.wav"), "wb").write(b"RIFF" + struct.pack("<I", len(body)) + body)
    open(os.path.join(wdir, "not_a_wav.wav"), "wb").write(b"OggS" + bytes(60))
    code = r"""
import json, os, struct, sys, types
import numpy as np
sys.path.insert(0, %r)
sf = types.ModuleType("soundfile")
def read(path, dtype="float32", always_2d=True):
    d = open(path, "rb").read()
    if d[:4] != b"RIFF" or d[8:12] != b"WAVE":
        raise RuntimeError("Error opening %%r: Format not recognised." %% path)
    pos, fmt = 12, None
    while pos + 8 <= len(d):
        cid, sz = d[pos:pos + 4], struct.unpack("<I", d[pos + 4:pos + 8])[0]
        b = pos + 8
        if cid == b"fmt ":
            fmt, ch, rate = struct.unpack("<HHI", d[b:b + 8]); bits = struct.unpack("<H", d[b + 14:b + 16])[0]
            if fmt == 0xFFFE: fmt = struct.unpack("<H", d[b + 24:b + 26])[0]
        elif cid == b"data":
            raw = d[b:b + sz]
            if fmt == 3 and bits == 64: x = np.frombuffer(raw, "<f8").astype(np.float32)
            elif fmt == 3: x = np.frombuffer(raw, "<f4").astype(np.float32)
            elif fmt == 7:   # libsndfile ulaw_decode table (Sun g711.c ulaw2linear), normalised by 1/0x8000
                u = ~np.frombuffer(raw, np.uint8).astype(np.int32) & 0xFF
                t = (((u & 0x0F) << 3) + 0x84) << ((u & 0x70) >> 4)
                x = np.where(u & 0x80, 0x84 - t, t - 0x84).astype(np.float32) * np.float32(1.0 / 32768)
            elif fmt == 6:   # libsndfile alaw_decode table (Sun g711.c alaw2linear)
                a = np.frombuffer(raw, np.uint8).astype(np.int32) ^ 0x55
                t, seg = (a & 0x0F) << 4, (a & 0x70) >> 4
                t = np.where(seg == 0, t + 8, (t + 0x108) << np.maximum(seg - 1, 0))
                x = np.where(a & 0x80, t, -t).astype(np.float32) * np.float32(1.0 / 32768)
            elif bits == 16: x = np.frombuffer(raw, "<i2").astype(np.float32) / np.float32(2 ** 15)
            elif bits == 32: x = (np.frombuffer(raw, "<i4").astype(np.float32) / np.float32(2 ** 31)).astype(np.float32)
            elif bits == 8: x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128) / np.float32(128)
            elif bits == 24:
                u = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
                v = ((u[:, 0] << 8) | (u[:, 1] << 16) | (u[:, 2] << 24)) >> 8
                x = v.astype(np.float32) / np.float32(2 ** 23)
            else: raise RuntimeError("unsupported")
            return x.reshape(-1, ch).astype(np.float32), rate
        pos = b + sz + (sz & 1)
    raise RuntimeError("no data")
sf.read = read
sys.modules["soundfile"] = sf
import qwen3_asr_server
srv = qwen3_asr_server.Qwen3ASRServer.__new__(qwen3_asr_server.Qwen3ASRServer)
out = {}
wdir = %r
for f in sorted(os.listdir(wdir)):
    if f.startswith(("adpcm", "not_a")): continue
    audio, dur, mode = srv._load_audio(os.path.join(wdir, f), None, None, None)
    out[f] = {"audio": np.asarray(audio, np.float32).astype(float).tolist(), "duration": dur, "mode": mode}
print(json.dumps(out))
""" % (REF_RES, wdir)
    env = dict(os.environ, LIGHT_WHISPER_DATA_DIR=tempfile.mkdtemp())
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, check=True)
    data = json.loads(res.stdout.strip().splitlines()[-1])
    arrs = {}
    for k, v in data.items():
        arrs[k + "__audio"] = np.asarray(v["audio"], np.float32)
        arrs[k + "__duration"] = np.float64(v["duration"])
    np.savez_compressed(os.path.join(HERE, "wav_expected.npz"), **arrs)
    print("wav_expected.npz", {k: len(v["audio"]) for k, v in data.items()})


if __name__ == "__main__":
    which = sys.argv[1:] or ["vad_post", "audio_io", "protocol", "dfsmn", "hf_tiny", "hf_06b", "bpe", "parse", "wav"]
    for w in which:
        globals()[f"make_{w}"]()
