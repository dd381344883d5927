"""ctypes wrapper around oracle/liboracle.so — the CPU restatement of the hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker (or the reported CPU baseline), never as the product path.
See qasr_oracle.c for what each function restates (reference file:line citations live there).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

QK = 32
QBYTES = 34


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "qasr_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        L = C.CDLL(build())
        P = C.c_void_p
        i64 = C.c_int64
        L.orc_set_mode.argtypes = [C.c_int, C.c_int]
        L.orc_num_threads.restype = C.c_int
        L.orc_set_num_threads.argtypes = [C.c_int]
        L.orc_quantize_row_q8.argtypes = [P, i64, P]
        L.orc_dequantize_row_q8.argtypes = [P, i64, P]
        L.orc_q8_block_dots.argtypes = [P, P, i64, P]
        L.orc_linear_q8.argtypes = [P, i64, i64, P, i64, P, P]
        L.orc_name_id.argtypes = [C.c_char_p]
        L.orc_name_id.restype = C.c_uint64
        L.orc_synth_q8.argtypes = [C.c_uint64, C.c_char_p, i64, i64, C.c_float, P]
        L.orc_synth_f32.argtypes = [C.c_uint64, C.c_char_p, i64, C.c_float, C.c_float, P]
        L.orc_synth_f16.argtypes = [C.c_uint64, C.c_char_p, i64, C.c_float, P]
        L.orc_kaldi_mel_banks.argtypes = [P]
        L.orc_fbank.argtypes = [P, i64, P]
        L.orc_fbank.restype = i64
        L.orc_dfsmn.argtypes = [P, i64, P, P]
        L.orc_vad_segments.argtypes = [P, i64, i64, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, P, i64]
        L.orc_vad_segments.restype = i64
        L.orc_mel_filters.argtypes = [C.c_int, P]
        L.orc_mel_dims.argtypes = [i64, P, P]
        L.orc_mel.argtypes = [P, i64, C.c_int, P]
        L.orc_mel.restype = i64
        L.orc_model_new.argtypes = [P, P]
        L.orc_model_new.restype = P
        L.orc_model_free.argtypes = [P]
        L.orc_model_set.argtypes = [P, C.c_char_p, P]
        L.orc_model_set.restype = C.c_int
        L.orc_model_synth.argtypes = [P, C.c_uint64]
        L.orc_model_get.argtypes = [P, C.c_char_p]
        L.orc_model_get.restype = P
        L.orc_audio_tokens.argtypes = [C.c_int]
        L.orc_audio_tokens.restype = C.c_int
        L.orc_encode.argtypes = [P, P, C.c_int, C.c_int, P, P]
        L.orc_encode.restype = C.c_int
        L.orc_kv_new.argtypes = [P, C.c_int]
        L.orc_kv_new.restype = P
        L.orc_kv_free.argtypes = [P]
        L.orc_kv_reset.argtypes = [P]
        L.orc_embed.argtypes = [P, P, C.c_int, P]
        L.orc_forward.argtypes = [P, P, C.c_int, P, C.c_int]
        L.orc_forward.restype = C.c_int
        L.orc_generate.argtypes = [P, P, C.c_int, C.c_int, P, C.c_int, P, C.c_int, C.c_int, C.c_int, P, P]
        L.orc_generate.restype = C.c_int
        L.orc_f32_to_f16_array.argtypes = [P, P, i64]
        L.orc_f16_to_f32_array.argtypes = [P, P, i64]
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def set_mode(engine: bool = True):
    lib().orc_set_mode(1 if engine else 0, 1 if engine else 0)


def set_threads(n: int):
    lib().orc_set_num_threads(int(n))


def num_threads() -> int:
    return lib().orc_num_threads()


# ------------------------------------------------------------------------------------------ Q8_0
def quantize_q8(x: np.ndarray) -> np.ndarray:
    """Q8_0 blocks of a [N][K] f32 matrix → uint8 [N][K/32*34] (ggml layout)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, k = x.shape
    out = np.empty((n, k // QK * QBYTES), dtype=np.uint8)
    for r in range(n):
        lib().orc_quantize_row_q8(_p(x[r]), k, _p(out[r]))
    return out


def dequantize_q8(blocks: np.ndarray, k: int) -> np.ndarray:
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, k // QK * QBYTES)
    out = np.empty((blocks.shape[0], k), dtype=np.float32)
    for r in range(blocks.shape[0]):
        lib().orc_dequantize_row_q8(_p(blocks[r]), k, _p(out[r]))
    return out


def linear_q8(x: np.ndarray, w_blocks: np.ndarray, n: int, bias: np.ndarray | None = None) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    m, k = x.shape
    y = np.empty((m, n), dtype=np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    lib().orc_linear_q8(_p(x), m, k, _p(np.ascontiguousarray(w_blocks)), n, None if b is None else _p(b), _p(y))
    return y


def synth_q8(seed: int, name: str, n: int, k: int, sigma: float) -> np.ndarray:
    out = np.empty((n, k // QK * QBYTES), dtype=np.uint8)
    lib().orc_synth_q8(seed, name.encode(), n, k, sigma, _p(out))
    return out


def f16_bits(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty(x.shape, dtype=np.uint16)
    lib().orc_f32_to_f16_array(_p(x), _p(y), x.size)
    return y


# ------------------------------------------------------------------------------------------ VAD
def fbank(pcm_int16_scale: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(pcm_int16_scale, dtype=np.float32)
    n = x.size
    t = 1 + (n - 400) // 160 if n >= 400 else 0
    out = np.empty((max(t, 0), 80), dtype=np.float32)
    got = lib().orc_fbank(_p(x), n, _p(out))
    assert got == t
    return out


def kaldi_mel_banks() -> np.ndarray:
    out = np.empty((80, 256), dtype=np.float32)
    lib().orc_kaldi_mel_banks(_p(out))
    return out


class VadWeights(C.Structure):
    _fields_ = (
        [("mean", C.c_void_p), ("istd", C.c_void_p), ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p),
         ("b2", C.c_void_p)]
        + [("lb", C.c_void_p * 8), ("la", C.c_void_p * 8), ("wa", C.c_void_p * 7), ("ba", C.c_void_p * 7),
           ("wb", C.c_void_p * 7)]
        + [("wd", C.c_void_p), ("bd", C.c_void_p), ("wo", C.c_void_p), ("bo", C.c_float)]
    )


def vad_probabilities(feats: np.ndarray, w: dict) -> np.ndarray:
    """DFSMN over raw log-fbank feats [T][80]; w = dict from assets/fireredvad (see qasr.vad_weights)."""
    feats = np.ascontiguousarray(feats, dtype=np.float32)
    t = feats.shape[0]
    keep = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in w.items()}
    s = VadWeights()
    s.mean, s.istd = _p(keep["mean"]).value, _p(keep["istd"]).value
    s.w1, s.b1, s.w2, s.b2 = (_p(keep[k]).value for k in ("w1", "b1", "w2", "b2"))
    for i in range(8):
        s.lb[i] = _p(keep[f"lb{i}"]).value
        s.la[i] = _p(keep[f"la{i}"]).value
    for i in range(7):
        s.wa[i] = _p(keep[f"wa{i}"]).value
        s.ba[i] = _p(keep[f"ba{i}"]).value
        s.wb[i] = _p(keep[f"wb{i}"]).value
    s.wd, s.bd, s.wo = _p(keep["wd"]).value, _p(keep["bd"]).value, _p(keep["wo"]).value
    s.bo = float(keep["bo"].reshape(-1)[0])
    out = np.empty(t, dtype=np.float32)
    if t:
        lib().orc_dfsmn(_p(feats), t, C.byref(s), _p(out))
    return out


def vad_segments(probs: np.ndarray, audio_len: int, threshold=0.5, smooth_window=5, min_speech_ms=150,
                 min_silence_ms=300, pad_ms=120) -> list[dict]:
    p = np.ascontiguousarray(probs, dtype=np.float32).reshape(-1)
    cap = max(1, p.size)
    out = np.empty(2 * cap, dtype=np.int64)
    n = lib().orc_vad_segments(_p(p), p.size, int(audio_len), float(threshold), int(smooth_window),
                               int(min_speech_ms), int(min_silence_ms), int(pad_ms), _p(out), cap)
    return [{"start": int(out[2 * i]), "end": int(out[2 * i + 1])} for i in range(n)]


# ------------------------------------------------------------------------------------------ mel
def mel_filters(n_mels=128) -> np.ndarray:
    out = np.empty((201, n_mels), dtype=np.float32)
    lib().orc_mel_filters(n_mels, _p(out))
    return out


def mel_dims(n: int):
    tv = np.zeros(1, np.int64)
    tp = np.zeros(1, np.int64)
    lib().orc_mel_dims(n, _p(tv), _p(tp))
    return int(tv[0]), int(tp[0])


def mel(pcm: np.ndarray, n_mels=128):
    x = np.ascontiguousarray(pcm, dtype=np.float32)
    tv, tp = mel_dims(x.size)
    out = np.empty((n_mels, tp), dtype=np.float32)
    got = lib().orc_mel(_p(x), x.size, n_mels, _p(out))
    assert got == tv
    return out, tv


# ------------------------------------------------------------------------------------------ model
CFG_INT_KEYS = ["n_mels", "conv_ch", "enc_d", "enc_layers", "enc_heads", "enc_ffn", "n_window", "n_window_infer",
                "proj_out", "txt_h", "txt_layers", "txt_heads", "txt_kv_heads", "head_dim", "txt_ffn", "vocab"]
CFG_FLOAT_KEYS = ["rope_theta", "rms_eps", "ln_eps"]

# Qwen2-tokenizer special ids the pinned checkpoints use (chat prompt, EOS; the engine's default_hparams)
QWEN_SPECIAL = dict(tok_im_start=151644, tok_im_end=151645, tok_system=8948, tok_user=872, tok_assistant=77091,
                    tok_newline=198, tok_audio_start=151669, tok_audio_end=151670, tok_audio_pad=151676,
                    tok_eos0=151645, tok_eos1=151643, tok_asr_text=151704)


def arch_config(arch: str) -> dict:
    """Hyper-parameters of the two pinned checkpoints (hf_cache_utils.py:11-26) — the same
    values as the engine's default_hparams (model.cpp)."""
    cfg = dict(n_mels=128, conv_ch=480, n_window=50, n_window_infer=800, txt_layers=28, txt_heads=16, txt_kv_heads=8,
               head_dim=128, vocab=151936, rope_theta=1e6, rms_eps=1e-6, ln_eps=1e-5)
    if arch == "qwen3-asr-0.6b":
        cfg.update(enc_d=896, enc_layers=18, enc_heads=14, enc_ffn=3584, txt_h=1024, txt_ffn=3072)
    elif arch == "qwen3-asr-1.7b":
        cfg.update(enc_d=1024, enc_layers=24, enc_heads=16, enc_ffn=4096, txt_h=2048, txt_ffn=6144)
    else:
        raise ValueError(arch)
    cfg["proj_out"] = cfg["txt_h"]
    return cfg


def chat_prompt(n_audio: int, sp: dict = QWEN_SPECIAL, context=()) -> list:
    """The engine's chat prompt (processing_qwen3_asr.py:534-553) with n_audio audio placeholders."""
    return ([sp["tok_im_start"], sp["tok_system"], sp["tok_newline"]] + list(context)
            + [sp["tok_im_end"], sp["tok_newline"], sp["tok_im_start"], sp["tok_user"], sp["tok_newline"],
               sp["tok_audio_start"]] + [sp["tok_audio_pad"]] * n_audio
            + [sp["tok_audio_end"], sp["tok_im_end"], sp["tok_newline"], sp["tok_im_start"], sp["tok_assistant"],
               sp["tok_newline"]])


class Model:
    """Oracle model: either bound to numpy tensors (GGUF-style names) or synthetic (seeded)."""

    def __init__(self, cfg: dict, tensors: dict | None = None, seed: int | None = None):
        self.cfg = dict(cfg)
        ints = np.array([cfg[k] for k in CFG_INT_KEYS], dtype=np.int32)
        floats = np.array([cfg[k] for k in CFG_FLOAT_KEYS], dtype=np.float32)
        self.h = lib().orc_model_new(_p(ints), _p(floats))
        self._keep = []
        if tensors is not None:
            for name, arr in tensors.items():
                a = np.ascontiguousarray(arr)
                self._keep.append(a)
                rc = lib().orc_model_set(self.h, name.encode(), _p(a))
                if rc != 0:
                    raise KeyError(name)
        if seed is not None:
            lib().orc_model_synth(self.h, int(seed))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_model_free(self.h)
            self.h = None

    def tensor_specs(self) -> dict:
        """name → (kind, shape) of every tensor in this engine's GGUF convention (kind: q8 / f32 / f16)."""
        c = self.cfg
        C_, d, H = c["conv_ch"], c["enc_d"], c["txt_h"]
        F3 = (((c["n_mels"] + 1) // 2 + 1) // 2 + 1) // 2
        QD, KD = c["txt_heads"] * c["head_dim"], c["txt_kv_heads"] * c["head_dim"]
        t = {"a.conv1.weight": ("f16", (C_, 1, 3, 3)), "a.conv2.weight": ("f16", (C_, C_, 3, 3)),
             "a.conv3.weight": ("f16", (C_, C_, 3, 3)), "a.conv_out.weight": ("q8", (d, C_ * F3)),
             "a.ln_post.weight": ("f32", (d,)), "a.ln_post.bias": ("f32", (d,)), "a.proj1.weight": ("q8", (d, d)),
             "a.proj1.bias": ("f32", (d,)), "a.proj2.weight": ("q8", (c["proj_out"], d)),
             "a.proj2.bias": ("f32", (c["proj_out"],)), "token_embd.weight": ("q8", (c["vocab"], H)),
             "output_norm.weight": ("f32", (H,))}
        for i in (1, 2, 3):
            t[f"a.conv{i}.bias"] = ("f32", (C_,))
        for l in range(c["enc_layers"]):
            for n_ in ("ln1", "ln2"):
                t[f"a.blk.{l}.{n_}.weight"] = ("f32", (d,))
                t[f"a.blk.{l}.{n_}.bias"] = ("f32", (d,))
            for n_, nn, kk in (("attn_q", d, d), ("attn_k", d, d), ("attn_v", d, d), ("attn_out", d, d),
                               ("ffn_up", c["enc_ffn"], d), ("ffn_down", d, c["enc_ffn"])):
                t[f"a.blk.{l}.{n_}.weight"] = ("q8", (nn, kk))
                t[f"a.blk.{l}.{n_}.bias"] = ("f32", (nn,))
        for l in range(c["txt_layers"]):
            for n_ in ("attn_norm", "ffn_norm"):
                t[f"blk.{l}.{n_}.weight"] = ("f32", (H,))
            for n_ in ("attn_q_norm", "attn_k_norm"):
                t[f"blk.{l}.{n_}.weight"] = ("f32", (c["head_dim"],))
            for n_, nn, kk in (("attn_q", QD, H), ("attn_k", KD, H), ("attn_v", KD, H), ("attn_output", H, QD),
                               ("ffn_gate", c["txt_ffn"], H), ("ffn_up", c["txt_ffn"], H),
                               ("ffn_down", H, c["txt_ffn"])):
                t[f"blk.{l}.{n_}.weight"] = ("q8", (nn, kk))
        return t

    def export(self) -> dict:
        """copy every bound tensor out (Q8_0 as GGUF blocks [N][K/32*34] uint8, f16 as uint16 bits)."""
        out = {}
        for name, (kind, shape) in self.tensor_specs().items():
            p = lib().orc_model_get(self.h, name.encode())
            if not p:
                continue
            if kind == "q8":
                nbytes = shape[0] * shape[1] // QK * QBYTES
                a = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p)).copy().reshape(shape[0], -1)
            elif kind == "f32":
                a = np.ctypeslib.as_array((C.c_float * int(np.prod(shape))).from_address(p)).copy().reshape(shape)
            else:
                a = np.ctypeslib.as_array((C.c_uint16 * int(np.prod(shape))).from_address(p)).copy().reshape(shape)
            out[name] = a
        return out

    def export_one(self, name: str) -> np.ndarray:
        """one bound tensor in GGUF storage form, flattened to bytes (as Model.export_tensor returns it)"""
        kind, shape = self.tensor_specs()[name]
        p = lib().orc_model_get(self.h, name.encode())
        assert p, name
        n = shape[0] * shape[1] // QK * QBYTES if kind == "q8" else int(np.prod(shape)) * (4 if kind == "f32" else 2)
        return np.ctypeslib.as_array((C.c_uint8 * n).from_address(p)).copy()

    def audio_tokens(self, t_valid: int) -> int:
        return lib().orc_audio_tokens(int(t_valid))

    def encode(self, mel: np.ndarray, t_valid: int, want_enc=False):
        mel = np.ascontiguousarray(mel, dtype=np.float32)
        t_pad = mel.shape[1]
        n_tok = self.audio_tokens(t_valid)
        out = np.empty((n_tok, self.cfg["proj_out"]), dtype=np.float32)
        enc = np.empty((n_tok, self.cfg["enc_d"]), dtype=np.float32) if want_enc else None
        got = lib().orc_encode(self.h, _p(mel), t_pad, t_valid, _p(out), None if enc is None else _p(enc))
        assert got == n_tok
        return (out, enc) if want_enc else out


class KV:
    def __init__(self, model: Model, n_ctx: int):
        self.model = model
        self.h = lib().orc_kv_new(model.h, int(n_ctx))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_kv_free(self.h)
            self.h = None

    def reset(self):
        lib().orc_kv_reset(self.h)

    def embed(self, ids) -> np.ndarray:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        out = np.empty((ids.size, self.model.cfg["txt_h"]), dtype=np.float32)
        lib().orc_embed(self.model.h, _p(ids), ids.size, _p(out))
        return out

    def forward(self, x: np.ndarray, all_logits=False) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[0]
        v = self.model.cfg["vocab"]
        lg = np.empty((n if all_logits else 1, v), dtype=np.float32)
        rc = lib().orc_forward(self.h, _p(x), n, _p(lg), 1 if all_logits else 0)
        assert rc == 0
        return lg

    def generate(self, prompt, audio_pad: int, audio: np.ndarray, eos=(151645, 151643), max_new=64, force_len=0,
                 want_logits=False):
        prompt = np.ascontiguousarray(prompt, dtype=np.int32)
        audio = np.ascontiguousarray(audio, dtype=np.float32)
        eos = np.ascontiguousarray(eos, dtype=np.int32)
        limit = force_len if force_len > 0 else max_new
        out = np.empty(max(limit, 1), dtype=np.int32)
        lg = np.empty((max(limit, 1), self.model.cfg["vocab"]), dtype=np.float32) if want_logits else None
        n = lib().orc_generate(self.h, _p(prompt), prompt.size, int(audio_pad), _p(audio), audio.shape[0], _p(eos),
                               eos.size, int(max_new), int(force_len), _p(out), None if lg is None else _p(lg))
        assert n >= 0
        return (out[:n].copy(), lg[:n].copy()) if want_logits else out[:n].copy()


# ---------------------------------------------------------------------------------------------------- MXFP8 (C5)
# The fp8 precision mode has no counterpart in the reference ("tolerance parity only"); these
# restate the OCP Microscaling v1.0 formats it uses — e4m3 elements (bias 7, no infinities, max 448) and e8m0
# block exponents — with the engine's choices: E = the smallest exponent putting the block maximum ≤ 448,
# round-to-nearest-even elements.

def mx_block_exp(amax: np.ndarray) -> np.ndarray:
    amax = np.asarray(amax, np.float32)
    m, e = np.frexp(amax)
    E = np.where(m <= 0.875, e - 9, e - 8)
    return np.clip(np.where(amax > 0, E, -127), -127, 127).astype(np.int32)


def e4m3_rne(x: np.ndarray) -> np.ndarray:
    """float32 values with |x| ≤ 448 → e4m3 codes (uint8), round to nearest even"""
    x = np.asarray(x, np.float32)
    a = np.abs(x).astype(np.float64)
    sg = np.where(x < 0, 0x80, 0).astype(np.int64)
    sub = np.rint(a * 512.0).astype(np.int64)
    _, ex = np.frexp(a)
    e = ex.astype(np.int64) - 1
    m = np.rint(np.ldexp(a, (3 - e).astype(np.int32))).astype(np.int64)
    carry = m == 16
    e = e + carry
    m = np.where(carry, 8, m)
    normal = ((e + 7) << 3) | (m - 8)
    return (sg | np.where(a < 2.0 ** -6, sub, normal)).astype(np.uint8)


def e4m3_value(code: np.ndarray) -> np.ndarray:
    c = np.asarray(code, np.int64)
    s = np.where(c & 0x80, -1.0, 1.0)
    e = (c >> 3) & 15
    m = c & 7
    return s * np.where(e == 0, m * 2.0 ** -9, (1 + m / 8.0) * np.ldexp(1.0, (e - 7).astype(np.int32)))


def q8_to_mx(q: np.ndarray, d: np.ndarray):
    """Q8 blocks q [nblk, 32] int8, d [nblk] (f32 or f16 values) → (codes [nblk, 32] uint8, E [nblk] int32)"""
    q = np.asarray(q, np.int8).reshape(-1, 32)
    d = np.asarray(d, np.float32).reshape(-1)
    mq = np.abs(q.astype(np.int32)).max(axis=1).astype(np.float32)
    E = mx_block_exp(np.abs(d) * mq)
    with np.errstate(over="ignore"):
        sc = np.where(mq == 0, 0.0, np.ldexp(d, -E)).astype(np.float32)
    return e4m3_rne(q.astype(np.float32) * sc[:, None]), E


def mx_matrix(codes: np.ndarray, E: np.ndarray, rows: int, k: int) -> np.ndarray:
    """the real values an MXFP8 matrix stands for, float64 [rows][k]"""
    v = e4m3_value(codes).reshape(rows, k // 32, 32) * np.ldexp(1.0, E.reshape(rows, k // 32, 1))
    return v.reshape(rows, k)
