"""Drop-in for the `transcribe_cpp` Python API that the reference server binds, backed by libqasr (HIP).

Reference call sites (sypsyp97/light-whisper src-tauri/resources/qwen3_asr_server.py):
    model = transcribe_cpp.Model(model_path, backend=backend)          # :122
    session = model.session(kv_type="f16", n_ctx=32768)                 # :123
    result = session.run(audio_f32_16k, timestamps="none")             # :144, :321
    result.text, result.language                                        # :326-327
    session.close(); model.close()                                      # :100-112
Backends: "hip" and "auto" select the MI355X engine; "cuda", "vulkan" and "cpu" raise (the reference's
fallback loop then reports every backend's error, :117-133).  There is no CPU path.

Extensions used by the bench and the parity tests: Model.synthetic(), Session.run_batch(),
Session.forced_logits(), Session.mel(), Session.encode(), Session.prefill_logits().
"""
from __future__ import annotations

import ctypes as C
from types import SimpleNamespace

import numpy as np

from . import _lib
from ._lib import HParams, Result, RunOpts, check

__version__ = "0.1.3+mi355x"


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))


def _take_result(r: Result) -> SimpleNamespace:
    toks = [r.tokens[i] for i in range(r.n_tokens)]
    out = SimpleNamespace(
        text=(r.text or b"").decode("utf-8", "replace"),
        language=(r.language or b"").decode("utf-8", "replace") or None,
        raw=(r.raw or b"").decode("utf-8", "replace"),
        tokens=toks,
        n_audio_tokens=r.n_audio_tokens,
        n_prompt=r.n_prompt,
        truncated=bool(r.truncated),
        timings_ms={"mel": r.ms_mel, "encoder": r.ms_encoder, "prefill": r.ms_prefill, "decode": r.ms_decode},
    )
    _lib.load().qasr_result_free(C.byref(r))
    return out


class Model:
    def __init__(self, path: str, backend: str = "auto", _handle=None):
        lib = _lib.load()
        self._h = C.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            check(lib.qasr_model_open(path.encode(), backend.encode(), C.byref(self._h)))
        self.path = path
        self.backend = "hip"

    @classmethod
    def synthetic(cls, arch: str | None = "qwen3-asr-1.7b", seed: int = 0, hparams: dict | None = None):
        lib = _lib.load()
        h = C.c_void_p()
        hp = None
        if hparams is not None:
            hp = HParams()
            for k, v in hparams.items():
                setattr(hp, k, v)
        check(lib.qasr_model_open_synthetic(arch.encode() if arch else None, C.byref(hp) if hp is not None else None,
                                            int(seed), C.byref(h)))
        return cls(f"synthetic:{arch or 'custom'}:{seed}", _handle=h)

    @classmethod
    def shell(cls, arch: str | None = "qwen3-asr-1.7b", gguf_path: str | None = None, hparams: dict | None = None):
        """Receiving side of the one-time weight broadcast: the device layout of `arch` (or of the GGUF's metadata)
        allocated but not filled.  Fill `weight_blob()` (one collective from rank 0), then `weights_received()`."""
        lib = _lib.load()
        h = C.c_void_p()
        hp = None
        if hparams is not None:
            hp = HParams()
            for k, v in hparams.items():
                setattr(hp, k, v)
        check(lib.qasr_model_open_shell(gguf_path.encode() if gguf_path else None, arch.encode() if arch else None,
                                        C.byref(hp) if hp is not None else None, C.byref(h)))
        return cls(gguf_path or f"shell:{arch or 'custom'}", _handle=h)

    def weight_blob(self):
        """(device pointer, bytes) of the single allocation holding every weight and table."""
        p, n = C.c_void_p(), C.c_size_t()
        check(_lib.load().qasr_model_weight_blob(self._h, C.byref(p), C.byref(n)))
        return int(p.value or 0), int(n.value)

    def tensor_table(self) -> dict:
        """{name: (ggml type, rows, cols, conv_cin)} of every GGUF tensor of the model."""
        import json

        lib = _lib.load()
        need = C.c_size_t()
        check(lib.qasr_model_tensor_table(self._h, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        check(lib.qasr_model_tensor_table(self._h, buf, need.value, C.byref(need)))
        return {k: tuple(v) for k, v in json.loads(buf.value.decode()).items()}

    def set_precision(self, mode: str):
        """"q8" (the reference's arithmetic) or "mxfp8" (block-scaled fp8 GEMMs)"""
        check(_lib.load().qasr_model_set_precision(self._h, mode.encode()))

    def tokenize(self, text: str) -> list[int]:
        """UTF-8 text → token ids (greedy longest match; for the opt-in hot-word context)"""
        b = text.encode("utf-8")
        n = C.c_size_t()
        lib = _lib.load()
        check(lib.qasr_model_tokenize(self._h, b, len(b), None, 0, C.byref(n)))
        ids = np.empty(max(1, n.value), np.int32)
        check(lib.qasr_model_tokenize(self._h, b, len(b), ids.ctypes.data_as(C.c_void_p), ids.size, C.byref(n)))
        return ids[: n.value].tolist()

    def detokenize(self, ids) -> str:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.int32).reshape(-1))
        n = C.c_size_t()
        lib = _lib.load()
        p = a.ctypes.data_as(C.c_void_p) if a.size else None
        check(lib.qasr_model_detokenize(self._h, p, int(a.size), None, 0, C.byref(n)))
        buf = C.create_string_buffer(max(1, n.value))
        check(lib.qasr_model_detokenize(self._h, p, int(a.size), buf, n.value, C.byref(n)))
        return buf.raw[: n.value].decode("utf-8")

    def weights_received(self):
        check(_lib.load().qasr_model_weights_received(self._h))

    @property
    def hparams(self) -> dict:
        hp = HParams()
        check(_lib.load().qasr_model_hparams(self._h, C.byref(hp)))
        return hp.to_dict()

    def weight_bytes(self) -> int:
        return int(_lib.load().qasr_model_weight_bytes(self._h))

    def export_tensor(self, name: str, nbytes: int) -> np.ndarray:
        buf = np.empty(nbytes, np.uint8)
        written = C.c_size_t()
        check(_lib.load().qasr_model_export_tensor(self._h, name.encode(), buf.ctypes.data_as(C.c_void_p), nbytes,
                                                   C.byref(written)))
        return buf[: written.value]

    def session(self, kv_type: str = "f16", n_ctx: int = 32768) -> "Session":
        return Session(self, kv_type, n_ctx)

    def close(self):
        if self._h:
            _lib.load().qasr_model_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Session:
    def __init__(self, model: Model, kv_type: str = "f16", n_ctx: int = 32768):
        self.model = model
        self._h = C.c_void_p()
        check(_lib.load().qasr_session_open(model._h, kv_type.encode(), int(n_ctx), C.byref(self._h)))
        self.n_ctx = n_ctx

    def run(self, audio, timestamps: str = "none", max_new_tokens: int = 0, force_tokens_per_s: int = 0):
        if timestamps not in ("none", None):
            raise ValueError("only timestamps='none' is supported")
        a = _f32(audio)
        r = Result()
        opts = RunOpts(int(max_new_tokens), int(force_tokens_per_s), 0)
        check(_lib.load().qasr_session_run_opts(self._h, a.ctypes.data_as(C.c_void_p), a.size, C.byref(opts),
                                                C.byref(r)))
        return _take_result(r)

    def run_batch(self, audios, max_new_tokens: int = 0, force_tokens_per_s: int = 0):
        arrs = [_f32(a) for a in audios]
        n = len(arrs)
        ptrs = (C.c_void_p * n)(*[a.ctypes.data_as(C.c_void_p).value for a in arrs])
        lens = (C.c_size_t * n)(*[a.size for a in arrs])
        res = (Result * n)()
        opts = RunOpts(int(max_new_tokens), int(force_tokens_per_s), 0)
        check(_lib.load().qasr_run_batch(self._h, ptrs, lens, n, C.byref(opts), res))
        return [_take_result(res[i]) for i in range(n)]

    def run_batch_device(self, dev_ptr: int, offsets, lengths, max_new_tokens: int = 0, force_tokens_per_s: int = 0,
                         want_results: bool = True):
        n = len(lengths)
        off = (C.c_int64 * n)(*[int(x) for x in offsets])
        ln = (C.c_int64 * n)(*[int(x) for x in lengths])
        res = (Result * n)() if want_results else None
        opts = RunOpts(int(max_new_tokens), int(force_tokens_per_s), 0)
        check(_lib.load().qasr_run_batch_device(self._h, C.c_void_p(dev_ptr), off, ln, n, C.byref(opts), res))
        return [_take_result(res[i]) for i in range(n)] if want_results else None

    def set_context(self, ids):
        """system-prompt context token ids for the following runs (hot words; [] = the reference's prompt)"""
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.int32).reshape(-1))
        check(_lib.load().qasr_session_set_context(self._h, a.ctypes.data_as(C.c_void_p) if a.size else None,
                                                   int(a.size)))

    def set_draft(self, on: bool = True):
        """streaming decode: draft from this session's earlier transcripts, verify in one pass (greedy's tokens)"""
        check(_lib.load().qasr_session_set_draft(self._h, 1 if on else 0))

    def set_batch_invariant(self, on: bool = True):
        """batch runs decode every utterance with its single-utterance arithmetic (tokens independent of the batch)"""
        check(_lib.load().qasr_session_set_batch_invariant(self._h, 1 if on else 0))

    def set_draft_noise(self, rate: float, seed: int = 0):
        """benchmark / test hook: replace each proposed draft token by a random id with probability `rate`"""
        check(_lib.load().qasr_session_set_draft_noise(self._h, float(rate), int(seed)))

    def draft_stats(self) -> dict:
        st = (C.c_int64 * 4)()
        check(_lib.load().qasr_session_draft_stats(self._h, st))
        return dict(zip(("passes", "proposed", "accepted", "tokens"), list(st)))

    def set_encoder_cache(self, on: bool = True):
        """streaming encoder cache: reuse the previous run's complete encoder windows when the samples extend it"""
        check(_lib.load().qasr_session_set_encoder_cache(self._h, 1 if on else 0))

    def encoder_cache_stats(self) -> dict:
        st = (C.c_int64 * 3)()
        check(_lib.load().qasr_session_encoder_cache_stats(self._h, st))
        return dict(zip(("runs", "windows_reused", "windows_computed"), list(st)))

    def prompt_kv_rows_reused(self) -> int:
        """prompt rows whose K/V runs took over from the previous run (growing windows with the encoder cache)"""
        n = C.c_int64(0)
        check(_lib.load().qasr_session_prompt_kv_stats(self._h, C.byref(n)))
        return int(n.value)

    def audio_embeds(self) -> np.ndarray:
        """the audio-embedding rows [tokens][hidden] of this session's last run"""
        lib, n = _lib.load(), C.c_size_t(0)
        check(lib.qasr_session_audio_embeds(self._h, None, 0, C.byref(n)))
        out = np.empty(n.value, np.float32)
        check(lib.qasr_session_audio_embeds(self._h, out.ctypes.data_as(C.c_void_p), n.value, C.byref(n)))
        return out

    def forced_logits(self, audio, forced, one_pass: bool = False) -> np.ndarray:
        """teacher-forced logits [len(forced)+1][vocab]: one decode step per forced token, or (one_pass) the forced
        tokens as ONE draft verify pass (≤ 32) — bit-identical by the exact-row contract"""
        a = _f32(audio)
        f = np.ascontiguousarray(forced, dtype=np.int32)
        v = self.model.hparams["vocab"]
        out = np.empty((f.size + 1, v), np.float32)
        fn = _lib.load().qasr_session_forced_logits_verify if one_pass else _lib.load().qasr_session_forced_logits
        check(fn(self._h, a.ctypes.data_as(C.c_void_p), a.size, f.ctypes.data_as(C.c_void_p), f.size,
                 out.ctypes.data_as(C.c_void_p)))
        return out

    def forced_logits_batch(self, audios, forced, want) -> np.ndarray:
        """teacher forcing through the batched path (qasr_session_forced_logits_batch): audios[u] fed forced[u]
        ([count][n] ids); logits of the utterances in `want`, [len(want)][n + 1][vocab]"""
        arrs = [_f32(a) for a in audios]
        n = len(arrs)
        f = np.ascontiguousarray(forced, dtype=np.int32).reshape(n, -1)
        w = np.ascontiguousarray(want, dtype=np.int32)
        v = self.model.hparams["vocab"]
        out = np.empty((w.size, f.shape[1] + 1, v), np.float32)
        ptrs = (C.c_void_p * n)(*[a.ctypes.data_as(C.c_void_p).value for a in arrs])
        lens = (C.c_size_t * n)(*[a.size for a in arrs])
        check(_lib.load().qasr_session_forced_logits_batch(self._h, ptrs, lens, n, f.ctypes.data_as(C.c_void_p),
                                                           f.shape[1], w.ctypes.data_as(C.c_void_p), w.size,
                                                           out.ctypes.data_as(C.c_void_p)))
        return out

    def mel(self, audio):
        a = _f32(audio)
        n = max(a.size, 8000)
        tv = (n + 159) // 160
        tp = (tv + 99) // 100 * 100
        out = np.empty((self.model.hparams["n_mels"], tp), np.float32)
        t_valid, t_pad = C.c_int32(), C.c_int32()
        check(_lib.load().qasr_session_mel(self._h, a.ctypes.data_as(C.c_void_p), a.size,
                                           out.ctypes.data_as(C.c_void_p), C.byref(t_valid), C.byref(t_pad)))
        assert t_pad.value == tp
        return out, t_valid.value

    def encode(self, mel: np.ndarray, t_valid: int, want_enc: bool = False):
        hp = self.model.hparams
        mel = np.ascontiguousarray(mel, dtype=np.float32)
        t_pad = mel.shape[1]
        full, tail = divmod(t_valid, 100)
        n = tail
        for _ in range(3):
            n = (n - 1) // 2 + 1 if n > 0 else 0
        n_tok = full * 13 + n
        emb = np.empty((n_tok, hp["txt_h"]), np.float32)
        enc = np.empty((n_tok, hp["enc_d"]), np.float32) if want_enc else None
        got = C.c_int32()
        check(_lib.load().qasr_session_encode(self._h, mel.ctypes.data_as(C.c_void_p), t_pad, int(t_valid),
                                              emb.ctypes.data_as(C.c_void_p),
                                              enc.ctypes.data_as(C.c_void_p) if enc is not None else None,
                                              C.byref(got)))
        assert got.value == n_tok
        return (emb, enc) if want_enc else emb

    def prefill_logits(self, embeds: np.ndarray) -> np.ndarray:
        e = np.ascontiguousarray(embeds, dtype=np.float32)
        v = self.model.hparams["vocab"]
        out = np.empty((e.shape[0], v), np.float32)
        check(_lib.load().qasr_session_prefill_logits(self._h, e.ctypes.data_as(C.c_void_p), e.shape[0],
                                                      out.ctypes.data_as(C.c_void_p)))
        return out

    def close(self):
        if self._h:
            _lib.load().qasr_session_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
