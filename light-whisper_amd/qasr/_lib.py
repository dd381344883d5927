"""ctypes binding of libqasr.so (include/qasr.h).

This is the reference-side binding a maintainer adds next to `transcribe_cpp`: it loads
the in-tree HIP library and fails loudly when it is missing — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)                 # light-whisper_amd/
LIB_PATH = os.environ.get("QASR_LIB") or os.path.join(PKG_ROOT, "libqasr.so")   # QASR_LIB: A/B builds (tools)
ENGINE_PATH = os.path.join(PKG_ROOT, "engine")
REPO_ROOT = os.path.dirname(PKG_ROOT)
VAD_ASSET = os.path.join(REPO_ROOT, "assets", "fireredvad_dfsmn.qvad")

QASR_OK = 0
EPI_STORE, EPI_RESID, EPI_GELU = 0, 1, 2


class QasrError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"qasr error {code}: {msg}")
        self.code = code


class HParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "n_mels", "conv_ch", "enc_d", "enc_layers", "enc_heads", "enc_ffn", "n_window", "n_window_infer",
        "proj_out", "txt_h", "txt_layers", "txt_heads", "txt_kv_heads", "head_dim", "txt_ffn", "vocab")] + [
        ("rope_theta", C.c_float), ("rms_eps", C.c_float), ("ln_eps", C.c_float)] + [(n, C.c_int32) for n in (
            "tok_im_start", "tok_im_end", "tok_system", "tok_user", "tok_assistant", "tok_newline",
            "tok_audio_start", "tok_audio_end", "tok_audio_pad", "tok_eos0", "tok_eos1", "tok_asr_text")]

    def to_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Result(C.Structure):
    _fields_ = [("text", C.c_char_p), ("language", C.c_char_p), ("raw", C.c_char_p),
                ("tokens", C.POINTER(C.c_int32)), ("n_tokens", C.c_int32), ("n_audio_tokens", C.c_int32),
                ("n_prompt", C.c_int32), ("ms_mel", C.c_double), ("ms_encoder", C.c_double),
                ("ms_prefill", C.c_double), ("ms_decode", C.c_double), ("truncated", C.c_int32)]


class RunOpts(C.Structure):
    _fields_ = [("max_new_tokens", C.c_int32), ("force_tokens_per_s", C.c_int32), ("return_logits", C.c_int32)]


class VadOptions(C.Structure):
    _fields_ = [("threshold", C.c_float), ("smooth_window_frames", C.c_int32),
                ("min_speech_duration_ms", C.c_int32), ("min_silence_duration_ms", C.c_int32),
                ("speech_pad_ms", C.c_int32)]


class Segment(C.Structure):
    _fields_ = [("start", C.c_int64), ("end", C.c_int64)]


# every exported symbol with (restype, argtypes); the not-gpu test checks each one is exported
P, I32, I64, F32, SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_size_t
SIGNATURES = {
    "qasr_last_error": (C.c_char_p, []),
    "qasr_version": (C.c_char_p, []),
    "qasr_device_info": (C.c_int, [C.c_char_p, SZ, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "qasr_set_device": (C.c_int, [C.c_int]),
    "qasr_model_open": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(P)]),
    "qasr_model_open_synthetic": (C.c_int, [C.c_char_p, C.POINTER(HParams), C.c_uint64, C.POINTER(P)]),
    "qasr_model_hparams": (C.c_int, [P, C.POINTER(HParams)]),
    "qasr_model_weight_bytes": (C.c_int64, [P]),
    "qasr_model_open_shell": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(HParams), C.POINTER(P)]),
    "qasr_model_weight_blob": (C.c_int, [P, C.POINTER(P), C.POINTER(C.c_size_t)]),
    "qasr_model_weights_received": (C.c_int, [P]),
    "qasr_model_set_precision": (C.c_int, [P, C.c_char_p]),
    "qasr_model_tokenize": (C.c_int, [P, C.c_char_p, C.c_size_t, P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "qasr_session_set_context": (C.c_int, [P, P, I32]),
    "qasr_model_detokenize": (C.c_int, [P, P, I32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "qasr_model_tensor_table": (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "qasr_model_export_tensor": (C.c_int, [P, C.c_char_p, P, SZ, C.POINTER(SZ)]),
    "qasr_model_close": (None, [P]),
    "qasr_session_open": (C.c_int, [P, C.c_char_p, I32, C.POINTER(P)]),
    "qasr_session_run": (C.c_int, [P, P, SZ, I32, C.POINTER(Result)]),
    "qasr_session_run_opts": (C.c_int, [P, P, SZ, C.POINTER(RunOpts), C.POINTER(Result)]),
    "qasr_run_batch": (C.c_int, [P, C.POINTER(P), C.POINTER(SZ), I32, C.POINTER(RunOpts), C.POINTER(Result)]),
    "qasr_run_batch_device": (C.c_int, [P, P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), I32,
                                        C.POINTER(RunOpts), C.POINTER(Result)]),
    "qasr_result_free": (None, [C.POINTER(Result)]),
    "qasr_session_close": (None, [P]),
    "qasr_session_forced_logits": (C.c_int, [P, P, SZ, P, I32, P]),
    "qasr_session_forced_logits_verify": (C.c_int, [P, P, SZ, P, I32, P]),
    "qasr_session_forced_logits_batch": (C.c_int, [P, P, P, I32, P, I32, P, I32, P]),
    "qasr_session_mel": (C.c_int, [P, P, SZ, P, C.POINTER(I32), C.POINTER(I32)]),
    "qasr_session_encode": (C.c_int, [P, P, I32, I32, P, P, C.POINTER(I32)]),
    "qasr_session_prefill_logits": (C.c_int, [P, P, I32, P]),
    "qasr_vad_default_options": (None, [C.POINTER(VadOptions)]),
    "qasr_vad_open": (C.c_int, [C.c_char_p, C.POINTER(P)]),
    "qasr_vad_probabilities": (C.c_int, [P, P, SZ, P, SZ, C.POINTER(SZ)]),
    "qasr_vad_features": (C.c_int, [P, P, SZ, P, SZ, C.POINTER(SZ)]),
    "qasr_vad_speech_timestamps": (C.c_int, [P, P, SZ, C.POINTER(VadOptions), C.POINTER(Segment), SZ,
                                             C.POINTER(SZ)]),
    "qasr_vad_timestamps_from_probabilities": (C.c_int, [P, SZ, I64, C.POINTER(VadOptions), C.POINTER(Segment),
                                                         SZ, C.POINTER(SZ)]),
    "qasr_vad_close": (None, [P]),
    "qasr_utf8_replace_invalid": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "qasr_decode_pcm_s16le": (C.c_int, [C.c_char_p, SZ, P, SZ, C.POINTER(SZ)]),
    "qasr_resample_linear": (C.c_int, [P, SZ, C.c_double, P, SZ, C.POINTER(SZ)]),
    "qasr_audio_load_path": (C.c_int, [C.c_char_p, P, SZ, C.POINTER(SZ)]),
    "qasr_session_set_draft": (C.c_int, [P, I32]),
    "qasr_session_set_batch_invariant": (C.c_int, [P, I32]),
    "qasr_dist_unique_id": (C.c_int, [P, SZ]),
    "qasr_dist_init": (C.c_int, [P, I32, I32, I32, P]),
    "qasr_dist_init_deadline": (C.c_int, [P, I32, I32, I32, C.c_double, P]),
    "qasr_dist_close": (None, [P]),
    "qasr_dist_broadcast": (C.c_int, [P, P, P, SZ, I32]),
    "qasr_dist_broadcast_weights": (C.c_int, [P, P, I32, P]),
    "qasr_dist_gather_tokens": (C.c_int, [P, P, I32, P, P, P, SZ, P, SZ, P, P]),
    "qasr_dist_agree": (C.c_int, [P, I32, P]),
    "qasr_tokenizer_open": (C.c_int, [P, I32, P, P, I32, P]),
    "qasr_tokenizer_encode": (C.c_int, [P, C.c_char_p, SZ, P, SZ, P]),
    "qasr_tokenizer_close": (None, [P]),
    "qasr_session_set_draft_noise": (C.c_int, [P, F32, C.c_uint64]),
    "qasr_session_draft_stats": (C.c_int, [P, C.POINTER(C.c_int64)]),
    "qasr_session_set_encoder_cache": (C.c_int, [P, I32]),
    "qasr_session_encoder_cache_stats": (C.c_int, [P, C.POINTER(C.c_int64)]),
    "qasr_session_prompt_kv_stats": (C.c_int, [P, C.POINTER(C.c_int64)]),
    "qasr_session_audio_embeds": (C.c_int, [P, P, SZ, C.POINTER(SZ)]),
    "qasr_parse_transcript": (C.c_int, [C.c_char_p, SZ, C.c_char_p, SZ, C.POINTER(SZ), C.c_char_p, SZ,
                                        C.POINTER(SZ)]),
    "qasr_op_quant_rows": (C.c_int, [P, I32, I32, I32, P, P, P]),
    "qasr_op_repack_q8": (C.c_int, [P, I64, P, P, P]),
    "qasr_op_linear_q8": (C.c_int, [P, P, I32, P, P, I32, I32, P, P, P, I32, I32, I32, P]),
    "qasr_op_rmsnorm_q8": (C.c_int, [P, I32, I32, P, F32, P, P, P]),
    "qasr_op_layernorm_q8": (C.c_int, [P, I32, I32, P, P, F32, P, P, P, P]),
    "qasr_op_swiglu_q8": (C.c_int, [P, I32, I32, P, P, P]),
    "qasr_op_interleave_gate_up": (C.c_int, [P, P, I32, I32, P]),
    "qasr_op_gemm_swiglu_q8": (C.c_int, [P, P, I32, P, P, I32, I32, P, P, P]),
    "qasr_op_gemm_swiglu_q8_cfg": (C.c_int, [P, P, I32, P, P, I32, I32, P, P, I32, P]),
    "qasr_op_set_gemm_fixup": (C.c_int, [P, C.c_int64, P, I32]),
    "qasr_op_gemm_exact_rows": (C.c_int, [P, P, I32, P, P, I32, I32, P, P, I32, I32, P]),
    "qasr_op_swiglu_q8_interleaved": (C.c_int, [P, I32, I32, P, P, P]),
    "qasr_op_xr_vocab": (C.c_int, [P, P, I32, P, P, I32, I32, P, I32, P]),
    "qasr_op_gemv_fused": (C.c_int, [I32, P, I32, P, F32, I32, P, P, P, P, I32, I32, P, P, I32, I32, P, P, P]),
    "qasr_op_qk_norm_rope": (C.c_int, [P, I32, I32, I32, I32, P, P, P, P, P, F32, P, P, P, P]),
    "qasr_op_q8_to_mx": (C.c_int, [P, P, I32, C.c_int64, P, P, P]),
    "qasr_op_stage_scales": (C.c_int, [P, I32, I32, P, P]),
    "qasr_op_register_stage_scales": (C.c_int, [P, I32, I32, P]),
    "qasr_op_xr_linear": (C.c_int, [P, P, P, P, C.c_float, I32, P, P, I32, I32, P, I32, I32, P]),
    "qasr_op_xr_gu_swiglu": (C.c_int, [P, P, P, P, C.c_float, I32, P, P, I32, I32, P, P, P]),
    "qasr_op_gemm_mx": (C.c_int, [P, P, I32, P, P, I32, I32, P, P, P, I32, I32, P, P, I32, P]),
    "qasr_op_linear_q8_ex": (C.c_int, [P, P, I32, P, P, I32, I32, P, P, I32, I32, P, P, I32, P]),
    "qasr_op_attention_decode_fused": (C.c_int, [P, I32, I32, I32, I32, P, P, P, P, P, F32, P, P, P, P, F32, P, P,
                                                 P]),
    "qasr_op_attention_decode_split": (C.c_int, [P, I32, I32, I32, I32, P, P, P, P, P, F32, P, P, P, P, F32, P, P,
                                                 P, P, P]),
    "qasr_op_attention": (C.c_int, [P, I32, P, P, I32, P, P, I32, I32, I32, I32, F32, P, P, P, P]),
    "qasr_op_attention_dense": (C.c_int, [P, I32, P, P, I32, P, P, I32, I32, I32, I32, F32, P, P, P, I32, P]),
    "qasr_op_argmax": (C.c_int, [P, I32, I32, P, P]),
    "qasr_op_embed_rows": (C.c_int, [P, I32, P, P, I32, P, P, P]),
    "qasr_op_synth_q8": (C.c_int, [C.c_uint64, C.c_char_p, I64, I64, F32, P, P, P]),
    "qasr_op_rope_table": (C.c_int, [I32, I32, F32, P]),
    "qasr_op_mel": (C.c_int, [P, I64, I32, P, P]),
    "qasr_op_conv3x3_gelu": (C.c_int, [P, I32, I32, I32, P, P, I32, P, I32, P]),
    "qasr_op_fbank": (C.c_int, [P, I64, P, P]),
    "qasr_stream_sync": (C.c_int, [P]),
    "qasr_prof_enable": (C.c_int, [C.c_int]),
    "qasr_set_deterministic": (C.c_int, [I32]),
    "qasr_get_deterministic": (C.c_int, [P]),
    "qasr_prof_reset": (C.c_int, []),
    "qasr_prof_report": (C.c_int, [C.c_char_p, SZ, C.POINTER(SZ)]),
}

_LIB = None


def load(path: str = LIB_PATH):
    """Load libqasr.so (raises if it is missing — no fallback path exists)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise FileNotFoundError(f"libqasr.so not built at {path}; run `make -C light-whisper_amd` "
                                "(or __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int):
    if rc != QASR_OK:
        raise QasrError(rc, load().qasr_last_error().decode("utf-8", "replace"))
    return rc


def exported_symbols(path: str = LIB_PATH):
    lib = C.CDLL(path)
    return {n for n in SIGNATURES if hasattr(lib, n)}
