#!/usr/bin/env python3
"""Write a device-resident model back out as a GGUF v3 file in this engine's naming convention (DESIGN.md §tensor
names; the metadata keys `load_gguf_model` in light-whisper_amd/csrc/model.cpp reads).  Used by the loader's
round-trip parity tests (a synthetic model → GGUF → qasr_model_open must give the same weights and tokens) and to
hand-craft checkpoints for the engine.  Tensor data comes from qasr_model_export_tensor, already in GGUF order
(Q8_0 blocks of f16 d + 32 int8; conv kernels [Cout][Cin][3][3])."""
from __future__ import annotations

import struct

GT_U32, GT_I32, GT_F32, GT_STR, GT_ARR = 4, 5, 6, 8, 9
ALIGN = 32

_INT_KEYS = {
    "audio.n_mels": "n_mels", "audio.conv_channels": "conv_ch", "audio.embedding_length": "enc_d",
    "audio.block_count": "enc_layers", "audio.attention.head_count": "enc_heads",
    "audio.feed_forward_length": "enc_ffn", "audio.n_window": "n_window", "audio.n_window_infer": "n_window_infer",
    "embedding_length": "txt_h", "audio.projection_dim": "proj_out", "block_count": "txt_layers",
    "attention.head_count": "txt_heads", "attention.head_count_kv": "txt_kv_heads", "attention.key_length": "head_dim",
    "feed_forward_length": "txt_ffn",
    "token.im_start": "tok_im_start", "token.im_end": "tok_im_end", "token.system": "tok_system",
    "token.user": "tok_user", "token.assistant": "tok_assistant", "token.newline": "tok_newline",
    "token.audio_start": "tok_audio_start", "token.audio_end": "tok_audio_end", "token.audio_pad": "tok_audio_pad",
    "token.eos0": "tok_eos0", "token.eos1": "tok_eos1", "token.asr_text": "tok_asr_text",
}
_FLOAT_KEYS = {"rope.freq_base": "rope_theta", "attention.layer_norm_rms_epsilon": "rms_eps",
               "audio.attention.layer_norm_epsilon": "ln_eps"}


def _s(x: str) -> bytes:
    b = x.encode()
    return struct.pack("<Q", len(b)) + b


def _kv(key: str, vtype: int, payload: bytes) -> bytes:
    return _s(key) + struct.pack("<I", vtype) + payload


def export_gguf(model, path: str, name: str = "qwen3-asr-custom", tokens: list[str] | None = None,
                token_types: list[int] | None = None, untied: bool = False) -> None:
    """`model`: a qasr.transcribe_cpp.Model.  `tokens`: optional vocabulary pieces (tokenizer.ggml.tokens);
    `untied`: also write output.weight (a copy of token_embd) to exercise the untied-checkpoint layout."""
    hp = model.hparams
    table = model.tensor_table()
    arch = "qwen3-asr"
    kvs = [_kv("general.architecture", GT_STR, _s(arch)), _kv("general.name", GT_STR, _s(name)),
           _kv("general.alignment", GT_U32, struct.pack("<I", ALIGN))]
    for k, f in _INT_KEYS.items():
        kvs.append(_kv(f"{arch}.{k}", GT_I32, struct.pack("<i", int(hp[f]))))
    for k, f in _FLOAT_KEYS.items():
        kvs.append(_kv(f"{arch}.{k}", GT_F32, struct.pack("<f", float(hp[f]))))
    if tokens is not None:
        kvs.append(_kv("tokenizer.ggml.tokens", GT_ARR,
                       struct.pack("<IQ", GT_STR, len(tokens)) + b"".join(_s(t) for t in tokens)))
        types = token_types if token_types is not None else [1] * len(tokens)
        kvs.append(_kv("tokenizer.ggml.token_type", GT_ARR,
                       struct.pack("<IQ", GT_I32, len(types)) + b"".join(struct.pack("<i", t) for t in types)))

    infos, blobs, off = [], [], 0
    entries = sorted(table.items())
    if untied:
        entries.append(("output.weight", table["token_embd.weight"]))
    for tname, (gtype, rows, cols, cin) in entries:
        src = "token_embd.weight" if tname == "output.weight" else tname
        if gtype == 8:
            nbytes, dims = rows * (cols // 32) * 34, (cols, rows)
        elif gtype == 0:
            nbytes, dims = rows * 4, (rows,)
        else:
            nbytes, dims = rows * 2, (3, 3, cin, rows // (9 * cin))
        data = model.export_tensor(src, nbytes).tobytes()
        assert len(data) == nbytes, tname
        infos.append(_s(tname) + struct.pack("<I", len(dims)) + b"".join(struct.pack("<Q", d) for d in dims)
                     + struct.pack("<IQ", gtype, off))
        pad = (-len(data)) % ALIGN
        blobs.append(data + b"\0" * pad)
        off += len(data) + pad

    head = b"GGUF" + struct.pack("<IQQ", 3, len(infos), len(kvs)) + b"".join(kvs) + b"".join(infos)
    head += b"\0" * ((-len(head)) % ALIGN)
    with open(path, "wb") as f:
        f.write(head)
        for b in blobs:
            f.write(b)
