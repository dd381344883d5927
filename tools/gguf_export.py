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


_AUDIO_LAYER = {"ln1": "self_attn_layer_norm", "ln2": "final_layer_norm", "attn_q": "self_attn.q_proj",
                "attn_k": "self_attn.k_proj", "attn_v": "self_attn.v_proj", "attn_out": "self_attn.out_proj",
                "ffn_up": "fc1", "ffn_down": "fc2"}
_TEXT_LAYER = {"attn_norm": "input_layernorm", "ffn_norm": "post_attention_layernorm", "attn_q_norm": "self_attn.q_norm",
               "attn_k_norm": "self_attn.k_norm", "attn_q": "self_attn.q_proj", "attn_k": "self_attn.k_proj",
               "attn_v": "self_attn.v_proj", "attn_output": "self_attn.o_proj", "ffn_gate": "mlp.gate_proj",
               "ffn_up": "mlp.up_proj", "ffn_down": "mlp.down_proj"}


def convention_name(canon: str, names: str) -> str:
    """This engine's tensor name → the same tensor in another naming convention: "engine" (as is), "hf-thinker"
    (the original qwen_asr state dict: thinker.audio_tower.* / thinker.model.* / thinker.lm_head) or "hf"
    (transformers' Qwen3ASRForConditionalGeneration: model.audio_tower.*, model.multi_modal_projector.linear_{1,2},
    model.language_model.*, lm_head)."""
    if names == "engine":
        return canon
    ap, tp, lm = (("thinker.audio_tower.", "thinker.model.", "thinker.lm_head.weight") if names == "hf-thinker" else
                  ("model.audio_tower.", "model.language_model.", "lm_head.weight"))
    parts = canon.split(".")
    leaf = parts[-1]
    if canon.startswith("a.conv") and not canon.startswith("a.conv_out"):
        return f"{ap}conv2d{parts[1][4:]}.{leaf}"
    if canon == "a.conv_out.weight":
        return ap + "conv_out.weight"
    if canon.startswith("a.blk."):
        return f"{ap}layers.{parts[2]}.{_AUDIO_LAYER[parts[3]]}.{leaf}"
    if canon.startswith("a.ln_post."):
        return f"{ap}ln_post.{leaf}"
    if canon.startswith("a.proj"):
        k = parts[1][4]
        return f"{ap}proj{k}.{leaf}" if names == "hf-thinker" else f"model.multi_modal_projector.linear_{k}.{leaf}"
    if canon == "token_embd.weight":
        return tp + "embed_tokens.weight"
    if canon == "output_norm.weight":
        return tp + "norm.weight"
    if canon == "output.weight":
        return lm
    if canon.startswith("blk."):
        return f"{tp}layers.{parts[1]}.{_TEXT_LAYER[parts[2]]}.{leaf}"
    raise KeyError(canon)


def _s(x: str) -> bytes:
    b = x.encode()
    return struct.pack("<Q", len(b)) + b


def _kv(key: str, vtype: int, payload: bytes) -> bytes:
    return _s(key) + struct.pack("<I", vtype) + payload


def export_gguf(model, path: str, name: str = "qwen3-asr-custom", tokens: list[str] | None = None,
                token_types: list[int] | None = None, untied: bool = False, names: str = "engine",
                f16_vectors: tuple = (), f16_round: tuple = (), drop_keys: tuple = (),
                extra_tensors: tuple = ()) -> None:
    """`model`: a qasr.transcribe_cpp.Model.  `tokens`: optional vocabulary pieces (tokenizer.ggml.tokens);
    `untied`: also write output.weight (a copy of token_embd) to exercise the untied-checkpoint layout.
    `names`: tensor naming convention (convention_name); the "hf*" conventions write llama.cpp's text-model metadata
    keys (qwen3.rope.freq_base, qwen3.attention.layer_norm_rms_epsilon) and no audio / special-token keys, so the
    loader must derive the audio hyper-parameters from the shapes and the special tokens from the vocabulary.
    `f16_vectors`: f32 tensors to store as F16 (rounded); `f16_round`: f32 tensors rounded to f16 but stored as F32
    (the same values: the loader must give identical models); `drop_keys`: metadata keys to omit;
    `extra_tensors`: (name, f32 values) written as well (negative tests)."""
    import numpy as np

    hp = model.hparams
    table = model.tensor_table()
    arch = "qwen3-asr" if names == "engine" else "qwen3asr"
    kvs = [_kv("general.architecture", GT_STR, _s(arch)), _kv("general.name", GT_STR, _s(name)),
           _kv("general.alignment", GT_U32, struct.pack("<I", ALIGN))]
    if names == "engine":
        ints, floats = {f"{arch}.{k}": f for k, f in _INT_KEYS.items()}, {f"{arch}.{k}": f for k, f in _FLOAT_KEYS.items()}
    else:
        ints = {"qwen3.block_count": "txt_layers", "qwen3.embedding_length": "txt_h"}
        floats = {"qwen3.rope.freq_base": "rope_theta", "qwen3.attention.layer_norm_rms_epsilon": "rms_eps"}
    for k, f in ints.items():
        if k not in drop_keys:
            kvs.append(_kv(k, GT_I32, struct.pack("<i", int(hp[f]))))
    for k, f in floats.items():
        if k not in drop_keys:
            kvs.append(_kv(k, GT_F32, struct.pack("<f", float(hp[f]))))
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
        if gtype == 0 and tname in f16_vectors:      # stored as F16 (rounded)
            data, gtype = np.frombuffer(data, np.float32).astype(np.float16).tobytes(), 1
        elif gtype == 0 and tname in f16_round:      # the same rounded values, stored as F32
            data = np.frombuffer(data, np.float32).astype(np.float16).astype(np.float32).tobytes()
        infos.append(_s(convention_name(tname, names)) + struct.pack("<I", len(dims))
                     + b"".join(struct.pack("<Q", d) for d in dims) + struct.pack("<IQ", gtype, off))
        pad = (-len(data)) % ALIGN
        blobs.append(data + b"\0" * pad)
        off += len(data) + pad

    for tname, values in extra_tensors:
        data = np.asarray(values, np.float32).tobytes()
        infos.append(_s(tname) + struct.pack("<I", 1) + struct.pack("<Q", len(data) // 4) + struct.pack("<IQ", 0, off))
        pad = (-len(data)) % ALIGN
        blobs.append(data + b"\0" * pad)
        off += len(data) + pad

    head = b"GGUF" + struct.pack("<IQQ", 3, len(infos), len(kvs)) + b"".join(kvs) + b"".join(infos)
    head += b"\0" * ((-len(head)) % ALIGN)
    with open(path, "wb") as f:
        f.write(head)
        for b in blobs:
            f.write(b)
