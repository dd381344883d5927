"""Convert the reference's FireRedVAD assets into this repo's weight container (run once, offline).

Inputs (reference, read-only): src-tauri/resources/fireredvad_vad.onnx (DFSMN graph, firered_vad.py:76-85)
and fireredvad_cmvn.json (firered_vad.py:59-63).  Output: assets/fireredvad_dfsmn.qvad — a named-array
container (format in light-whisper_amd/csrc/vad_weights.cpp) holding the same fp32 values, re-laid out for
the HIP kernels.  FireRedVAD is Apache-2.0 (reference FireRedVAD-LICENSE.txt); see assets/NOTICE.
"""
import json
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import onnx_wire  # noqa: E402

REF = "/root/reference/src-tauri/resources"


def load_reference_vad(onnx_path=f"{REF}/fireredvad_vad.onnx", cmvn_path=f"{REF}/fireredvad_cmvn.json"):
    m = onnx_wire.load_model(onnx_path)
    init = m["initializers"]
    mats = [n["inputs"][1] for n in m["nodes"] if n["op"] == "MatMul"]
    assert len(mats) == 18, len(mats)
    w = {}
    w["w1"], w["w2"] = init[mats[0]], init[mats[1]]
    for k in range(7):
        w[f"wa{k}"] = init[mats[2 + 2 * k]]
        w[f"wb{k}"] = init[mats[3 + 2 * k]]
    w["wd"], w["wo"] = init[mats[16]], init[mats[17]].reshape(256)
    w["b1"] = init["model.dfsmn.fc1.0.bias"]
    w["b2"] = init["model.dfsmn.fc2.0.bias"]
    for k in range(7):
        w[f"ba{k}"] = init[f"model.dfsmn.fsmns.{k}.fc1.0.bias"]
    w["bd"] = init["model.dfsmn.dnns.0.bias"]
    w["bo"] = init["model.out.bias"].reshape(1)
    w["lb0"] = init["model.dfsmn.fsmn1.lookback_filter.weight"].reshape(128, 20)
    w["la0"] = init["model.dfsmn.fsmn1.lookahead_filter.weight"].reshape(128, 20)
    for k in range(7):
        w[f"lb{k+1}"] = init[f"model.dfsmn.fsmns.{k}.fsmn.lookback_filter.weight"].reshape(128, 20)
        w[f"la{k+1}"] = init[f"model.dfsmn.fsmns.{k}.fsmn.lookahead_filter.weight"].reshape(128, 20)
    cm = json.load(open(cmvn_path, encoding="utf-8"))
    w["mean"] = np.asarray(cm["mean"], dtype=np.float32)
    w["istd"] = np.asarray(cm["inverse_std"], dtype=np.float32)
    return {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in w.items()}, m


ORDER = (["mean", "istd", "w1", "b1", "w2", "b2"] + [f"lb{i}" for i in range(8)] + [f"la{i}" for i in range(8)]
         + [f"wa{i}" for i in range(7)] + [f"ba{i}" for i in range(7)] + [f"wb{i}" for i in range(7)]
         + ["wd", "bd", "wo", "bo"])


def write_qvad(path, w):
    with open(path, "wb") as f:
        f.write(b"QVADF32\0")
        f.write(struct.pack("<II", 1, len(ORDER)))
        for name in ORDER:
            a = w[name]
            dims = list(a.shape) + [1] * (4 - a.ndim)
            f.write(name.encode().ljust(32, b"\0"))
            f.write(struct.pack("<5I", a.ndim, *dims))
        pos = f.tell()
        f.write(b"\0" * ((-pos) % 16))
        for name in ORDER:
            f.write(w[name].astype("<f4").tobytes())
            f.write(b"\0" * ((-w[name].nbytes) % 16))


def read_qvad(path):
    data = open(path, "rb").read()
    assert data[:8] == b"QVADF32\0"
    ver, n = struct.unpack_from("<II", data, 8)
    pos = 16
    meta = []
    for _ in range(n):
        name = data[pos:pos + 32].rstrip(b"\0").decode()
        nd, *dims = struct.unpack_from("<5I", data, pos + 32)
        meta.append((name, tuple(dims[:nd])))
        pos += 52
    pos += (-pos) % 16
    out = {}
    for name, shape in meta:
        cnt = int(np.prod(shape))
        out[name] = np.frombuffer(data, dtype="<f4", count=cnt, offset=pos).reshape(shape).copy()
        pos += cnt * 4
        pos += (-pos) % 16
    return out


if __name__ == "__main__":
    w, _ = load_reference_vad()
    out = os.path.join(os.path.dirname(__file__), "..", "assets", "fireredvad_dfsmn.qvad")
    write_qvad(out, w)
    back = read_qvad(out)
    assert all(np.array_equal(back[k], w[k]) for k in w)
    print("wrote", os.path.abspath(out), sum(v.size for v in w.values()), "floats")
