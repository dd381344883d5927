"""Minimal protobuf wire-format reader for ONNX ModelProto (no onnx package needed).

Used only offline (in this container) to convert the FireRedVAD ONNX graph shipped with the
reference (src-tauri/resources/fireredvad_vad.onnx) into this repo's own weight container.
Field numbers follow onnx.proto (ModelProto.graph=7, GraphProto.node=1/initializer=5/input=11/
output=12, NodeProto input=1/output=2/name=3/op_type=4/attribute=5, TensorProto dims=1/
data_type=2/float_data=4/int64_data=7/name=8/raw_data=9, AttributeProto name=1/f=2/i=3/s=4/
t=5/floats=7/ints=8/type=20).
"""
import struct

import numpy as np


def _varint(buf, pos):
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def fields(buf):
    """Yield (field_number, wire_type, value) for one message."""
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            val, pos = _varint(buf, pos)
        elif wt == 1:
            val = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            val = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            val = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fno, wt, val


def _packed_varints(val):
    out = []
    pos = 0
    while pos < len(val):
        v, pos = _varint(val, pos)
        if v >= 1 << 63:
            v -= 1 << 64
        out.append(v)
    return out


_DT = {1: np.float32, 6: np.int32, 7: np.int64, 10: np.float16, 11: np.float64}


def tensor(buf):
    dims, dt, name, raw, fdata, idata = [], 1, "", None, [], []
    for f, wt, v in fields(buf):
        if f == 1:
            dims.extend(_packed_varints(v) if wt == 2 else [v])
        elif f == 2:
            dt = v
        elif f == 8:
            name = bytes(v).decode()
        elif f == 9:
            raw = bytes(v)
        elif f == 4:
            fdata.extend(struct.unpack(f"<{len(v)//4}f", v) if wt == 2 else struct.unpack("<f", v))
        elif f == 7:
            idata.extend(_packed_varints(v) if wt == 2 else [v])
    if raw is not None:
        arr = np.frombuffer(raw, dtype=_DT[dt]).copy()
    elif fdata:
        arr = np.asarray(fdata, dtype=np.float32)
    else:
        arr = np.asarray(idata, dtype=np.int64)
    return name, arr.reshape(dims) if dims else arr.reshape(())


def attribute(buf):
    a = {"name": "", "value": None}
    ints, floats = [], []
    for f, wt, v in fields(buf):
        if f == 1:
            a["name"] = bytes(v).decode()
        elif f == 2:
            a["value"] = struct.unpack("<f", v)[0]
        elif f == 3:
            a["value"] = v - (1 << 64) if v >= 1 << 63 else v
        elif f == 4:
            a["value"] = bytes(v).decode(errors="replace")
        elif f == 5:
            a["value"] = tensor(v)[1]
        elif f == 7:
            floats.extend(struct.unpack(f"<{len(v)//4}f", v) if wt == 2 else struct.unpack("<f", v))
        elif f == 8:
            ints.extend(_packed_varints(v) if wt == 2 else [v - (1 << 64) if v >= 1 << 63 else v])
    if ints:
        a["value"] = ints
    if floats:
        a["value"] = floats
    return a


def node(buf):
    n = {"inputs": [], "outputs": [], "name": "", "op": "", "attrs": {}}
    for f, wt, v in fields(buf):
        if f == 1:
            n["inputs"].append(bytes(v).decode())
        elif f == 2:
            n["outputs"].append(bytes(v).decode())
        elif f == 3:
            n["name"] = bytes(v).decode()
        elif f == 4:
            n["op"] = bytes(v).decode()
        elif f == 5:
            a = attribute(v)
            n["attrs"][a["name"]] = a["value"]
    return n


def load_model(path):
    data = memoryview(open(path, "rb").read())
    graph = None
    for f, wt, v in fields(data):
        if f == 7:
            graph = v
    nodes, inits, inputs, outputs = [], {}, [], []
    for f, wt, v in fields(graph):
        if f == 1:
            nodes.append(node(v))
        elif f == 5:
            name, arr = tensor(v)
            inits[name] = arr
        elif f == 11:
            for ff, _, vv in fields(v):
                if ff == 1:
                    inputs.append(bytes(vv).decode())
        elif f == 12:
            for ff, _, vv in fields(v):
                if ff == 1:
                    outputs.append(bytes(vv).decode())
    return {"nodes": nodes, "initializers": inits, "inputs": inputs, "outputs": outputs}
