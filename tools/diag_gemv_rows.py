#!/usr/bin/env python3
"""Diagnosis (GPU): the exact-row contract of the fused norm + QKV GEMV on the rows where a draft verify pass departed
(tools/diag_layers.py: layer 16, row 24 of a 32-row pass, 1.7B, 4 s clip seed 31).  Takes the pass's layer input rows
from the stage dump, the layer's real weights from the oracle's seeded model, and compares every row of one 32-row
gemv_fused launch with its own 1-row launch, and the separate rmsnorm_q8 rows.
usage: python tools/diag_gemv_rows.py [arch] [layer] [seconds] [n] [audio seed] [prior runs]"""
import ctypes as C
import os
import re
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
TMP = tempfile.mkdtemp(prefix="qasr_dump_")
os.environ["QASR_DUMP_DIR"] = TMP
os.environ["QASR_NO_GRAPH"] = "1"   # dumps synchronise the stream: eager passes only (engine.cpp dump_rows)
from bench import speech_like  # noqa: E402


def q8_split(blocks, n, k):
    b = blocks.reshape(n, k // 32, 34)
    d = b[:, :, :2].copy().view(np.float16).reshape(n, k // 32)
    q = b[:, :, 2:].copy().view(np.int8).reshape(n, k)
    return q, d


def main():
    import torch

    import oracle
    from qasr import _lib
    from qasr.transcribe_cpp import Model

    arch = sys.argv[1] if len(sys.argv) > 1 else "qwen3-asr-1.7b"
    layer = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    secs = float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    aseed = int(sys.argv[5]) if len(sys.argv) > 5 else 31
    prior = [int(v) for v in sys.argv[6].split(",")] if len(sys.argv) > 6 else [2, 9]
    m = Model.synthetic(arch, seed=7)
    s = m.session(kv_type="f16", n_ctx=4096)
    audio = speech_like(np.random.default_rng(aseed), int(secs * 16000))
    for p in prior:
        f = np.array([1000 + 37 * i for i in range(p)], np.int32)
        s.forced_logits(audio, f)
        s.forced_logits(audio, f, one_pass=True)
    db = os.path.join(TMP, "verify")
    os.makedirs(db)
    os.environ["QASR_DUMP_DIR"] = db
    forced = np.array([1000 + 37 * i for i in range(n)], np.int32)
    s.forced_logits(audio, forced, one_pass=True)
    os.environ["QASR_DUMP_DIR"] = TMP
    xin = None
    for fn in sorted(os.listdir(db)):
        mm = re.match(r"(\d+)_(\w+?)_L(\d+)_r(\d+)\.bin", fn)
        if mm and mm.group(2) == "x_in" and int(mm.group(3)) == layer and int(mm.group(4)) == n:
            xin = np.fromfile(os.path.join(db, fn), np.float32).reshape(n, -1)
    assert xin is not None
    K = xin.shape[1]
    oracle.set_mode(engine=True)
    cfg = oracle.arch_config(arch)
    o = oracle.Model(cfg, seed=7)
    lib_o = oracle.lib()

    def get(name, kind, shape):
        p = lib_o.orc_model_get(o.h, name.encode())
        assert p, name
        if kind == "f32":
            return np.ctypeslib.as_array((C.c_float * int(np.prod(shape))).from_address(p)).copy().reshape(shape)
        nbytes = shape[0] * shape[1] // 32 * 34
        return np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p)).copy().reshape(shape[0], -1)

    nw = get(f"blk.{layer}.attn_norm.weight", "f32", (K,))
    QD, KD = cfg["txt_heads"] * cfg["head_dim"], cfg["txt_kv_heads"] * cfg["head_dim"]
    blocks = np.concatenate([get(f"blk.{layer}.attn_q.weight", "q8", (QD, K)),
                             get(f"blk.{layer}.attn_k.weight", "q8", (KD, K)),
                             get(f"blk.{layer}.attn_v.weight", "q8", (KD, K))])
    N = QD + 2 * KD
    qs, sc = q8_split(blocks, N, K)
    dev = torch.device("cuda:0")
    L = _lib.load()
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    x = torch.from_numpy(xin).to(dev)
    w = torch.from_numpy(nw).to(dev)
    wq = torch.from_numpy(qs).to(dev)
    ws = torch.from_numpy(sc).to(dev)

    def gemv(r0, rows):
        y = torch.empty((rows, N), dtype=torch.float32, device=dev)
        _lib.check(L.qasr_op_gemv_fused(1, C.c_void_p(x.data_ptr() + r0 * K * 4), K, P(w), 1e-6, rows, None, None,
                                        P(wq), P(ws), N, K, P(y), P(y), N, 0, None, None, None))
        return y.cpu().numpy()

    def rms(r0, rows):
        q = torch.empty((rows, K), dtype=torch.int8, device=dev)
        d = torch.empty((rows, K // 32), dtype=torch.float32, device=dev)
        _lib.check(L.qasr_op_rmsnorm_q8(C.c_void_p(x.data_ptr() + r0 * K * 4), rows, K, P(w), 1e-6, P(q), P(d), None))
        return q.cpu().numpy(), d.cpu().numpy()

    full = gemv(0, n)
    bad = []
    for r in range(n):
        one = gemv(r, 1)[0]
        if not np.array_equal(one, full[r]):
            bad.append((r, float(np.abs(one - full[r]).max()), int((one != full[r]).sum())))
    print(f"{arch} L{layer}: rows of the {n}-row fused norm+QKV GEMV differing from their 1-row launch: {bad}", flush=True)
    for grp in (8, 4, 2):
        got = np.concatenate([gemv(g0, min(grp, n - g0)) for g0 in range(0, n, grp)])
        print(f"  launches of {grp} rows vs {n}: rows differing {[r for r in range(n) if not np.array_equal(got[r], full[r])]}",
              flush=True)
    qa, da = rms(0, n)
    for r in range(n):
        q1, d1 = rms(r, 1)
        if not (np.array_equal(q1[0], qa[r]) and np.array_equal(d1[0], da[r])):
            print(f"  rmsnorm_q8 row {r} differs between M={n} and M=1", flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
