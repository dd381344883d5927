"""MXFP8 precision mode (tolerance parity only): the Q8 → MXFP8 conversion bit for bit against
the oracle's restatement of the OCP MX formats, and the block-scaled fp8 GEMM (v_mfma_scale_f32_16x16x128_f8f6f4)
against a float64 product of the same MXFP8 operands.

Tolerance of the GEMM: |y - ref| ≤ 1e-4 · Σ|a·b| per output.  The block-scaled instruction's internal sum is not a
full f32 chain: single 128-deep products land up to ~1.1e-5 · Σ|a·b| from the float64 value (measured), far below
the e4m3 element rounding (2^-4 relative) that dominates this mode's error.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from qasr import _lib
from test_ops_gpu import L, dev, empty, host, ptr, quant_ref

pytestmark = pytest.mark.gpu


def _mx_on_gpu(q, d, f16, torch_dev):
    import torch

    nblk = q.size // 32
    qt, dt = dev(q, torch_dev), dev(d, torch_dev)
    q8 = empty((q.size,), torch.uint8, torch_dev)
    s8 = empty((nblk,), torch.uint8, torch_dev)
    _lib.check(L().qasr_op_q8_to_mx(ptr(qt), ptr(dt), 1 if f16 else 0, nblk, ptr(q8), ptr(s8), None))
    return host(q8).reshape(q.shape), host(s8)


@pytest.mark.parametrize("f16", [False, True])
def test_q8_to_mx_bit_exact(torch_dev, f16):
    rng = np.random.default_rng(3 + f16)
    nblk = 4096
    q = rng.integers(-127, 128, (nblk, 32)).astype(np.int8)
    q[5] = 0                                   # empty block
    q[6] = 0
    q[6, 3] = -1                               # tiny block
    scale = np.exp(rng.uniform(-14, 6, nblk)).astype(np.float32)
    d = scale.astype(np.float16) if f16 else scale.astype(np.float16).astype(np.float32)
    q8, s8 = _mx_on_gpu(q, d, f16, torch_dev)
    codes, E = oracle.q8_to_mx(q, d.astype(np.float32))
    assert np.array_equal(s8.astype(np.int32) - 127, E)
    bad = np.argwhere(q8 != codes)
    assert bad.size == 0, [(int(b), int(j), int(q[b, j]), float(d[b]), int(E[b]), int(q8[b, j]), int(codes[b, j]))
                           for b, j in bad[:6]]
    assert not (q8 & 0x7f == 0x7f).any()      # never NaN
    # the MXFP8 values stay within e4m3's relative step of the Q8 values
    v = oracle.mx_matrix(codes, E, nblk, 32)
    x = q.astype(np.float64) * d.astype(np.float64)[:, None]
    assert np.all(np.abs(v - x) <= 2.0 ** -4 * np.abs(x) + 2.0 ** -9 * np.ldexp(1.0, E)[:, None])


def _mx_operands(rng, rows, k, torch_dev, f16):
    x = rng.standard_normal((rows, k)).astype(np.float32) * rng.uniform(0.2, 3.0, (rows, 1)).astype(np.float32)
    q, d = quant_ref(x)
    q8, s8 = _mx_on_gpu(q.reshape(-1, 32), d.astype(np.float16) if f16 else d, f16, torch_dev)
    return dev(q8.reshape(rows, k), torch_dev), dev(s8, torch_dev), oracle.mx_matrix(q8, s8.astype(np.int32) - 127, rows, k)


@pytest.mark.parametrize("cfg", [-1, 0, 1, 2, 3, 4])
@pytest.mark.parametrize("m,n,k,epi", [(5, 128, 256, 0), (130, 192, 512, 0), (300, 256, 1024, 1), (64, 128, 2048, 2),
                                       (257, 384, 384, 1), (40, 64, 128, 0)])
def test_gemm_mx_vs_float64(torch_dev, cfg, m, n, k, epi):
    import torch
    from scipy.special import erf

    rng = np.random.default_rng(m + n + k)
    x8, xs, xa = _mx_operands(rng, m, k, torch_dev, False)
    w8, ws, wa = _mx_operands(rng, n, k, torch_dev, True)
    bias = rng.standard_normal(n).astype(np.float32) if epi != 1 else None
    res = rng.standard_normal((m, n)).astype(np.float32)
    y = dev(res, torch_dev) if epi == 1 else torch.zeros((m, n), dtype=torch.float32, device=torch_dev)
    bt = dev(bias, torch_dev) if bias is not None else None
    _lib.check(L().qasr_op_gemm_mx(ptr(x8), ptr(xs), m, ptr(w8), ptr(ws), n, k, ptr(bt), ptr(y) if epi == 1 else None,
                                   ptr(y), n, epi, None, None, cfg, None))
    got = host(y)
    ref = xa @ wa.T
    mag = np.abs(xa) @ np.abs(wa).T
    if bias is not None:
        ref = ref + bias
        mag = mag + np.abs(bias)
    if epi == 1:
        ref = ref + res
        mag = mag + np.abs(res)
    if epi == 2:
        ref = 0.5 * ref * (1 + erf(ref / np.sqrt(2)))
    err = np.abs(got - ref) / (mag + 1e-6)
    i = np.unravel_index(np.argmax(err), err.shape)
    assert err.max() <= 1e-4, (float(err.max()), i, float(got[i]), float(ref[i]), float(mag[i]))


@pytest.mark.parametrize("cfg", [0, 2])
def test_gemm_mx_swiglu_epilogue(torch_dev, cfg):
    """fused SwiGLU + Q8 epilogue on the MXFP8 GEMM (gate|up rows interleaved by 16, as the engine stores them)"""
    import torch

    from test_ops_gpu import _il16

    rng = np.random.default_rng(9)
    m, f, k = 70, 256, 512
    x8, xs, xa = _mx_operands(rng, m, k, torch_dev, False)
    w8, ws, wa = _mx_operands(rng, 2 * f, k, torch_dev, True)   # rows already in the interleaved order
    hq = empty((m, f), torch.int8, torch_dev)
    hd = empty((m, f // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_gemm_mx(ptr(x8), ptr(xs), m, ptr(w8), ptr(ws), 2 * f, k, None, None, None, 0, 3, ptr(hq),
                                   ptr(hd), cfg, None))
    gu = (xa @ wa.T)[:, _il16(f)]   # logical gate | up column r sits at physical column _il16(f)[r]
    g, u = gu[:, :f], gu[:, f:]
    h = (g / (1 + np.exp(-g)) * u).astype(np.float32)
    qr, dr = quant_ref(h)
    assert np.allclose(host(hd), dr, rtol=1e-3)
    assert (np.abs(host(hq).astype(int) - qr) <= 1).all()
