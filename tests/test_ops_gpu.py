"""Kernel-level parity: every qasr_op_* (HIP, through the C ABI) against the CPU oracle on seeded inputs.

Bars: integer/byte work bit-exact (activation int8 + scales, synthetic weights, argmax, exact-int GEMM);
fp32 math within the stated tolerances (sum-order differences only).
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from qasr import _lib

pytestmark = pytest.mark.gpu


def L():
    return _lib.load()


def dev(a, torch_dev):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).to(torch_dev)


def ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


def empty(shape, dtype, torch_dev):
    import torch

    return torch.empty(shape, dtype=dtype, device=torch_dev)


def q8_split(blocks, n, k):
    """GGUF Q8_0 blocks [N][K/32*34] → (qs int8 [N][K], sc f16-bits [N][K/32])"""
    b = blocks.reshape(n, k // 32, 34)
    sc = b[:, :, :2].copy().view(np.uint16).reshape(n, k // 32)
    qs = b[:, :, 2:].copy().view(np.int8).reshape(n, k)
    return qs, sc


def quant_ref(x):
    blocks = oracle.quantize_q8(x)
    m, k = x.shape
    qs, sc = q8_split(blocks, m, k)
    return qs, sc.view(np.float16).astype(np.float32)


@pytest.mark.parametrize("m,k", [(1, 32), (7, 256), (33, 2048)])
def test_quant_rows_bit_exact(torch_dev, m, k):
    import torch

    rng = np.random.default_rng(m * 1000 + k)
    x = (rng.standard_normal((m, k)) * rng.uniform(0.01, 100, size=(m, 1))).astype(np.float32)
    x[0, :32] = 0.0                           # all-zero block → d = 0, q = 0
    x[-1, -32:] = np.float32(127.0) * np.sign(rng.standard_normal(32)).astype(np.float32)  # amax exactly 127
    x[-1, -31] = np.float32(63.5)             # a .5 tie: roundf rounds away from zero
    xd = dev(x, torch_dev)
    q = empty((m, k), torch.int8, torch_dev)
    d = empty((m, k // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_quant_rows(ptr(xd), m, k, k, ptr(q), ptr(d), None))
    qr, dr = quant_ref(x)
    assert np.array_equal(host(q), qr)
    assert np.array_equal(host(d), dr)


def test_synth_q8_matches_oracle(torch_dev):
    import torch

    n, k = 96, 256
    qs = empty((n, k), torch.int8, torch_dev)
    sc = empty((n, k // 32), torch.float16, torch_dev)
    _lib.check(L().qasr_op_synth_q8(1234, b"blk.3.attn_q.weight", n, k, 0.02, ptr(qs), ptr(sc), None))
    ref = oracle.synth_q8(1234, "blk.3.attn_q.weight", n, k, 0.02)
    rq, rs = q8_split(ref, n, k)
    assert np.array_equal(host(qs), rq)
    assert np.array_equal(host(sc).view(np.uint16), rs)


def test_repack_q8(torch_dev):
    import torch

    n, k = 40, 128
    blocks = oracle.synth_q8(7, "x", n, k, 1.0)
    bd = dev(blocks.reshape(-1), torch_dev)
    qs = empty((n, k), torch.int8, torch_dev)
    sc = empty((n, k // 32), torch.float16, torch_dev)
    _lib.check(L().qasr_op_repack_q8(ptr(bd), n * k // 32, ptr(qs), ptr(sc), None))
    rq, rs = q8_split(blocks, n, k)
    assert np.array_equal(host(qs), rq)
    assert np.array_equal(host(sc).view(np.uint16), rs)


def _linear_case(torch_dev, m, n, k, path, epi, seed=0, exact=False, s4=False):
    """s4: register the regrouped stage scales (Q8Mat::sc4) of the weight matrix for this call, so the K-128 tiles
    stage their scales by 16-byte DMA (kernels_q8.hip k_gemm_q8d WS4)"""
    import torch

    rng = np.random.default_rng(seed)
    if exact:
        # every block's amax = 127 → d_x = 1, weights with d_w = 1: results are exact integers in any order
        x = rng.integers(-127, 128, size=(m, k)).astype(np.float32)
        x[:, ::32] = 127.0
        w = oracle.synth_q8(seed, "w", n, k, 1.0).reshape(n, k // 32, 34)
        w[:, :, 0:2] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)
        blocks = w.reshape(n, -1)
    else:
        x = rng.standard_normal((m, k)).astype(np.float32)
        blocks = oracle.synth_q8(seed, "w", n, k, 0.05)
    bias = rng.standard_normal(n).astype(np.float32) if epi != 1 and not exact else None
    res = rng.standard_normal((m, n)).astype(np.float32)
    oracle.set_mode(engine=True)
    ref = oracle.linear_q8(x, blocks, n, bias)
    if epi == 1:
        ref = ref + res
    elif epi == 2:
        from scipy.special import erf

        ref = 0.5 * ref * (1 + erf(ref / np.sqrt(2)))
    qs, sc = q8_split(blocks, n, k)
    xq = empty((m, k), torch.int8, torch_dev)
    xdd = empty((m, k // 32), torch.float32, torch_dev)
    xt = dev(x, torch_dev)
    _lib.check(L().qasr_op_quant_rows(ptr(xt), m, k, k, ptr(xq), ptr(xdd), None))
    wq, ws = dev(qs, torch_dev), dev(sc, torch_dev)
    bt = dev(bias, torch_dev) if bias is not None else None
    y = dev(res, torch_dev) if epi == 1 else empty((m, n), torch.float32, torch_dev)
    s4t = None
    if s4:
        s4t = empty((n, k // 32), torch.float16, torch_dev)
        _lib.check(L().qasr_op_stage_scales(ptr(ws), n, k, ptr(s4t), None))
        _lib.check(L().qasr_op_register_stage_scales(ptr(ws), n, k, ptr(s4t)))
    try:
        _lib.check(L().qasr_op_linear_q8(ptr(xq), ptr(xdd), m, ptr(wq), ptr(ws), n, k, ptr(bt),
                                         ptr(y) if epi == 1 else None, ptr(y), n, epi, path, None))
        out = host(y)
    finally:
        if s4:
            _lib.check(L().qasr_op_register_stage_scales(ptr(ws), n, k, None))
    return out, ref.astype(np.float32)


# path: 1 GEMV, 2 auto, 16 + cfg (+ 32·splits) forces a GEMM configuration (kernels_q8.hip kGemmCfgs: 0..3 register-
# staged, 4..23 LDS-DMA, 24..30 the decode kernel with K split over waves; a configuration whose K granule does not
# divide K falls back to the heuristic)
GEMM_PATHS = ([1, 2, 3, 4, 5] + [16 + c for c in range(31)] + [16 + 4 + 32 * 2, 16 + 9 + 32 * 4, 16 + 10 + 32 * 3,
                                                                 16 + 16 + 32, 16 + 21 + 32])


@pytest.mark.parametrize("path", GEMM_PATHS)
@pytest.mark.parametrize("m,n,k", [(1, 64, 1024), (3, 130, 512), (8, 64, 1024), (9, 70, 96), (64, 128, 1024),
                                   (100, 192, 512), (32, 2048, 2048), (300, 2048, 1024), (33, 96, 160)])
def test_linear_q8_exact_integer(torch_dev, path, m, n, k):
    if path in (1, 3, 4, 5) and m > 8:
        pytest.skip("GEMV path is M<=8")
    y, ref = _linear_case(torch_dev, m, n, k, path, 0, seed=m + n, exact=True)
    assert np.array_equal(y, ref)


@pytest.mark.parametrize("path", GEMM_PATHS)
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("m,n,k", [(1, 2048, 2048), (5, 256, 6144), (37, 320, 2048), (130, 1024, 1024),
                                   (24, 2048, 6144), (257, 2048, 2048)])
def test_linear_q8_vs_oracle(torch_dev, path, epi, m, n, k):
    if path in (1, 3, 4, 5) and m > 8:
        pytest.skip("GEMV path is M<=8")
    y, ref = _linear_case(torch_dev, m, n, k, path, epi, seed=k + epi)
    scale = np.abs(ref).max() + 1e-6
    assert np.abs(y - ref).max() <= 2e-5 * scale * np.sqrt(k / 256)


@pytest.mark.parametrize("cfg", [-1, 0, 2, 4, 5, 10, 14, 17, 23, 25, 27, 29, 30])
@pytest.mark.parametrize("m,n,k", [(37, 320, 2048), (300, 1024, 1024), (9, 64, 96), (70, 256, 2048)])
def test_linear_fused_epilogues(torch_dev, m, n, k, cfg):
    """GELU + Q8 quantisation (encoder up-projection, projector) and f16 store (encoder QKV) in the GEMM epilogue"""
    import torch
    from scipy.special import erf

    rng = np.random.default_rng(m + n + k)
    x = rng.standard_normal((m, k)).astype(np.float32)
    blocks = oracle.synth_q8(k, "w", n, k, 0.05)
    bias = rng.standard_normal(n).astype(np.float32)
    oracle.set_mode(engine=True)
    ref = oracle.linear_q8(x, blocks, n, bias).astype(np.float64)
    g = (0.5 * ref * (1 + erf(ref / np.sqrt(2)))).astype(np.float32)
    qr, dr = quant_ref(g)
    qs, sc = q8_split(blocks, n, k)
    xq = empty((m, k), torch.int8, torch_dev)
    xdd = empty((m, k // 32), torch.float32, torch_dev)
    keep = [dev(a, torch_dev) for a in (x, qs, sc, bias)]
    _lib.check(L().qasr_op_quant_rows(ptr(keep[0]), m, k, k, ptr(xq), ptr(xdd), None))
    hq = empty((m, n), torch.int8, torch_dev)
    hd = empty((m, n // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_linear_q8_ex(ptr(xq), ptr(xdd), m, ptr(keep[1]), ptr(keep[2]), n, k, ptr(keep[3]), None, n,
                                        4, ptr(hq), ptr(hd), cfg, None))
    assert np.allclose(host(hd), dr, rtol=2e-3)
    assert (np.abs(host(hq).astype(int) - qr) <= 1).all() and (host(hq) != qr).mean() < 1e-2
    yh = empty((m, n + 8), torch.float16, torch_dev)
    _lib.check(L().qasr_op_linear_q8_ex(ptr(xq), ptr(xdd), m, ptr(keep[1]), ptr(keep[2]), n, k, ptr(keep[3]), ptr(yh),
                                        n + 8, 5, None, None, cfg, None))
    y = host(yh)[:, :n].astype(np.float32)
    assert np.abs(y - ref).max() <= 1e-3 * np.abs(ref).max() + 2e-5 * np.abs(ref).max() * np.sqrt(k / 256)


@pytest.mark.parametrize("m,h", [(9, 2048), (256, 1024), (5, 896), (3000, 2048)])
def test_rmsnorm_q8(torch_dev, m, h):
    """workgroup-per-row kernel (M <= 2048) and wave-per-row kernel (larger M)"""
    import torch

    rng = np.random.default_rng(3)
    x = (rng.standard_normal((m, h)) * 3).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(h)).astype(np.float32)
    xt, wt = dev(x, torch_dev), dev(w, torch_dev)
    q = empty((m, h), torch.int8, torch_dev)
    d = empty((m, h // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_rmsnorm_q8(ptr(xt), m, h, ptr(wt), 1e-6, ptr(q), ptr(d), None))
    y = x / np.sqrt((x.astype(np.float64) ** 2).mean(1, keepdims=True) + 1e-6) * w
    qr, dr = quant_ref(y.astype(np.float32))
    qh, dh = host(q), host(d)
    # the block scale is stored as f16: a 1-ulp f32 difference in the row norm can flip its f16 rounding (one f16
    # ulp, 2^-10 relative) — allowed on a small fraction of blocks
    assert np.allclose(dh, dr, rtol=1.5e-3) and np.isclose(dh, dr, rtol=1e-5).mean() > 0.99
    assert (np.abs(qh.astype(int) - qr) <= 1).all() and (qh != qr).mean() < 1e-2


def test_layernorm_q8(torch_dev):
    import torch

    rng = np.random.default_rng(4)
    m, h = 5, 1024
    x = (rng.standard_normal((m, h)) * 2 + 0.5).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(h)).astype(np.float32)
    b = (0.1 * rng.standard_normal(h)).astype(np.float32)
    xt, wt, bt = dev(x, torch_dev), dev(w, torch_dev), dev(b, torch_dev)
    q = empty((m, h), torch.int8, torch_dev)
    d = empty((m, h // 32), torch.float32, torch_dev)
    y = empty((m, h), torch.float32, torch_dev)
    _lib.check(L().qasr_op_layernorm_q8(ptr(xt), m, h, ptr(wt), ptr(bt), 1e-5, ptr(q), ptr(d), ptr(y), None))
    x64 = x.astype(np.float64)
    ref = (x64 - x64.mean(1, keepdims=True)) / np.sqrt(x64.var(1, keepdims=True) + 1e-5) * w + b
    assert np.abs(host(y) - ref).max() < 1e-5 * np.abs(ref).max()


def _il16(f):
    """physical row of each logical gate|up row after qasr_op_interleave_gate_up"""
    r = np.arange(2 * f)
    return np.where(r < f, 32 * (r // 16) + r % 16, 32 * ((r - f) // 16) + 16 + (r - f) % 16)


@pytest.mark.parametrize("cfg,s4", [(c, False) for c in (-1, 1, 4, 5, 8, 9, 12, 13, 15, 20, 22, 23, 28, 29, 30)] +
                         [(4096 + c, True) for c in (8, 12, 15, 23, 33, 35, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47,
                                                     48)])
@pytest.mark.parametrize("m,f,k", [(3, 256, 512), (40, 512, 1024), (300, 1024, 512), (70, 512, 2048)])
def test_gemm_swiglu_q8(torch_dev, m, f, k, cfg, s4):
    """fused gate-up GEMM + SwiGLU + Q8 epilogue vs the oracle's linear_q8 of gate and up (s4: the K-128 tiles with
    the regrouped stage scales, including the 16-wave and 128-row decode tiles of round 4)"""
    import torch

    rng = np.random.default_rng(m + f)
    x = rng.standard_normal((m, k)).astype(np.float32)
    blocks = oracle.synth_q8(7, "gu", 2 * f, k, 0.05)
    oracle.set_mode(engine=True)
    gu = oracle.linear_q8(x, blocks, 2 * f, None)
    g, u = gu[:, :f], gu[:, f:]
    yref = (g / (1 + np.exp(-g)) * u).astype(np.float32)
    qr, dr = quant_ref(yref)
    qs, sc = q8_split(blocks, 2 * f, k)
    wq, ws = dev(qs, torch_dev), dev(sc, torch_dev)
    _lib.check(L().qasr_op_interleave_gate_up(ptr(wq), ptr(ws), 2 * f, k, None))
    assert np.array_equal(host(wq)[_il16(f)], qs)
    xq = empty((m, k), torch.int8, torch_dev)
    xdd = empty((m, k // 32), torch.float32, torch_dev)
    xt = dev(x, torch_dev)
    _lib.check(L().qasr_op_quant_rows(ptr(xt), m, k, k, ptr(xq), ptr(xdd), None))
    hq = empty((m, f), torch.int8, torch_dev)
    hd = empty((m, f // 32), torch.float32, torch_dev)
    s4t = None
    if s4:
        s4t = empty((2 * f, k // 32), torch.float16, torch_dev)
        _lib.check(L().qasr_op_stage_scales(ptr(ws), 2 * f, k, ptr(s4t), None))
        _lib.check(L().qasr_op_register_stage_scales(ptr(ws), 2 * f, k, ptr(s4t)))
    try:
        _lib.check(L().qasr_op_gemm_swiglu_q8_cfg(ptr(xq), ptr(xdd), m, ptr(wq), ptr(ws), 2 * f, k, ptr(hq), ptr(hd),
                                                  cfg, None))
        torch.cuda.synchronize()
    finally:
        if s4:
            _lib.check(L().qasr_op_register_stage_scales(ptr(ws), 2 * f, k, None))
    assert np.allclose(host(hd), dr, rtol=2e-3)
    assert (np.abs(host(hq).astype(int) - qr) <= 1).all()
    # the unfused path (GEMV rows) on the interleaved layout
    gut = dev(gu[:, np.argsort(_il16(f))], torch_dev)
    q2 = empty((m, f), torch.int8, torch_dev)
    d2 = empty((m, f // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_swiglu_q8_interleaved(ptr(gut), m, f, ptr(q2), ptr(d2), None))
    assert np.allclose(host(d2), dr, rtol=1e-5)
    assert (np.abs(host(q2).astype(int) - qr) <= 1).all()


def _q8_weights(torch_dev, n, k, seed):
    qs, sc = q8_split(oracle.synth_q8(seed, "gv", n, k, 0.05), n, k)
    return dev(qs, torch_dev), dev(sc, torch_dev)


@pytest.mark.parametrize("m,n,k,epi", [(1, 4096, 2048, 0), (1, 2048, 1024, 1), (2, 12288, 2048, 0),
                                       (4, 6144, 1024, 1), (1, 40000, 1024, 0), (3, 512, 4096, 0),
                                       (1, 384, 256, 1), (2, 100, 896, 0), (8, 4096, 2048, 0), (6, 2048, 1024, 1)])
def test_gemv_fused_rms(torch_dev, m, n, k, epi):
    """norm-in-prologue GEMV == rmsnorm_q8 then the GEMV, bit for bit (the decode fusion's parity contract)"""
    import torch

    rng = np.random.default_rng(11)
    x = dev((rng.standard_normal((m, k)) * 3).astype(np.float32), torch_dev)
    w = dev((1 + 0.1 * rng.standard_normal(k)).astype(np.float32), torch_dev)
    res = dev(rng.standard_normal((m, n)).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, n, k, 3)
    q = empty((m, k), torch.int8, torch_dev)
    d = empty((m, k // 32), torch.float32, torch_dev)
    y0, y1 = res.clone(), res.clone()
    _lib.check(L().qasr_op_rmsnorm_q8(ptr(x), m, k, ptr(w), 1e-6, ptr(q), ptr(d), None))
    _lib.check(L().qasr_op_linear_q8(ptr(q), ptr(d), m, ptr(wq), ptr(ws), n, k, None, ptr(y0), ptr(y0), n, epi, 1,
                                     None))
    _lib.check(L().qasr_op_gemv_fused(1, ptr(x), k, ptr(w), 1e-6, m, None, None, ptr(wq), ptr(ws), n, k, ptr(y1),
                                      ptr(y1), n, epi, None, None, None))
    assert np.array_equal(host(y0), host(y1))


@pytest.mark.parametrize("m,n,k,epi", [(1, 2048, 6144, 1), (8, 2048, 6144, 1), (7, 2048, 2048, 0), (4, 1024, 3072, 1), (1, 2048, 2048, 1), (2, 1024, 2048, 0),
                                       (3, 4096, 5120, 1), (1, 300, 96, 0)])
def test_gemv_fused_q8_rows(torch_dev, m, n, k, epi):
    """the per-CU GEMV on given Q8 rows (O / down projections) == gemv_q8, bit for bit"""
    import torch

    rng = np.random.default_rng(13)
    xq = dev(rng.integers(-127, 128, (m, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((m, k // 32)) * 0.02).astype(np.float32), torch_dev)
    res = dev(rng.standard_normal((m, n)).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, n, k, 5)
    y0, y1 = res.clone(), res.clone()
    _lib.check(L().qasr_op_linear_q8(ptr(xq), ptr(xd), m, ptr(wq), ptr(ws), n, k, None, ptr(y0), ptr(y0), n, epi, 1,
                                     None))
    _lib.check(L().qasr_op_gemv_fused(0, None, 0, None, 0.0, m, ptr(xq), ptr(xd), ptr(wq), ptr(ws), n, k, ptr(y1),
                                      ptr(y1), n, epi, None, None, None))
    assert np.array_equal(host(y0), host(y1))


@pytest.mark.parametrize("m,f,k", [(1, 6144, 2048), (4, 3072, 1024), (2, 256, 256), (3, 512, 4096), (8, 6144, 2048),
                                   (5, 3072, 1024)])
def test_gemv_fused_swiglu(torch_dev, m, f, k):
    """norm + interleaved gate/up GEMV + SwiGLU + Q8 in one launch == rmsnorm_q8, the GEMV into f32 gate/up rows and
    swiglu_q8 (interleaved), bit for bit"""
    import torch

    rng = np.random.default_rng(12)
    x = dev((rng.standard_normal((m, k)) * 3).astype(np.float32), torch_dev)
    w = dev((1 + 0.1 * rng.standard_normal(k)).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, 2 * f, k, 4)
    _lib.check(L().qasr_op_interleave_gate_up(ptr(wq), ptr(ws), 2 * f, k, None))
    q = empty((m, k), torch.int8, torch_dev)
    d = empty((m, k // 32), torch.float32, torch_dev)
    gu = empty((m, 2 * f), torch.float32, torch_dev)
    h0, hd0 = empty((m, f), torch.int8, torch_dev), empty((m, f // 32), torch.float32, torch_dev)
    h1, hd1 = empty((m, f), torch.int8, torch_dev), empty((m, f // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_rmsnorm_q8(ptr(x), m, k, ptr(w), 1e-6, ptr(q), ptr(d), None))
    _lib.check(L().qasr_op_linear_q8(ptr(q), ptr(d), m, ptr(wq), ptr(ws), 2 * f, k, None, None, ptr(gu), 2 * f, 0, 1,
                                     None))
    _lib.check(L().qasr_op_swiglu_q8_interleaved(ptr(gu), m, f, ptr(h0), ptr(hd0), None))
    _lib.check(L().qasr_op_gemv_fused(1, ptr(x), k, ptr(w), 1e-6, m, None, None, ptr(wq), ptr(ws), 2 * f, k, None,
                                      None, 0, 3, ptr(h1), ptr(hd1), None))
    assert np.array_equal(host(h0), host(h1)) and np.array_equal(host(hd0), host(hd1))


def test_gemv_fused_rejects_bad_shapes(torch_dev):
    import torch

    x = empty((8, 8192), torch.float32, torch_dev)
    y = empty((8, 64), torch.float32, torch_dev)
    for pro, m, k, epi in ((1, 33, 1024, 0), (0, 33, 1024, 0), (1, 1, 8192, 0), (0, 1, 8192, 0), (3, 1, 1024, 0),
                           (1, 1, 100, 0), (0, 1, 1024, 3)):
        with pytest.raises(_lib.QasrError):
            _lib.check(L().qasr_op_gemv_fused(pro, ptr(x), 2 * k, ptr(x), 1e-6, m, ptr(x), ptr(x), ptr(x), ptr(x), 64,
                                              k, None, ptr(y), 64, epi, ptr(x), ptr(x), None))


@pytest.mark.parametrize("pro,n,k,epi", [(1, 4096, 2048, 0), (0, 2048, 2048, 1), (0, 2048, 6144, 1),
                                         (0, 151936, 2048, 0), (1, 12288, 2048, 3), (1, 1024, 1024, 1)])
def test_gemv_exact_rows(torch_dev, pro, n, k, epi):
    """exact-row contract of the draft verify passes (engine.cpp): every row of a 2–32-row gemv_fused launch (rows in
    groups of 8 against the weights held in registers) is the same bits as that row in a 1-row launch; for given Q8
    rows also the same bits as gemv_q8's single row (the 1-row decode step's vocabulary projection)"""
    import torch

    rng = np.random.default_rng(21)
    M = 32
    x = dev((rng.standard_normal((M, k)) * 3).astype(np.float32), torch_dev)
    w = dev((1 + 0.1 * rng.standard_normal(k)).astype(np.float32), torch_dev)
    xq = dev(rng.integers(-127, 128, (M, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((M, k // 32)) * 0.02).astype(np.float32), torch_dev)
    res = dev(rng.standard_normal((M, n)).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, n, k, 6)
    f = n // 2

    def launch(rows, r0):
        y = res[r0:r0 + rows].clone()
        h = empty((rows, f), torch.int8, torch_dev) if epi == 3 else None
        hd = empty((rows, f // 32), torch.float32, torch_dev) if epi == 3 else None
        yp = None if epi == 3 else ptr(y)
        if pro == 1:
            _lib.check(L().qasr_op_gemv_fused(1, C.c_void_p(x.data_ptr() + r0 * k * 4), k, ptr(w), 1e-6, rows, None,
                                              None, ptr(wq), ptr(ws), n, k, yp, yp, n, epi, ptr(h), ptr(hd), None))
        else:
            _lib.check(L().qasr_op_gemv_fused(0, None, 0, None, 0.0, rows, C.c_void_p(xq.data_ptr() + r0 * k),
                                              C.c_void_p(xd.data_ptr() + r0 * (k // 32) * 4), ptr(wq), ptr(ws), n, k,
                                              yp, yp, n, epi, None, None, None))
        return (host(h), host(hd)) if epi == 3 else host(y)

    single = [launch(1, r) for r in range(M)]
    for rows in (2, 5, 8, 9, 16, 23, 32):
        got = launch(rows, 0)
        for r in range(rows):
            if epi == 3:
                assert np.array_equal(got[0][r], single[r][0][0]) and np.array_equal(got[1][r], single[r][1][0]), (rows, r)
            else:
                assert np.array_equal(got[r], single[r][0]), (rows, r)
    if pro == 0:
        for r in (0, 17, 31):
            y = res[r:r + 1].clone()
            _lib.check(L().qasr_op_linear_q8(C.c_void_p(xq.data_ptr() + r * k),
                                             C.c_void_p(xd.data_ptr() + r * (k // 32) * 4), 1, ptr(wq), ptr(ws), n, k,
                                             None, ptr(y), ptr(y), n, epi, 1, None))
            assert np.array_equal(host(y)[0], single[r][0]), r


GEMM_CHAIN_CFGS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 16, 17, 18, 21, 22, 23, 36, 37]


@pytest.mark.parametrize("m,f,k", [(300, 1024, 1024), (520, 3072, 2048)])
def test_gemm_swiglu_stable_tiles_bit_identical(torch_dev, m, f, k):
    """the row-count-independent order's SwiGLU tile above 256 rows (stable_pick: cfg 4, 128×128 with 64-column wave
    tiles, K-64 stages) gives the bits of cfg 13 (128×64, 4×1 waves, K-128 stages) and cfg 12 — each output one block
    chain in K order, the SwiGLU + Q8 epilogue per 64-column wave tile (every prefill of round 5 runs this order)"""
    import torch

    rng = np.random.default_rng(m + 3 * f)
    x = rng.standard_normal((m, k)).astype(np.float32)
    qs, sc = q8_split(oracle.synth_q8(11, "gu", 2 * f, k, 0.05), 2 * f, k)
    wq, ws = dev(qs, torch_dev), dev(sc, torch_dev)
    _lib.check(L().qasr_op_interleave_gate_up(ptr(wq), ptr(ws), 2 * f, k, None))
    xq = empty((m, k), torch.int8, torch_dev)
    xdd = empty((m, k // 32), torch.float32, torch_dev)
    xt = dev(x, torch_dev)
    _lib.check(L().qasr_op_quant_rows(ptr(xt), m, k, k, ptr(xq), ptr(xdd), None))
    outs = []
    for cfg in (4, 13, 12):
        hq = empty((m, f), torch.int8, torch_dev)
        hd = empty((m, f // 32), torch.float32, torch_dev)
        _lib.check(L().qasr_op_gemm_swiglu_q8_cfg(ptr(xq), ptr(xdd), m, ptr(wq), ptr(ws), 2 * f, k, ptr(hq), ptr(hd),
                                                  cfg, None))
        torch.cuda.synchronize()
        outs.append((host(hq), host(hd)))
    for hq, hd in outs[1:]:
        assert np.array_equal(hq, outs[0][0]) and np.array_equal(hd.view(np.uint32), outs[0][1].view(np.uint32))


@pytest.mark.parametrize("m,n,k,epi", [(13, 1024, 1024, 0), (104, 3072, 1024, 0), (160, 1024, 4096, 1),
                                       (300, 4096, 1024, 0), (7, 2048, 2048, 1)])
def test_gemm_chain_configs_bit_identical(torch_dev, m, n, k, epi):
    """the stable GEMM order (StableOrderScope: single-utterance encoder runs, the encoder cache): every one-K-group,
    unsplit configuration computes each output as the same fma chain over its K blocks, so all of them — any tile
    shape, any row count — give the same bits; a row subset gives the rows' bits of the full launch"""
    rng = np.random.default_rng(22)
    xq = dev(rng.integers(-127, 128, (m, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((m, k // 32)) * 0.02).astype(np.float32), torch_dev)
    res = dev(rng.standard_normal((m, n)).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, n, k, 7)

    def run(cfg, rows=m):
        y = res[:rows].clone()
        path = 16 + cfg + 32 if cfg < 31 else 4096 + cfg + 256
        _lib.check(L().qasr_op_linear_q8(ptr(xq), ptr(xd), rows, ptr(wq), ptr(ws), n, k, None, ptr(y), ptr(y), n,
                                         epi, path, None))
        return host(y)

    want = run(10)
    for cfg in GEMM_CHAIN_CFGS:
        assert np.array_equal(run(cfg), want), cfg
    for cfg in (10, 16, 4):
        assert np.array_equal(run(cfg, rows=max(1, m // 3)), want[:max(1, m // 3)]), cfg


@pytest.mark.parametrize("m", [1, 4, 40])
def test_swiglu_q8(torch_dev, m):
    """lane-per-element kernel (M <= 16) and thread-per-block kernel (larger M)"""
    import torch

    rng = np.random.default_rng(5)
    f = 512
    gu = rng.standard_normal((m, 2 * f)).astype(np.float32) * 3
    gt = dev(gu, torch_dev)
    q = empty((m, f), torch.int8, torch_dev)
    d = empty((m, f // 32), torch.float32, torch_dev)
    _lib.check(L().qasr_op_swiglu_q8(ptr(gt), m, f, ptr(q), ptr(d), None))
    g, u = gu[:, :f], gu[:, f:]
    y = (g / (1 + np.exp(-g)) * u).astype(np.float32)
    qr, dr = quant_ref(y)
    assert np.allclose(host(d), dr, rtol=1e-5)
    assert (np.abs(host(q).astype(int) - qr) <= 1).all()


@pytest.mark.parametrize("nh,nkv,hd", [(4, 2, 128), (16, 8, 128), (4, 4, 64)])
def test_qk_norm_rope(torch_dev, nh, nkv, hd):
    """row-per-workgroup kernel (hd 128) and head-per-wave kernel (hd 64)"""
    import torch

    rng = np.random.default_rng(6)
    rows = 3
    qkv = rng.standard_normal((rows, (nh + 2 * nkv) * hd)).astype(np.float32)
    pos = np.array([0, 5, 77], np.int32)
    slot = np.array([2, 0, 1], np.int32)
    qnw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    knw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    tab = np.empty((128, hd // 2, 2), np.float32)
    _lib.check(L().qasr_op_rope_table(128, hd, 1e6, tab.ctypes.data_as(C.c_void_p)))
    qo = empty((rows, nh * hd), torch.float16, torch_dev)
    kc = torch.zeros((4, nkv * hd), dtype=torch.float16, device=torch_dev)
    vc = torch.zeros((4, nkv * hd), dtype=torch.float16, device=torch_dev)
    # keep every device tensor referenced until the kernel has finished (a temporary would be freed and its
    # block reused by the next allocation while the launch still reads it)
    keep = [dev(a, torch_dev) for a in (qkv, pos, slot, qnw, knw, tab)]
    _lib.check(L().qasr_op_qk_norm_rope(ptr(keep[0]), rows, nh, nkv, hd, ptr(keep[1]), ptr(keep[2]), ptr(keep[3]),
                                        ptr(keep[4]), ptr(keep[5]), 1e-6, ptr(qo), ptr(kc), ptr(vc), None))

    def norm_rope(v, w, p):
        v = v / np.sqrt((v.astype(np.float64) ** 2).mean() + 1e-6) * w
        c, s = tab[p, :, 0], tab[p, :, 1]
        a, b = v[: hd // 2], v[hd // 2:]
        return np.concatenate([a * c - b * s, b * c + a * s])

    qh, kh, vh = host(qo).astype(np.float32), host(kc).astype(np.float32), host(vc).astype(np.float32)
    for r in range(rows):
        for h in range(nh):
            ref = norm_rope(qkv[r, h * hd:(h + 1) * hd], qnw, pos[r])
            assert np.abs(qh[r, h * hd:(h + 1) * hd] - ref).max() < 2e-3 * np.abs(ref).max()
        for h in range(nkv):
            ref = norm_rope(qkv[r, (nh + h) * hd:(nh + h + 1) * hd], knw, pos[r])
            assert np.abs(kh[slot[r], h * hd:(h + 1) * hd] - ref).max() < 2e-3 * np.abs(ref).max()
            vref = qkv[r, (nh + nkv + h) * hd:(nh + nkv + h + 1) * hd]
            assert np.abs(vh[slot[r], h * hd:(h + 1) * hd] - vref).max() < 2e-3 * np.abs(vref).max()


@pytest.mark.parametrize("nh,nkv,rows", [(16, 8, 5), (16, 4, 5), (16, 8, 200), (16, 4, 200)])
def test_attention_decode_fused(torch_dev, nh, nkv, rows):
    """decode attention with the q/k norm + RoPE + KV write fused in == qk_norm_rope then attention, bit for bit
    (Q8 output rows and both caches), over short and long key ranges; 200 rows take both kernels' 32-key-chunk
    form (≥ 192 rows)"""
    import torch

    hd = 128
    rng = np.random.default_rng(11)
    lens = np.resize(np.array([1, 7, 40, 130, 300], np.int32), rows)
    starts = np.concatenate([[3], 3 + np.cumsum(lens[:-1] + 2)]).astype(np.int32)
    slots = int(starts[-1] + lens[-1] + 4)
    qkv = rng.standard_normal((rows, (nh + 2 * nkv) * hd)).astype(np.float32)
    pos = (lens - 1).astype(np.int32)
    slot = (starts + lens - 1).astype(np.int32)
    qnw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    knw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    tab = np.empty((512, hd // 2, 2), np.float32)
    _lib.check(L().qasr_op_rope_table(512, hd, 1e6, tab.ctypes.data_as(C.c_void_p)))
    kc0 = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    vc0 = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    keep = [dev(a, torch_dev) for a in (qkv, pos, slot, qnw, knw, tab, starts, lens)]
    scale = 1.0 / np.sqrt(hd)
    outs = []
    for fused in (False, True):
        kc, vc = dev(kc0, torch_dev), dev(vc0, torch_dev)
        oq = torch.zeros((rows, nh * hd), dtype=torch.int8, device=torch_dev)
        od = torch.zeros((rows, nh * hd // 32), dtype=torch.float32, device=torch_dev)
        if fused:
            _lib.check(L().qasr_op_attention_decode_fused(ptr(keep[0]), rows, nh, nkv, hd, ptr(keep[1]), ptr(keep[2]),
                                                          ptr(keep[3]), ptr(keep[4]), ptr(keep[5]), 1e-6, ptr(kc),
                                                          ptr(vc), ptr(keep[6]), ptr(keep[7]), scale, ptr(oq),
                                                          ptr(od), None))
        else:
            qo = torch.zeros((rows, nh * hd), dtype=torch.float16, device=torch_dev)
            _lib.check(L().qasr_op_qk_norm_rope(ptr(keep[0]), rows, nh, nkv, hd, ptr(keep[1]), ptr(keep[2]),
                                                ptr(keep[3]), ptr(keep[4]), ptr(keep[5]), 1e-6, ptr(qo), ptr(kc),
                                                ptr(vc), None))
            _lib.check(L().qasr_op_attention(ptr(qo), nh * hd, ptr(kc), ptr(vc), nkv * hd, ptr(keep[6]),
                                             ptr(keep[7]), rows, nh, nkv, hd, scale, None, ptr(oq), ptr(od), None))
        torch.cuda.synchronize()
        outs.append([host(t) for t in (oq, od, kc, vc)])
    for name, a, b in zip(("oq", "od", "kc", "vc"), *outs):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"{name}: {len(bad)} differ, first {bad[:4].tolist()}"
    assert not np.array_equal(outs[1][2], kc0)   # the new K rows were written


@pytest.mark.parametrize("nh,nkv", [(16, 8), (16, 4)])
def test_attention_decode_split(torch_dev, nh, nkv):
    """≤ 4 decode rows over long key ranges split over workgroups (flash-decoding, pieces merged by the last to
    arrive): the same K/V cache writes as one workgroup per row, outputs within f32 merge-order noise of it and of an
    f64 reference, deterministic, arrival counters left zero"""
    import torch

    hd, rows = 128, 4
    rng = np.random.default_rng(21)
    lens = np.array([1, 700, 1500, 4000], np.int32)
    starts = np.concatenate([[2], 2 + np.cumsum(lens[:-1] + 3)]).astype(np.int32)
    slots = int(starts[-1] + lens[-1] + 4)
    qkv = rng.standard_normal((rows, (nh + 2 * nkv) * hd)).astype(np.float32)
    pos = (lens - 1).astype(np.int32)
    slot = (starts + lens - 1).astype(np.int32)
    qnw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    knw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    tab = np.empty((4096, hd // 2, 2), np.float32)
    _lib.check(L().qasr_op_rope_table(4096, hd, 1e6, tab.ctypes.data_as(C.c_void_p)))
    kc0 = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    vc0 = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    keep = [dev(a, torch_dev) for a in (qkv, pos, slot, qnw, knw, tab, starts, lens)]
    scale = 1.0 / np.sqrt(hd)
    G = nh // nkv
    part = torch.empty(4 * nkv * 16 * G * 130, dtype=torch.float32, device=torch_dev)
    cnt = torch.zeros(4 * nkv, dtype=torch.int32, device=torch_dev)
    outs = []
    for split in (False, True, True):
        kc, vc = dev(kc0, torch_dev), dev(vc0, torch_dev)
        oq = torch.zeros((rows, nh * hd), dtype=torch.int8, device=torch_dev)
        od = torch.zeros((rows, nh * hd // 32), dtype=torch.float32, device=torch_dev)
        args = (ptr(keep[0]), rows, nh, nkv, hd, ptr(keep[1]), ptr(keep[2]), ptr(keep[3]), ptr(keep[4]), ptr(keep[5]),
                1e-6, ptr(kc), ptr(vc), ptr(keep[6]), ptr(keep[7]), scale, ptr(oq), ptr(od))
        if split:
            _lib.check(L().qasr_op_attention_decode_split(*args, ptr(part), ptr(cnt), None))
        else:
            _lib.check(L().qasr_op_attention_decode_fused(*args, None))
        outs.append([host(t) for t in (oq, od, kc, vc)])
    assert not host(cnt).any()
    one, sp, sp2 = outs
    assert all(np.array_equal(a, b) for a, b in zip(sp, sp2))            # deterministic
    assert np.array_equal(one[2], sp[2]) and np.array_equal(one[3], sp[3])   # the same cache writes
    assert np.array_equal(one[0][0], sp[0][0])   # the 1-key row is not split: bit-identical
    deq = lambda o: o[0].astype(np.float64) * np.repeat(o[1], 32, axis=1)
    # reference: f64 attention of the f16-rounded q over the written caches (q from the unsplit kernel's own
    # norm/RoPE is not exported, so compare the two kernels' dequantised outputs to each other at the Q8 grain)
    step = np.repeat(np.maximum(one[1], sp[1]), 32, axis=1)
    assert (np.abs(deq(one) - deq(sp)) <= 1.01 * step + 1e-6).all()
    assert (one[0] != sp[0]).mean() < 0.05


def _attention_case(torch_dev, hd, nh, nkv, starts, lens, dense, seed):
    import torch

    rng = np.random.default_rng(seed)
    slots = int(max(s + n for s, n in zip(starts, lens))) + 5
    k = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    v = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    starts, lens = np.asarray(starts, np.int32), np.asarray(lens, np.int32)
    rows = len(starts)
    q = rng.standard_normal((rows, nh * hd)).astype(np.float16)
    o = empty((rows, nh * hd), torch.float32, torch_dev)
    oq = empty((rows, nh * hd), torch.int8, torch_dev)
    od = empty((rows, nh * hd // 32), torch.float32, torch_dev)
    scale = 1 / np.sqrt(hd)
    keep = [dev(a, torch_dev) for a in (q, k, v, starts, lens)]
    _lib.check(L().qasr_op_attention_dense(ptr(keep[0]), nh * hd, ptr(keep[1]), ptr(keep[2]), nkv * hd,
                                           ptr(keep[3]), ptr(keep[4]), rows, nh, nkv, hd, scale, ptr(o), ptr(oq),
                                           ptr(od), int(dense), None))
    oh = host(o)
    ref = np.zeros((rows, nh * hd), np.float64)
    for r in range(rows):
        for h in range(nh):
            g = h // (nh // nkv)
            kk = k[starts[r]:starts[r] + lens[r], g * hd:(g + 1) * hd].astype(np.float64)
            vv = v[starts[r]:starts[r] + lens[r], g * hd:(g + 1) * hd].astype(np.float64)
            s = kk @ q[r, h * hd:(h + 1) * hd].astype(np.float64) * scale
            p = np.exp(s - s.max())
            ref[r, h * hd:(h + 1) * hd] = p @ vv / p.sum()
    # MFMA tile kernel (dense rows, 1 or 2 query heads per KV head): P rounded to f16 before P·V (relative 2^-11 per
    # weight); the f32 per-row kernel (decode rows, other group sizes): 1e-4
    tile = dense and (nh // nkv) in (1, 2)
    assert np.abs(oh - ref).max() < (4e-3 if tile else 1e-4)
    qr, dr = quant_ref(oh.astype(np.float32))
    assert np.array_equal(host(oq), qr) and np.array_equal(host(od), dr)


@pytest.mark.parametrize("dense", [False, True])
@pytest.mark.parametrize("hd,nh,nkv", [(128, 4, 2), (64, 3, 3), (128, 16, 8), (64, 2, 2), (128, 8, 2)])
def test_attention(torch_dev, hd, nh, nkv, dense):
    """ragged per-row ranges (incl. a 1-key row) on both kernels"""
    _attention_case(torch_dev, hd, nh, nkv, [0, 10, 100, 0, 300], [1, 57, 300, 513, 104], dense, hd + nh)


@pytest.mark.parametrize("nh,nkv", [(16, 8), (16, 4)])
def test_attention_decode_many_rows(torch_dev, nh, nkv):
    """≥ 192 decode rows take the 32-key-chunk kernel: ragged ranges (1 … 300 keys) against the f64 reference"""
    rng = np.random.default_rng(5)
    lens = rng.integers(1, 300, 200)
    lens[:4] = [1, 31, 32, 33]
    starts = rng.integers(0, 200, 200)
    _attention_case(torch_dev, 128, nh, nkv, starts.tolist(), lens.tolist(), False, 3)


@pytest.mark.parametrize("hd,nh,nkv", [(128, 16, 8), (64, 16, 16)])
def test_attention_prefill_and_windows(torch_dev, hd, nh, nkv):
    """causal prompt rows of three utterances (tiles straddle utterance ends) and 104-key encoder windows"""
    starts, lens = [], []
    base = 0
    for n in (37, 70, 5):   # causal prefill: row i of an utterance sees keys [base, base + i]
        starts += [base] * n
        lens += list(range(1, n + 1))
        base += n + 3
    for w0 in range(0, 300, 104):   # bidirectional windows (the last one short)
        n = min(104, 300 - w0)
        starts += [base + w0] * n
        lens += [n] * n
    _attention_case(torch_dev, hd, nh, nkv, starts, lens, True, 7)
    _attention_case(torch_dev, hd, nh, nkv, starts[:40], lens[:40], False, 7)


def test_argmax(torch_dev):
    import torch

    rng = np.random.default_rng(8)
    x = rng.standard_normal((6, 151936)).astype(np.float32)
    x[2, 1000] = x[2, 5000] = 99.0  # tie → lowest index
    out = empty((6,), torch.int32, torch_dev)
    xt = dev(x, torch_dev)
    _lib.check(L().qasr_op_argmax(ptr(xt), 6, 151936, ptr(out), None))
    assert np.array_equal(host(out), x.argmax(1))


def test_embed_rows(torch_dev):
    import torch

    n, k = 50, 256
    blocks = oracle.synth_q8(11, "token_embd.weight", n, k, 1.0)
    qs, sc = q8_split(blocks, n, k)
    alt = np.random.default_rng(0).standard_normal((3, k)).astype(np.float32)
    ids = np.array([3, 0, -1, 49, -3, 3], np.int32)
    out = empty((len(ids), k), torch.float32, torch_dev)
    keep = [dev(a, torch_dev) for a in (ids, qs, sc, alt)]
    _lib.check(L().qasr_op_embed_rows(ptr(keep[0]), len(ids), ptr(keep[1]), ptr(keep[2]), k, ptr(keep[3]), ptr(out),
                                      None))
    deq = oracle.dequantize_q8(blocks, k)
    ref = np.stack([deq[i] if i >= 0 else alt[-(i + 1)] for i in ids])
    assert np.array_equal(host(out), ref)


@pytest.mark.parametrize("c,hi,wi,mode", [(480, 64, 50, 0), (480, 32, 25, 1), (64, 64, 50, 0), (64, 32, 25, 1)])
def test_conv3x3_gelu(torch_dev, c, hi, wi, mode):
    """conv 3×3 s2 p1 + erf-GELU implicit GEMM (f16 MFMA) vs an f64 numpy convolution of the same f16 data"""
    import torch
    from scipy.special import erf

    rng = np.random.default_rng(c + hi + mode)
    n = 2
    x = (rng.standard_normal((n, hi, wi, c)) * 0.5).astype(np.float16)
    w = (rng.standard_normal((c, c, 3, 3)) / np.sqrt(9 * c)).astype(np.float16)
    b = (rng.standard_normal(c) * 0.1).astype(np.float32)
    ho, wo = (hi + 1) // 2, (wi + 1) // 2
    xp = np.zeros((n, hi + 2, wi + 2, c), np.float64)
    xp[:, 1:-1, 1:-1] = x
    cols = np.stack([xp[:, ky:ky + 2 * ho:2, kx:kx + 2 * wo:2, :] for ky in range(3) for kx in range(3)], 3)
    ref = cols.reshape(n * ho * wo, 9 * c) @ w.astype(np.float64).transpose(2, 3, 1, 0).reshape(9 * c, c) + b
    ref = 0.5 * ref * (1 + erf(ref / np.sqrt(2)))
    wt = np.ascontiguousarray(w.transpose(0, 2, 3, 1).reshape(c, 9, c))    # [Cout][tap][Cin]
    xt, wd, bd = dev(x, torch_dev), dev(wt, torch_dev), dev(b, torch_dev)
    out = empty((n * ho * wo * c,), torch.float16 if mode == 0 else torch.float32, torch_dev)
    _lib.check(L().qasr_op_conv3x3_gelu(ptr(xt), n, hi, wi, ptr(wd), ptr(bd), c, ptr(out), mode, None))
    got = host(out).astype(np.float64)
    if mode == 0:
        got = got.reshape(n * ho * wo, c)
    else:  # [chunk][Wo][C][Ho] → rows (chunk, oy, ox)
        got = got.reshape(n, wo, c, ho).transpose(0, 3, 1, 2).reshape(n * ho * wo, c)
    tol = (2e-3 if mode == 0 else 1e-4) * np.abs(ref).max() + 1e-3 * np.abs(ref)
    assert (np.abs(got - ref) <= tol).all(), np.abs(got - ref).max()


@pytest.fixture
def fixup(torch_dev):
    """a registered split-K fix-up workspace (zeroed counters); unregistered afterwards"""
    import torch

    part = torch.empty(256 * 12288 * 8, dtype=torch.float32, device=torch_dev)
    cnt = torch.zeros(8192, dtype=torch.int32, device=torch_dev)
    _lib.check(L().qasr_op_set_gemm_fixup(ptr(part), part.numel() * 4, ptr(cnt), cnt.numel()))
    yield cnt
    _lib.check(L().qasr_op_set_gemm_fixup(None, 0, None, 0))


# split-K through the fix-up workspace: the decode tiles with 64-column wave tiles (≤ 64×64) × split counts
FIXUP_PATHS = [16 + c + 32 * s for c in (12, 15, 20, 22, 23) for s in (2, 3, 8)]


@pytest.mark.parametrize("path", FIXUP_PATHS)
@pytest.mark.parametrize("m,n,k", [(64, 128, 1024), (100, 192, 512), (32, 2048, 2048), (256, 4096, 2048)])
def test_linear_q8_fixup_exact_integer(torch_dev, fixup, path, m, n, k):
    y, ref = _linear_case(torch_dev, m, n, k, path, 0, seed=m + n, exact=True)
    assert np.array_equal(y, ref)
    assert not host(fixup).any()   # the last workgroup of every tile reset its counter


@pytest.mark.parametrize("path", FIXUP_PATHS)
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("m,n,k", [(37, 320, 2048), (24, 2048, 6144), (130, 1024, 1024)])
def test_linear_q8_fixup_vs_oracle(torch_dev, fixup, path, epi, m, n, k):
    """any epilogue on the summed tile (the residual and GELU are applied once, by the tile's last workgroup), and
    the partial tiles are added in split order: repeats are bit-identical"""
    y, ref = _linear_case(torch_dev, m, n, k, path, epi, seed=k + epi)
    scale = np.abs(ref).max() + 1e-6
    assert np.abs(y - ref).max() <= 2e-5 * scale * np.sqrt(k / 256)
    for _ in range(2):
        y2, _ = _linear_case(torch_dev, m, n, k, path, epi, seed=k + epi)
        assert np.array_equal(y, y2)
    assert not host(fixup).any()


# round 4: K-128 tiles with the stage scales by 16-byte DMA (WS4) and the one-group deep-ring 64×32 / 32×64 tiles;
# 4096 + cfg + 256·splits
S4_PATHS = [4096 + c + 256 * sp for c, sp in [(8, 1), (10, 1), (12, 1), (14, 1), (15, 1), (16, 1), (17, 1), (18, 1),
                                              (23, 1), (36, 1), (37, 1), (38, 1), (39, 1), (12, 3), (15, 4)]]


@pytest.mark.parametrize("path", S4_PATHS)
@pytest.mark.parametrize("m,n,k", [(64, 128, 1024), (100, 192, 512), (37, 320, 2048), (256, 256, 6144),
                                   (130, 1024, 1024), (256, 4096, 2048)])
def test_linear_q8_stage_scales(torch_dev, fixup, path, m, n, k):
    """exact integers through every new staging path, then real scales: the 16-byte scale DMA gives the bits of the
    4-byte gathers (same configuration), within the oracle bound; split counts through the fix-up"""
    y, ref = _linear_case(torch_dev, m, n, k, path, 0, seed=m + n, exact=True, s4=True)
    assert np.array_equal(y, ref)
    for epi in (0, 1):
        y4, ref = _linear_case(torch_dev, m, n, k, path, epi, seed=k + epi + 3, s4=True)
        y0, _ = _linear_case(torch_dev, m, n, k, path, epi, seed=k + epi + 3, s4=False)
        assert np.array_equal(y4, y0)
        scale = np.abs(ref).max() + 1e-6
        assert np.abs(y4 - ref).max() <= 2e-5 * scale * np.sqrt(k / 256)
    assert not host(fixup).any()


@pytest.mark.parametrize("path", [16 + 23 + 32 * 2, 16 + 15 + 32 * 8, 16 + 12 + 32 * 3])
@pytest.mark.parametrize("m,n,k", [(256, 12288, 2048), (48, 4096, 2048)])
def test_linear_q8_fixup_repeat_stress(torch_dev, fixup, path, m, n, k):
    """400 back-to-back launches on one stream with no host sync in between: the arrival counters are reused by
    every launch (the last workgroup of a tile resets its counter), so a missed reset or an early read of another
    workgroup's partial would show as a differing repeat or a non-zero counter"""
    import torch

    rng = np.random.default_rng(m + n)
    x = rng.standard_normal((m, k)).astype(np.float32)
    blocks = oracle.synth_q8(m + k, "w", n, k, 0.05)
    qs, sc = q8_split(blocks, n, k)
    xq = empty((m, k), torch.int8, torch_dev)
    xdd = empty((m, k // 32), torch.float32, torch_dev)
    xt = dev(x, torch_dev)
    _lib.check(L().qasr_op_quant_rows(ptr(xt), m, k, k, ptr(xq), ptr(xdd), None))
    wq, ws = dev(qs, torch_dev), dev(sc, torch_dev)
    reps = 400
    ys = torch.empty((reps, m, n), dtype=torch.float32, device=torch_dev)
    for r in range(reps):
        _lib.check(L().qasr_op_linear_q8(ptr(xq), ptr(xdd), m, ptr(wq), ptr(ws), n, k, None, None, ptr(ys[r]), n, 0,
                                         path, None))
    torch.cuda.synchronize()
    assert bool((ys == ys[0]).all())
    assert not host(fixup).any()
    ref = oracle.linear_q8(x, blocks, n, None) if m * n <= 48 * 4096 else None
    if ref is not None:
        scale = np.abs(ref).max() + 1e-6
        assert np.abs(host(ys[0]) - ref).max() <= 2e-5 * scale * np.sqrt(k / 256)


@pytest.mark.parametrize("cfg", [c + 32 * s for c in (12, 15, 20, 22) for s in (2, 4, 8)])
@pytest.mark.parametrize("m,f,k", [(40, 512, 1024), (70, 512, 2048), (256, 1024, 2048)])
def test_gemm_swiglu_q8_fixup(torch_dev, fixup, m, f, k, cfg):
    """split-K gate-up GEMM: the SwiGLU + Q8 epilogue runs once per tile on the summed partials"""
    test_gemm_swiglu_q8(torch_dev, m, f, k, cfg, False)
    assert not host(fixup).any()


@pytest.mark.parametrize("m", [1, 5, 16, 17, 32, 40, 97])
@pytest.mark.parametrize("n,k,epi", [(4096, 2048, 0), (2048, 2048, 1), (2048, 6144, 1), (12288, 2048, 0),
                                     (1024, 1024, 0), (1024, 3072, 1), (300, 4096, 0)])
def test_gemm_exact_rows_match_gemv(torch_dev, m, n, k, epi):
    """the verify passes' MFMA linear (gemm_exact_rows) == gemv_fused (pro 0) on each row ALONE, bit for bit: the same
    block fma chains and wave-sum tree (the exact-row contract of the drafted decode)"""
    import torch

    rng = np.random.default_rng(m + n + k)
    xq = dev(rng.integers(-127, 128, (m, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((m, k // 32)) * 0.02).astype(np.float32), torch_dev)
    xd[0, 3] = 0.0   # a zero block scale (all-zero block)
    res = dev((rng.standard_normal((m, n)) * 3).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, n, k, 9)
    y = res.clone()
    _lib.check(L().qasr_op_gemm_exact_rows(ptr(xq), ptr(xd), m, ptr(wq), ptr(ws), n, k, ptr(y) if epi else None, ptr(y),
                                           n, epi, None))
    for r in range(m):
        y1 = res[r:r + 1].clone()
        _lib.check(L().qasr_op_gemv_fused(0, None, 0, None, 0.0, 1, C.c_void_p(xq.data_ptr() + r * k),
                                          C.c_void_p(xd.data_ptr() + r * (k // 32) * 4), ptr(wq), ptr(ws), n, k,
                                          ptr(y1) if epi else None, ptr(y1), n, epi, None, None, None))
        assert np.array_equal(host(y)[r], host(y1)[0]), r


@pytest.mark.parametrize("split,P,R", [(True, 275, 17), (False, 275, 17), (True, 40, 9), (False, 600, 8)])
def test_attention_verify_rows_exact(torch_dev, split, P, R):
    """exact-row contract of the draft verify pass (engine.cpp decoder_layers, rows_share_kv): R consecutive positions
    of ONE utterance — qk_norm_rope writes every row's K/V first, then one fused decode attention launch (row i
    attends the rows 0…i-1 of the same pass) — gives, row by row, the same Q8 output bits and the same caches as R
    one-row decode steps (each step's fused kernel writes its own K/V), with and without the key-range split"""
    import torch

    hd, nh, nkv = 128, 16, 8
    nslot = nh + 2 * nkv
    rng = np.random.default_rng(31)
    qkv = rng.standard_normal((R, nslot * hd)).astype(np.float32)
    qnw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    knw = (1 + 0.1 * rng.standard_normal(hd)).astype(np.float32)
    tab = np.empty((1024, hd // 2, 2), np.float32)
    _lib.check(L().qasr_op_rope_table(1024, hd, 1e6, tab.ctypes.data_as(C.c_void_p)))
    slots = P + R + 1
    kc0 = (0.5 * rng.standard_normal((slots, nkv * hd))).astype(np.float16)
    vc0 = (0.5 * rng.standard_normal((slots, nkv * hd))).astype(np.float16)
    pos = np.arange(P, P + R, dtype=np.int32)
    start = np.zeros(R, np.int32)
    klen = (pos + 1).astype(np.int32)
    scale = 1.0 / np.sqrt(hd)
    keep = [dev(a, torch_dev) for a in (qkv, pos, qnw, knw, tab, start, klen)]
    part = torch.empty(32 * nkv * 16 * 2 * (2 + hd), dtype=torch.float32, device=torch_dev)
    cnt = torch.zeros(32 * nkv, dtype=torch.int32, device=torch_dev)

    def attn(qkv_p, rows, pos_p, kc, vc, st_p, len_p, oq, od):
        args = (qkv_p, rows, nh, nkv, hd, pos_p, pos_p, ptr(keep[2]), ptr(keep[3]), ptr(keep[4]), 1e-6, ptr(kc),
                ptr(vc), st_p, len_p, scale, ptr(oq), ptr(od))
        if split:
            _lib.check(L().qasr_op_attention_decode_split(*args, ptr(part), ptr(cnt), None))
        else:
            _lib.check(L().qasr_op_attention_decode_fused(*args, None))

    # steps: one row per launch, in position order
    kc_s, vc_s = dev(kc0, torch_dev), dev(vc0, torch_dev)
    oq_s = torch.zeros((R, nh * hd), dtype=torch.int8, device=torch_dev)
    od_s = torch.zeros((R, nh * hd // 32), dtype=torch.float32, device=torch_dev)
    for i in range(R):
        attn(C.c_void_p(keep[0].data_ptr() + i * nslot * hd * 4), 1, C.c_void_p(keep[1].data_ptr() + 4 * i), kc_s,
             vc_s, C.c_void_p(keep[5].data_ptr() + 4 * i), C.c_void_p(keep[6].data_ptr() + 4 * i),
             oq_s[i:i + 1], od_s[i:i + 1])
    # verify pass: K/V of all rows first, then one launch over the R rows
    kc_v, vc_v = dev(kc0, torch_dev), dev(vc0, torch_dev)
    qo = torch.empty((R, nh * hd), dtype=torch.float16, device=torch_dev)
    _lib.check(L().qasr_op_qk_norm_rope(ptr(keep[0]), R, nh, nkv, hd, ptr(keep[1]), ptr(keep[1]), ptr(keep[2]),
                                        ptr(keep[3]), ptr(keep[4]), 1e-6, ptr(qo), ptr(kc_v), ptr(vc_v), None))
    oq_v = torch.zeros_like(oq_s)
    od_v = torch.zeros_like(od_s)
    attn(ptr(keep[0]), R, ptr(keep[1]), kc_v, vc_v, ptr(keep[5]), ptr(keep[6]), oq_v, od_v)
    assert np.array_equal(host(kc_s), host(kc_v)) and np.array_equal(host(vc_s), host(vc_v))
    a, b = host(oq_s), host(oq_v)
    bad = [i for i in range(R) if not np.array_equal(a[i], b[i])]
    assert not bad, bad
    assert np.array_equal(host(od_s), host(od_v))


# the ≤ 32-row decode's per-phase launches (kernels_xr.hip xr_*): bit-identical to the exact-row chain
@pytest.mark.parametrize("m", [1, 3, 8, 16, 17, 32])
@pytest.mark.parametrize("n,k,epi", [(4096, 2048, 0), (2048, 2048, 1), (2048, 6144, 1), (1024, 3072, 1), (4096, 1024, 0)])
def test_xr_linear_bit_identical_to_exact_rows(torch_dev, m, n, k, epi):
    """qasr_op_xr_linear (weights loaded up front, rows staged in LDS) == qasr_op_gemm_exact_rows, bit for bit, and
    for ≤ 8 rows with the norm folded in (src rows, K ≤ 2,048) == qasr_op_rmsnorm_q8 + qasr_op_gemm_exact_rows"""
    rng = np.random.default_rng(m * 7 + n + k)
    xq = dev(rng.integers(-127, 128, (m, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((m, k // 32)) * 0.02).astype(np.float32), torch_dev)
    xd[0, 3] = 0.0
    res = dev((rng.standard_normal((m, n)) * 3).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, n, k, 11)
    y_ref, y = res.clone(), res.clone()
    _lib.check(L().qasr_op_gemm_exact_rows(ptr(xq), ptr(xd), m, ptr(wq), ptr(ws), n, k, ptr(y_ref) if epi else None,
                                           ptr(y_ref), n, epi, None))
    _lib.check(L().qasr_op_xr_linear(ptr(xq), ptr(xd), None, None, 0.0, m, ptr(wq), ptr(ws), n, k, ptr(y), n, epi,
                                     None))
    assert np.array_equal(host(y), host(y_ref))
    if m <= 8 and k <= 2048 and epi == 0:
        src = dev((rng.standard_normal((m, k)) * 2).astype(np.float32), torch_dev)
        nw = dev((1 + 0.1 * rng.standard_normal(k)).astype(np.float32), torch_dev)
        q2 = empty((m, k), __import__("torch").int8, torch_dev)
        d2 = empty((m, k // 32), __import__("torch").float32, torch_dev)
        _lib.check(L().qasr_op_rmsnorm_q8(ptr(src), m, k, ptr(nw), C.c_float(1e-6), ptr(q2), ptr(d2), None))
        _lib.check(L().qasr_op_gemm_exact_rows(ptr(q2), ptr(d2), m, ptr(wq), ptr(ws), n, k, None, ptr(y_ref), n, 0,
                                               None))
        _lib.check(L().qasr_op_xr_linear(None, None, ptr(src), ptr(nw), C.c_float(1e-6), m, ptr(wq), ptr(ws), n, k,
                                         ptr(y), n, 0, None))
        assert np.array_equal(host(y), host(y_ref))


@pytest.mark.parametrize("m", [1, 5, 8, 16, 32])
@pytest.mark.parametrize("f,k", [(6144, 2048), (3072, 1024)])
def test_xr_gu_swiglu_bit_identical(torch_dev, m, f, k):
    """qasr_op_xr_gu_swiglu (an h block per workgroup: 4 exact fragments + SwiGLU + Q8) == gemm_exact_rows on the
    interleaved gate/up + swiglu_q8_interleaved, bit for bit; with the norm folded in (≤ 8 rows) == rmsnorm_q8 first"""
    import torch

    rng = np.random.default_rng(m + f + k)
    xq = dev(rng.integers(-127, 128, (m, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((m, k // 32)) * 0.02).astype(np.float32), torch_dev)
    wq, ws = _q8_weights(torch_dev, 2 * f, k, 13)
    gu = empty((m, 2 * f), torch.float32, torch_dev)
    hq_ref, hd_ref = empty((m, f), torch.int8, torch_dev), empty((m, f // 32), torch.float32, torch_dev)
    hq, hd = empty((m, f), torch.int8, torch_dev), empty((m, f // 32), torch.float32, torch_dev)

    def ref(q, d):
        _lib.check(L().qasr_op_gemm_exact_rows(ptr(q), ptr(d), m, ptr(wq), ptr(ws), 2 * f, k, None, ptr(gu), 2 * f, 0,
                                               None))
        _lib.check(L().qasr_op_swiglu_q8_interleaved(ptr(gu), m, f, ptr(hq_ref), ptr(hd_ref), None))

    ref(xq, xd)
    _lib.check(L().qasr_op_xr_gu_swiglu(ptr(xq), ptr(xd), None, None, 0.0, m, ptr(wq), ptr(ws), 2 * f, k, ptr(hq),
                                        ptr(hd), None))
    assert np.array_equal(host(hq), host(hq_ref)) and np.array_equal(host(hd), host(hd_ref))
    if m <= 8:
        src = dev((rng.standard_normal((m, k)) * 2).astype(np.float32), torch_dev)
        nw = dev((1 + 0.1 * rng.standard_normal(k)).astype(np.float32), torch_dev)
        q2, d2 = empty((m, k), torch.int8, torch_dev), empty((m, k // 32), torch.float32, torch_dev)
        _lib.check(L().qasr_op_rmsnorm_q8(ptr(src), m, k, ptr(nw), C.c_float(1e-6), ptr(q2), ptr(d2), None))
        ref(q2, d2)
        _lib.check(L().qasr_op_xr_gu_swiglu(None, None, ptr(src), ptr(nw), C.c_float(1e-6), m, ptr(wq), ptr(ws), 2 * f,
                                            k, ptr(hq), ptr(hd), None))
        assert np.array_equal(host(hq), host(hq_ref)) and np.array_equal(host(hd), host(hd_ref))


@pytest.mark.parametrize("m", [1, 5, 9, 16])
@pytest.mark.parametrize("n,k", [(8224, 2048), (4112, 1024)])
def test_xr_vocab_bit_identical_to_gemv_rows(torch_dev, m, n, k):
    """qasr_op_xr_vocab (the 5–16-row vocabulary projection: resident workgroups walking the 16-column fragments, the
    next fragment's weights loading meanwhile; N chosen so the fragments do not divide the grid evenly) == the
    weight-streaming GEMV's row groups (qasr_op_gemv_fused) == gemm_exact_rows, bit for bit"""
    import torch

    rng = np.random.default_rng(m * 31 + n + k)
    xq = dev(rng.integers(-127, 128, (m, k), dtype=np.int8), torch_dev)
    xd = dev((rng.random((m, k // 32)) * 0.02).astype(np.float32), torch_dev)
    xd[0, 1] = 0.0
    wq, ws = _q8_weights(torch_dev, n, k, 17)
    y_gv, y_ex, y = (torch.full((m, n), 7.0, dtype=torch.float32, device=torch_dev) for _ in range(3))
    _lib.check(L().qasr_op_gemv_fused(0, None, 0, None, C.c_float(0.0), m, ptr(xq), ptr(xd), ptr(wq), ptr(ws), n, k,
                                      None, ptr(y_gv), n, 0, None, None, None))
    _lib.check(L().qasr_op_gemm_exact_rows(ptr(xq), ptr(xd), m, ptr(wq), ptr(ws), n, k, None, ptr(y_ex), n, 0, None))
    _lib.check(L().qasr_op_xr_vocab(ptr(xq), ptr(xd), m, ptr(wq), ptr(ws), n, k, ptr(y), n, None))
    assert np.array_equal(host(y), host(y_gv)) and np.array_equal(host(y), host(y_ex))
