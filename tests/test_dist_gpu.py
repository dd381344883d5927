"""libqasr's native RCCL collectives (include/qasr.h qasr_dist_*) on one GPU: a world-size-1
communicator — unique id, comm init, the blob broadcast into a shell (send = the source model's blob, recv = the
shell's: the data movement of a rank-0 → rank-k broadcast), the weight broadcast with its checksum hand-shake, and the
ragged token gather.  The N = 2/3 orchestration (LPT shards, ragged gathers, empty ranks) is covered on CPU with gloo
(tests/test_shard_cpu.py); RCCL refuses two ranks on one card, so N > 1 RCCL runs only on the driver's 8-GPU node."""
import os

import numpy as np
import pytest

from make_golden import TINY_SEED
from test_model_gpu import _tokens, tiny_hparams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden():
    import os

    return np.load(os.path.join(os.path.dirname(__file__), "golden", "hf_tiny.npz"))


def test_native_rccl_world1(torch_dev, golden):
    from qasr import _lib
    from qasr.dist import NativeComm
    from qasr.transcribe_cpp import Model

    comm = NativeComm(0, 1, 0, lambda b: b)
    m = Model.synthetic(arch=None, seed=TINY_SEED, hparams=tiny_hparams())
    sh = Model.shell(arch=None, hparams=tiny_hparams())
    try:
        s = m.session(kv_type="f16", n_ctx=2048)
        want = _tokens(s, golden)
        # the broadcast's data movement: the source blob into the shell's (send != recv)
        a, n = m.weight_blob()
        b, n2 = sh.weight_blob()
        assert n == n2 and a != b
        comm.broadcast(a, b, n, 0)
        sh.weights_received()
        s2 = sh.session(kv_type="f16", n_ctx=2048)
        assert _tokens(s2, golden) == want
        s2.close()
        # the weight broadcast itself (in place at the root) with the checksum hand-shake
        info = comm.broadcast_weights(m)
        assert info["bytes"] == n and info["checksums_agree"] and info["native_rccl"]
        assert _tokens(s, golden) == want
        # a shell that never received anything stays refused for sessions
        sh2 = Model.shell(arch=None, hparams=tiny_hparams())
        with pytest.raises(RuntimeError):
            sh2.session(kv_type="f16", n_ctx=2048)
        sh2.close()
        # the token gather: ragged, an empty segment included; world 1 → this rank's streams back
        streams = [[5, 6, 7], [], list(range(100, 140))]
        assert comm.gather_tokens(streams) == [streams]
        assert comm.gather_tokens([]) == [[]]
        s.close()
    finally:
        sh.close()
        m.close()
        comm.close()
    assert _lib.load() is not None


def test_native_init_deadline_when_a_rank_never_joins():
    """qasr_dist_init_deadline: rank 0 of a world-2 communicator whose rank 1 never calls init
    returns QASR_E_BACKEND at the deadline (the init on a helper thread the caller stops waiting for) instead of
    blocking forever.  Run in a child process, so even a hang could not take the
    test runner with it."""
    import subprocess
    import sys
    import textwrap
    import time

    code = textwrap.dedent("""
        import os, sys, time
        sys.path.insert(0, %r)
        from qasr.dist import NativeComm
        uid = NativeComm.unique_id()
        t0 = time.monotonic()
        try:
            NativeComm(0, 2, 0, uid=uid, timeout_ms=4000)
        except RuntimeError as e:
            print("ERR", round(time.monotonic() - t0, 2), str(e).replace(chr(10), " ")[:300], flush=True)
            os._exit(0)   # the abandoned init thread is still inside RCCL: leave without runtime teardown (qasr.h)
        print("JOINED", flush=True)
        os._exit(3)
    """ % os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "light-whisper_amd"))
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90)
    took = time.monotonic() - t0
    assert out.returncode == 0, (out.returncode, out.stdout[-500:], out.stderr[-2000:])
    line = [x for x in out.stdout.splitlines() if x.startswith("ERR")][0]
    waited = float(line.split()[1])
    print(line, f"(child {took:.1f} s)")
    assert 3.5 <= waited <= 60.0, line
    assert "timed out" in line, line

