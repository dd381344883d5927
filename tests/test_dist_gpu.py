"""libqasr's native RCCL collectives (include/qasr.h qasr_dist_*) on one GPU: a world-size-1
communicator — unique id, comm init, the blob broadcast into a shell (send = the source model's blob, recv = the
shell's: the data movement of a rank-0 → rank-k broadcast), the weight broadcast with its checksum hand-shake, and the
ragged token gather.  The N = 2/3 orchestration (LPT shards, ragged gathers, empty ranks) is covered on CPU with gloo
(tests/test_shard_cpu.py); RCCL refuses two ranks on one card, so N > 1 RCCL runs only on the driver's 8-GPU node."""
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
