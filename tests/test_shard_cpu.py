"""N>1 path of bench.py on CPU: world-size-2 gloo ranks shard the C4 segment list (LPT, no data-path collective)
and reduce the step time with MAX and the audio-seconds with SUM, exactly as bench.py does over RCCL."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(1)
    secs = rng.uniform(2.0, 12.0, size=bench.SEG_PER_RANK * world)
    lengths = [int(x * 16000) for x in secs]
    mine = sorted(bench.lpt_shard(lengths, world)[rank])
    audio_s = sum(lengths[i] for i in mine) / 16000.0
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    tot = torch.tensor([audio_s], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    got = [None] * world
    dist.all_gather_object(got, mine)
    q.put((rank, float(t.item()), float(tot.item()), got, float(sum(lengths)) / 16000.0))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_lpt_sharding_gloo(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, tmax, tot, shards, total in out:
        assert tmax == 0.5 + (world - 1)            # max over ranks
        assert abs(tot - total) < 1e-6               # every segment counted once
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(bench.SEG_PER_RANK * world))   # disjoint cover
        assert min(len(s) for s in shards) > 0


def test_lpt_balance():
    rng = np.random.default_rng(1)
    for world in (2, 4, 8):
        secs = rng.uniform(2.0, 12.0, size=256 * world)
        shards = bench.lpt_shard(list(secs), world)
        loads = [sum(secs[i] for i in s) for s in shards]
        assert max(loads) / min(loads) < 1.01


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_strong_sharding_256_total(world):
    """--scaling strong (the default; BASELINE configs[3] as stated): 256 segments IN TOTAL, LPT over N ranks —
    every segment on exactly one rank and the audio-seconds balanced (32 segments per GPU at N = 8)"""
    rng = np.random.default_rng(1)
    secs = rng.uniform(2.0, 12.0, size=256)
    lengths = [int(x * 16000) for x in secs]
    shards = bench.lpt_shard(lengths, world)
    flat = sorted(i for sh in shards for i in sh)
    assert flat == list(range(256))                             # disjoint cover of the 256
    loads = [sum(lengths[i] for i in sh) for sh in shards]
    assert max(loads) / min(loads) < (1.001 if world == 1 else 1.03)
    assert max(len(sh) for sh in shards) - min(len(sh) for sh in shards) <= max(2, 256 // world // 4)
    # make_workload(total=256) hands each rank exactly its shard's audio, and N = 1 is the weak-scaling list
    got = sum(len(bench.make_workload(world, r, total=256)) for r in range(world)) if world <= 2 else None
    if got is not None:
        assert got == 256
    if world == 1:
        a, b = bench.make_workload(1, 0, total=256), bench.make_workload(1, 0)
        assert len(a) == len(b) and all(np.array_equal(x, y) for x, y in zip(a, b))


def _xchg_rank(rank, world, key, d, q):
    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    x = qdist.file_exchange(rank, world, key=key, directory=d, timeout_s=60)
    payload = bytes(range(128)) if rank == 0 else bytes(128)
    got = x(payload)
    q.put((rank, got))


def test_file_unique_id_exchange(tmp_path):
    """the torch-free unique-id hand-off (qasr/dist.py file_exchange, what a Rust host does with a file of its own):
    rank 0's 128 bytes reach every rank, readers never see a partial file, rank 0 removes the file afterwards"""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 3
    procs = [ctx.Process(target=_xchg_rank, args=(r, world, "t1", str(tmp_path), q)) for r in (1, 2, 0)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(v == bytes(range(128)) for v in out.values())
    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    x = qdist.file_exchange(0, world, key="t1", directory=str(tmp_path))
    assert os.path.exists(x.path)
    x.cleanup()
    assert not os.path.exists(x.path) and not [f for f in os.listdir(tmp_path) if f.endswith(".tmp")]


def test_file_unique_id_default_key_is_launch_unique(tmp_path):
    """the default key (run id + master port + the launcher's pid): ranks started by one launcher agree on it (the
    exchange goes through), and a stale file an earlier launch left under the same run id and port is not read"""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    stale = os.path.join(str(tmp_path), "qasr_uid_run_0.bin")   # round 3's key format
    with open(stale, "wb") as f:
        f.write(bytes([7]) * 128)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_xchg_rank, args=(r, 2, None, str(tmp_path), q)) for r in (1, 0)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=60) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert out[1] == bytes(range(128))
    assert qdist.file_exchange(0, 2, directory=str(tmp_path)).path.endswith(f"_{os.getppid()}.bin")


def test_workload_deterministic():
    a = bench.make_workload(2, 1)
    b = bench.make_workload(2, 1)
    assert len(a) == len(b) and all(np.array_equal(x, y) for x, y in zip(a, b))
    assert all(x.dtype == np.float32 and np.abs(x).max() <= 1.0 for x in a)


def _collectives_rank(rank, world, port, q):
    """bench.py's two collectives (qasr/dist.py) on gloo: the weight-blob broadcast into a shell and the ragged
    token-stream gather (rank 1 has an empty segment; the last rank has no segments at all)."""
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blob = torch.from_numpy(np.random.default_rng(7).integers(0, 256, 4096, dtype=np.uint8)) if rank == 0 \
        else torch.zeros(4096, dtype=torch.uint8)
    info = qdist.broadcast_blob(blob, src=0)
    streams = [] if rank == world - 1 else [list(range(rank * 100, rank * 100 + n)) for n in (3, 0, 5 + rank)]
    got = qdist.gather_token_streams(streams, torch.device("cpu"))
    q.put((rank, info, blob.numpy().tobytes(), got))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_weight_broadcast_and_token_gather_gloo(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_collectives_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src = np.random.default_rng(7).integers(0, 256, 4096, dtype=np.uint8).tobytes()
    want = [[] if r == world - 1 else [list(range(r * 100, r * 100 + n)) for n in (3, 0, 5 + r)] for r in range(world)]
    for rank, info, blob, got in out:
        assert info["bytes"] == 4096 and info["checksums_agree"]
        assert blob == src
        assert got == want


def _agree_rank(rank, world, port, fail_rank, q):
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def attempt():
        if rank == fail_rank:
            raise RuntimeError("ncclCommInitRank: invalid usage")
        return {"rank": rank}

    got = qdist.agreed_attempt(attempt)
    # the ranks must still be in step afterwards: one more collective completes on all of them
    after = qdist.gather_token_streams([[rank]], __import__("torch").device("cpu"))
    q.put((rank, got, after))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (3, 0), (3, -1)])
def test_native_failure_is_agreed_by_every_rank(world, fail_rank):
    """bench.py's native-RCCL attempt (communicator + weight broadcast) is agreed over the gloo group: an error on
    ANY rank makes every rank return the fallback verdict together (no rank goes on alone into a collective that
    would block), and with no error every rank keeps its own result"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_rank, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, (res, err), after in out:
        assert after == [[[r]] for r in range(world)]
        if fail_rank < 0:
            assert res == {"rank": rank} and err is None
        else:
            assert res is None
            assert err == ("RuntimeError: ncclCommInitRank: invalid usage" if rank == fail_rank
                           else "failed on another rank")


def _setup_rank(rank, world, port, fail, rdv, q):
    """bench.py's native setup (qasr.dist.native_setup) with a fake communicator whose init is a BLOCKING collective
    (a gloo barrier, like ncclCommInitRank): `fail` = ("uid", rank) injects an error in the id hand-off (rank 0
    cannot create it, or another rank cannot read it)"""
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    step, frank = fail
    inits = []

    class FakeComm:
        @staticmethod
        def unique_id():
            if step == "uid" and frank == 0:
                raise RuntimeError("qasr_dist_unique_id failed")
            return bytes(range(128))

        def __init__(self, r, w, dev, uid=None):
            assert uid == bytes(range(128))
            dist.barrier()   # the blocking collective every rank must enter together
            inits.append(r)

        def broadcast_weights(self, model):
            dist.barrier()
            return {"ok": True}

        def close(self):
            pass

    xchg = qdist.file_exchange(rank, world, key=f"t{port}", directory=rdv, timeout_s=60.0)
    if step == "uid" and frank > 0 and rank == frank:   # this rank cannot read the id (e.g. another host)
        xchg = lambda payload: (_ for _ in ()).throw(TimeoutError("no unique id"))  # noqa: E731
    comm, info, err = qdist.native_setup(rank, world, 0, None, xchg, comm_cls=FakeComm)
    after = qdist.gather_token_streams([[rank]], __import__("torch").device("cpu"))
    q.put((rank, comm is not None, info, err, inits, after))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail", [(2, ("uid", 0)), (3, ("uid", 0)), (3, ("uid", 2)), (2, ("uid", 1)),
                                        (3, ("none", -1))])
def test_native_setup_agrees_before_each_collective(world, fail, tmp_path):
    """the native setup agrees after the id hand-off and before the (blocking) communicator init, and again
    before the broadcast — a rank that fails to get the id (rank 0 cannot create it: the others stop polling at the
    marker file; or a rank cannot read it) never leaves the others waiting inside the init, and every rank returns the
    same verdict within seconds"""
    import time

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_setup_rank, args=(r, world, port, fail, str(tmp_path), q)) for r in range(world)]
    t0 = time.monotonic()
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert time.monotonic() - t0 < 90
    step, frank = fail
    for rank, ok, info, err, inits, after in out:
        assert after == [[[r]] for r in range(world)]   # still in step afterwards
        if step == "none":
            assert ok and info == {"ok": True} and err is None and inits == [rank]
            continue
        assert not ok and info is None and err
        if rank == frank:
            assert "qasr_dist_unique_id failed" in err or "no unique id" in err, err
        else:
            assert err == "failed on another rank" or "rank 0 failed to publish" in err, err
        assert inits == []   # nobody entered the blocking init
    assert not os.listdir(tmp_path) or all(not f.endswith(".bin") for f in os.listdir(tmp_path))


def _stage_rank(rank, world, port, fail_rank, stage, q):
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import dist as qdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fail_rank is not None:
        os.environ.update(QASR_FAIL_STAGE=stage, QASR_FAIL_RANK=str(fail_rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    done = []
    err = None
    try:
        for name in ("model", "vad", "asr"):
            qdist.agreed_stage(name, lambda: done.append(name), qdist.gloo_agree, rank=rank)
            dist.barrier()   # the collective that follows the stage
    except qdist.StageFailed as e:
        err = str(e)
    q.put((rank, done, err))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,stage", [(2, 0, "vad"), (2, 1, "asr"), (3, 0, "asr"), (3, 2, "vad"),
                                                   (3, 2, "model"), (3, None, "asr")])
def test_longform_stage_agreement_gloo(world, fail_rank, stage):
    """engine_longform.cpp's failure agreement (qasr_dist_agree before each collective), in its Python mirror
    qasr.dist.agreed_stage over gloo: one rank's stage failure (first rank and last rank) makes EVERY rank stop at that
    stage with an error — none is left in the collective that follows"""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stage_rank, args=(r, world, port, fail_rank, stage, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    order = ["model", "vad", "asr"]
    for rank, done, err in out:
        if fail_rank is None:
            assert done == order and err is None
            continue
        k = order.index(stage)
        assert done == order[:k + (0 if rank == fail_rank else 1)], (rank, done)
        assert err == (f"RuntimeError: injected failure (QASR_FAIL_STAGE={stage})" if rank == fail_rank
                       else f"{stage}: failed on another rank"), err


def _prob_gather_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
    from qasr import longform

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = 1001
    f0, f1, h0, h1 = longform.frame_shard(T, rank, world)
    local = np.arange(f0, f1, dtype=np.float32) / T
    q.put((rank, longform.gather_probabilities(local, torch.device("cpu")), (f0, f1, h0, h1)))
    dist.destroy_process_group()


def test_long_form_probability_gather_gloo():
    """the ranks' core frame ranges tile the recording and the all-gather reassembles it in time order"""
    import torch.multiprocessing as mp

    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_prob_gather_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.arange(1001, dtype=np.float32) / 1001
    for rank, got, (f0, f1, h0, h1) in out:
        assert np.array_equal(got, want)
        assert h0 == max(0, f0 - 160) and h1 == min(1001, f1 + 160)


def _bench(args, env_extra=None, timeout=120):
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_launcher_dry_run():
    """`bench.py --gpus N` without WORLD_SIZE spawns N ranks through torch.distributed.run on 127.0.0.1; every
    child sees WORLD_SIZE == N (the launcher logic end to end, minus the GPU work)."""
    import json

    r = _bench(["--gpus", "2", "--steps", "3", "--dry-run-launch"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=2" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:] == \
        ["--gpus", "2", "--steps", "3"]
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd + ["--dry-run-launch"], env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 2 and all(x == {"launch": None, "world": 2} for x in lines)


def test_bench_gpus_fails_loudly_without_devices():
    """--gpus 2 with fewer visible GPUs (none here) exits non-zero before any rank starts; a rank whose WORLD_SIZE
    disagrees with --gpus exits non-zero too."""
    r = _bench(["--gpus", "2", "--no-cpu-baseline"], {"QASR_DIST_BACKEND": "nccl"})
    assert r.returncode == 2 and "only 0 GPU(s) visible" in r.stderr
    r = _bench(["--gpus", "1", "--no-cpu-baseline"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in r.stderr
