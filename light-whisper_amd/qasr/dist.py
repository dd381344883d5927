"""The two collectives of the multi-GPU path (north_star: "RCCL over xGMI used only to broadcast Q8
weights and gather token streams").  One process per GPU; nothing here runs inside a timed step.

On GPUs the collectives are libqasr's own RCCL communicator (`NativeComm`, include/qasr.h qasr_dist_*: the path a
host without PyTorch — the Rust app — drives); the 128-byte unique id reaches the other ranks through a file
(`file_exchange`), as a Rust host would hand it over, and bench.py's barrier / timing reductions run over a CPU (gloo)
group, so each rank holds exactly one RCCL communicator.  The torch.distributed versions below serve the "gloo"
rehearsal (ranks sharing one card, which RCCL refuses), the `torch-nccl` fallback and the CPU tests.

* `broadcast_weights`: rank 0 holds the loaded (or generated) model, every other rank a shell with the identical
  device layout (`Model.shell`, include/qasr.h qasr_model_open_shell); ONE broadcast over the whole weight blob
  (2.2 GB for 1.7B — a single large message, the shape a per-link-bound ring over xGMI wants) makes them equal,
  and a wrapping int64 checksum gathered from every rank proves it.
* `gather_token_streams`: after a batch, every rank's per-segment token ids reach rank 0 as two all-gathers —
  the (segments, tokens) counts, then the ragged payload padded to the largest rank.

The reference has no multi-GPU path (SURVEY §8(e) "Reference equivalent: none").
"""
from __future__ import annotations

import contextlib
import time

import numpy as np


def device_bytes(ptr: int, nbytes: int, device):
    """A uint8 torch tensor over `nbytes` of device memory owned elsewhere (the model's weight blob), through
    __cuda_array_interface__ — no copy; the owner must outlive the view."""
    import torch

    class _Iface:
        __cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False),
                                    "version": 3, "strides": None}

    t = torch.as_tensor(_Iface(), device=device)
    assert t.data_ptr() == int(ptr) and t.numel() == int(nbytes), "device view does not alias the blob"
    return t


def blob_checksum(t) -> int:
    """Wrapping int64 sum of a byte blob (length a multiple of 8; the weight arena is 256-B granular):
    order-independent, so every rank's reduction gives the same value for the same bytes."""
    import torch

    assert t.numel() % 8 == 0
    return int(t.view(torch.int64).sum(dtype=torch.int64).item())


def broadcast_blob(t, src: int = 0) -> dict:
    """Broadcast the byte tensor `t` from `src` and verify it arrived: returns bytes, wall ms of the collective
    and whether every rank's checksum equals the source's."""
    import torch
    import torch.distributed as dist

    sync = torch.cuda.synchronize if t.is_cuda else (lambda: None)
    staged = t.is_cuda and dist.get_backend() == "gloo"   # rehearsal runs: gloo moves host tensors only
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    if staged:
        h = t.cpu()
        dist.broadcast(h, src=src)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src)
    sync()
    ms = (time.perf_counter() - t0) * 1e3
    cdev = torch.device("cpu") if staged else t.device
    mine = torch.tensor([blob_checksum(t)], dtype=torch.int64, device=cdev)
    every = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(every, mine)
    sums = [int(x.item()) for x in every]
    return {"bytes": int(t.numel()), "ms": round(ms, 3), "staged_via_host": staged,
            "GB_per_s": round(t.numel() / ms / 1e6, 1) if ms > 0 else None,
            "checksums_agree": all(s == sums[src] for s in sums)}


def broadcast_weights(model, rank: int, device, src: int = 0) -> dict:
    """Rank `src` passes its loaded model, the others a `Model.shell` of the same layout; afterwards every rank's
    model holds rank `src`'s weights and the shells accept sessions."""
    ptr, nbytes = model.weight_blob()
    info = broadcast_blob(device_bytes(ptr, nbytes, device), src=src)
    if not info["checksums_agree"]:
        raise RuntimeError("weight broadcast: checksums differ across ranks")
    if rank != src:
        model.weights_received()
    return info


def agreed_attempt(attempt, group=None):
    """Run `attempt()` on every rank and agree on the outcome over `group` (default: the default process group — a
    gloo group, so the agreement does not depend on the RCCL path being tried).  Returns (result, None) on every rank
    when every rank succeeded, else (None, error text) on every rank — the failing rank's exception, or "failed on
    another rank" — so all ranks take the fallback together instead of one going on alone into a collective that
    would block the job (bench.py: the native communicator + weight broadcast)."""
    import torch
    import torch.distributed as dist

    result, err = None, None
    try:
        result = attempt()
    except Exception as e:  # noqa: BLE001 — returned to the caller, never silent
        err = f"{type(e).__name__}: {e}"
    ok = torch.tensor([0 if err else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if int(ok.item()):
        return result, None
    return None, err or "failed on another rank"


def gloo_agree(failed: bool, group=None) -> bool:
    """`agree` over a torch.distributed group: True on every rank if any rank's `failed` is set"""
    import torch
    import torch.distributed as dist

    t = torch.tensor([1 if failed else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(int(t.item()))


class StageFailed(RuntimeError):
    pass


def agreed_stage(name: str, fn, agree, rank: int = 0):
    """engine_longform.cpp's failure-agreement protocol (the Rust host copies it): run `fn()` locally, then agree on
    every rank's outcome — `agree(failed) -> any_failed`, NativeComm.agree (qasr_dist_agree over RCCL) or gloo_agree —
    before the collective that follows; if any rank failed, EVERY rank raises StageFailed (the failing rank with its
    own reason), so no rank goes on alone into a collective that would block.  QASR_FAIL_STAGE=<name>
    [QASR_FAIL_RANK=r] injects a failure (tests)."""
    import os

    err = None
    try:
        inj = os.environ.get("QASR_FAIL_STAGE")
        if inj == name and int(os.environ.get("QASR_FAIL_RANK", "-1")) in (-1, rank):
            raise RuntimeError(f"injected failure (QASR_FAIL_STAGE={name})")
        result = fn()
    except Exception as e:  # noqa: BLE001 — agreed on, then raised on every rank
        err, result = f"{type(e).__name__}: {e}", None
    if agree(err is not None):
        raise StageFailed(err or f"{name}: failed on another rank")
    return result


def native_setup(rank: int, world: int, device: int, model, exchange, comm_cls=None, agree_group=None):
    """bench.py's native collectives, each step agreed over the gloo group (which does not depend on RCCL) before the
    next collective starts: (1) the unique-id hand-off (`exchange`, e.g. file_exchange), (2) the communicator init,
    (3) the weight broadcast.  Returns (comm, broadcast info, None) or (None, None, error text) — the same verdict on
    every rank, so all ranks take the fallback together, and no rank enters RCCL's blocking init unless every rank
    holds the id.  (A rank that fails INSIDE RCCL's init is the one case this cannot cover.)"""
    comm_cls = comm_cls or NativeComm
    holder = []

    def get_uid():
        if rank != 0:
            return exchange(bytes(128))
        try:
            return exchange(comm_cls.unique_id())
        except Exception:
            if hasattr(exchange, "fail"):
                exchange.fail()
            raise

    uid, err = agreed_attempt(get_uid, group=agree_group)
    if err is None:
        _, err = agreed_attempt(lambda: holder.append(comm_cls(rank, world, device, uid=uid)), group=agree_group)
    if err is None:
        if hasattr(exchange, "cleanup"):
            exchange.cleanup()   # after the collective init: every rank has read the id
        info, err = agreed_attempt(lambda: holder[0].broadcast_weights(model), group=agree_group)
        if err is None:
            return holder[0], info, None
    if hasattr(exchange, "cleanup"):
        exchange.cleanup()
    if holder:
        holder[0].close()
    return None, None, err


def gather_token_streams(streams: list[list[int]], device) -> list[list[list[int]]]:
    """All-gather every rank's per-segment token ids; returns, on every rank, [rank][segment] -> ids."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    lens = np.array([len(s) for s in streams], dtype=np.int32)
    flat = np.concatenate([np.asarray(s, np.int32) for s in streams]) if lens.sum() else np.zeros(0, np.int32)
    counts = torch.tensor([lens.size, flat.size], dtype=torch.int64, device=device)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts)
    all_counts = [tuple(int(v) for v in c.tolist()) for c in all_counts]
    max_seg = max(1, max(c[0] for c in all_counts))
    max_tok = max(1, max(c[1] for c in all_counts))
    lens_t = torch.zeros(max_seg, dtype=torch.int32, device=device)
    lens_t[: lens.size] = torch.from_numpy(lens).to(device)
    tok_t = torch.zeros(max_tok, dtype=torch.int32, device=device)
    tok_t[: flat.size] = torch.from_numpy(flat).to(device)
    all_lens = [torch.zeros_like(lens_t) for _ in range(world)]
    all_toks = [torch.zeros_like(tok_t) for _ in range(world)]
    dist.all_gather(all_lens, lens_t)
    dist.all_gather(all_toks, tok_t)
    out = []
    for (nseg, ntok), lt, tt in zip(all_counts, all_lens, all_toks):
        ln = lt[:nseg].cpu().numpy()
        tk = tt[:ntok].cpu().numpy()
        offs = np.concatenate([[0], np.cumsum(ln)])
        out.append([tk[offs[i]:offs[i + 1]].tolist() for i in range(nseg)])
    return out


@contextlib.contextmanager
def stdout_to_stderr():
    """fd 1 → stderr around RCCL's first initialisation: RCCL prints its version banner on stdout, which is bench.py's
    JSON channel.  The library itself leaves process-wide descriptors alone (include/qasr.h "Multi-GPU")."""
    import os
    import sys

    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class NativeComm:
    """libqasr's RCCL communicator (qasr_dist_*).  Rank 0 creates the unique id; `exchange` (any callable that
    returns rank 0's bytes on every rank, e.g. torch.distributed.broadcast_object_list) distributes it."""

    def __init__(self, rank: int, world: int, device: int, exchange=None, uid: bytes | None = None,
                 timeout_ms: float = 0.0):
        """either `exchange` (rank 0 creates the id here and the callable distributes it) or `uid` (the 128 bytes,
        already on every rank — the caller then agrees on the hand-off before this collective init).  timeout_ms: the
        communicator's deadline for the init and every collective (qasr_dist_init_deadline; 0 = QASR_DIST_TIMEOUT_MS
        or 300 s) — a rank that never joins makes this one raise instead of blocking"""
        import ctypes as C

        from . import _lib

        self._lib = _lib.load()
        if uid is None:
            got = exchange(NativeComm.unique_id() if rank == 0 else bytes(128))
        else:
            got = uid
        uid = (C.c_uint8 * 128).from_buffer_copy(got)
        self._h = C.c_void_p()
        with stdout_to_stderr():
            _lib.check(self._lib.qasr_dist_init_deadline(uid, rank, world, device, C.c_double(timeout_ms),
                                                         C.byref(self._h)))
        self.rank, self.world = rank, world

    @staticmethod
    def unique_id() -> bytes:
        """rank 0: a fresh 128-byte RCCL unique id (qasr_dist_unique_id)"""
        import ctypes as C

        from . import _lib

        lib = _lib.load()
        uid = (C.c_uint8 * 128)()
        with stdout_to_stderr():
            _lib.check(lib.qasr_dist_unique_id(uid, 128))
        return bytes(uid)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.qasr_dist_close(self._h)
            self._h = None

    def broadcast_weights(self, model, root: int = 0) -> dict:
        """rank `root`'s model blob into every other rank's shell; checksums compared inside (error if any differs)"""
        import ctypes as C

        from . import _lib

        class Info(C.Structure):
            _fields_ = [("bytes", C.c_uint64), ("ms", C.c_double), ("checksum", C.c_uint64),
                        ("checksums_agree", C.c_int32)]

        info = Info()
        _lib.check(self._lib.qasr_dist_broadcast_weights(self._h, model._h, root, C.byref(info)))
        return {"bytes": int(info.bytes), "ms": round(info.ms, 3), "native_rccl": True,
                "GB_per_s": round(info.bytes / info.ms / 1e6, 1) if info.ms > 0 else None,
                "checksums_agree": bool(info.checksums_agree)}

    def agree(self, failed: bool) -> bool:
        """qasr_dist_agree: every rank's local outcome over RCCL; True on every rank if any rank failed"""
        import ctypes as C

        from . import _lib

        anyf = C.c_int32(0)
        _lib.check(self._lib.qasr_dist_agree(self._h, 1 if failed else 0, C.byref(anyf)))
        return bool(anyf.value)

    def broadcast(self, send_ptr, recv_ptr: int, nbytes: int, root: int = 0):
        from . import _lib

        _lib.check(self._lib.qasr_dist_broadcast(self._h, send_ptr, recv_ptr, nbytes, root))

    def gather_tokens(self, streams: list[list[int]]) -> list[list[list[int]]]:
        """every rank's per-segment token ids → [rank][segment] -> ids, on every rank"""
        import ctypes as C

        from . import _lib

        lens = np.array([len(x) for x in streams], np.int32)
        flat = np.concatenate([np.asarray(x, np.int32) for x in streams]) if lens.sum() else np.zeros(1, np.int32)
        rank_segs = (C.c_int32 * self.world)()
        ns, nt = C.c_size_t(0), C.c_size_t(0)
        vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        _lib.check(self._lib.qasr_dist_gather_tokens(self._h, vp(lens) if lens.size else None, int(lens.size),
                                                     vp(flat), rank_segs, None, 0, None, 0, C.byref(ns),
                                                     C.byref(nt)))
        al = np.zeros(max(1, ns.value), np.int32)
        at = np.zeros(max(1, nt.value), np.int32)
        _lib.check(self._lib.qasr_dist_gather_tokens(self._h, vp(lens) if lens.size else None, int(lens.size),
                                                     vp(flat), rank_segs, vp(al), al.size, vp(at), at.size,
                                                     C.byref(ns), C.byref(nt)))
        out, s0, t0 = [], 0, 0
        for r in range(self.world):
            segs = []
            for ln in al[s0:s0 + rank_segs[r]]:
                segs.append(at[t0:t0 + int(ln)].tolist())
                t0 += int(ln)
            s0 += rank_segs[r]
            out.append(segs)
        return out


def file_exchange(rank: int, world: int, key: str | None = None, directory: str | None = None,
                  timeout_s: float = 600.0):
    """The unique-id hand-off without PyTorch (one node): returns `exchange(payload) -> bytes` for NativeComm.  Rank 0
    publishes its bytes in `<directory>/qasr_uid_<key>.bin` — written under a temporary name and renamed, so a reader
    never sees a partial file — and every other rank polls for the file.  This is what a host without torch (the Rust
    app) does with a file or a pipe of its own.  `key` defaults to the launcher's rendezvous
    (TORCHELASTIC_RUN_ID + MASTER_PORT + the launcher's pid, fresh for every launch; $QASR_RDV_KEY overrides),
    `directory` to $QASR_RDV_DIR or the temp dir.
    Rank 0 removes the file once its communicator exists (ncclCommInitRank returns only when every rank joined, i.e.
    after every rank has read it): call `exchange.cleanup()` then."""
    import os
    import tempfile

    if key is None:
        # the launch's rendezvous + the launcher's pid (torchrun's agent is every rank's parent): a file a crashed
        # earlier launch left behind under the same run id and port is never taken for this one's.  QASR_RDV_KEY
        # overrides (ranks started by separate launchers)
        key = os.environ.get("QASR_RDV_KEY") or (f"{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}_"
                                                 f"{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}")
    directory = directory or os.environ.get("QASR_RDV_DIR") or tempfile.gettempdir()
    path = os.path.join(directory, f"qasr_uid_{key}.bin")

    def exchange(payload: bytes) -> bytes:
        if world == 1:
            return payload
        if rank == 0:
            try:   # a stale marker of an earlier launch under the same key
                os.remove(path + ".fail")
            except FileNotFoundError:
                pass
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(payload)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, path)
            return payload
        t0 = time.monotonic()
        while True:
            try:
                with open(path, "rb") as f:
                    got = f.read()
                if len(got) == len(payload):
                    return got
            except FileNotFoundError:
                pass
            if os.path.exists(path + ".fail"):
                raise RuntimeError(f"rank {rank}: rank 0 failed to publish the unique id")
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError(f"rank {rank}: no unique id at {path} after {timeout_s:.0f} s")
            time.sleep(0.01)

    def cleanup():
        if rank == 0:
            for p in (path, path + ".fail"):
                try:
                    os.remove(p)
                except FileNotFoundError:
                    pass

    def fail():
        """rank 0 could not create or publish the id: a marker file, so the other ranks stop polling at once"""
        if rank == 0:
            with open(path + ".fail", "wb"):
                pass

    exchange.cleanup = cleanup
    exchange.fail = fail
    exchange.path = path
    return exchange


def torch_exchange(payload: bytes) -> bytes:
    """rank 0's bytes on every rank over the initialised torch.distributed group (the unique-id hand-off)"""
    import torch.distributed as dist

    box = [payload if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]
