"""Long-form audio across ranks (SURVEY §8(e) "Long-form VAD", §8(d) C5): every rank runs FireRedVAD on one
contiguous frame range of the recording plus a ±160-frame halo — the DFSMN's receptive field (8 memory blocks of
19 look-back / 20 look-ahead taps) — so its core probabilities are bit-identical to one pass over the whole
recording; one all-gather (RCCL) assembles the probability vector on every rank, the host segmenter
(`_timestamps_from_probabilities`, firered_vad.py:121-191, a sequential state machine) runs on it identically
everywhere, and the speech segments are LPT-sharded over the ranks for ASR.  The reference runs none of this: it
handles one short utterance per request.
"""
from __future__ import annotations

import numpy as np

FRAME_SHIFT, FRAME_LEN = 160, 400
HALO = 160   # frames: ≥ the DFSMN receptive field on either side


def n_frames(n_samples: int) -> int:
    """Kaldi snip_edges frame count (firered_vad.py:87-104: 25 ms / 10 ms at 16 kHz)"""
    return 0 if n_samples < FRAME_LEN else 1 + (n_samples - FRAME_LEN) // FRAME_SHIFT


def frame_shard(total_frames: int, rank: int, world: int):
    """core frame range [f0, f1) of `rank` and the halo-extended range [h0, h1) whose samples it reads"""
    f0 = total_frames * rank // world
    f1 = total_frames * (rank + 1) // world
    return f0, f1, max(0, f0 - HALO), min(total_frames, f1 + HALO)


def shard_probabilities(vad, audio: np.ndarray, rank: int, world: int) -> np.ndarray:
    """this rank's core-frame probabilities, computed from its halo-extended sample range"""
    T = n_frames(audio.size)
    f0, f1, h0, h1 = frame_shard(T, rank, world)
    if f1 <= f0:
        return np.zeros(0, np.float32)
    pcm = audio[h0 * FRAME_SHIFT: (h1 - 1) * FRAME_SHIFT + FRAME_LEN]
    p = vad.probabilities(pcm)
    assert p.size == h1 - h0, (p.size, h1 - h0)
    return p[f0 - h0: f1 - h0]


def gather_probabilities(local: np.ndarray, device) -> np.ndarray:
    """all-gather of the ranks' core probabilities, in rank (= time) order"""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    n = torch.tensor([local.size], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    buf = torch.zeros(max(1, max(ns)), dtype=torch.float32, device=device)
    buf[: local.size] = torch.from_numpy(local).to(device)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return np.concatenate([p[:k].cpu().numpy() for p, k in zip(parts, ns)])


def segments(probs: np.ndarray, n_samples: int, options=None):
    """speech segments [(start, end)] in samples (the reference's post-processing, on the host)"""
    from qasr.firered_vad import timestamps_from_probabilities

    return [(int(s["start"]), int(s["end"])) for s in timestamps_from_probabilities(probs, n_samples, options)]
