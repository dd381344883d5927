"""Drop-in for the reference FireRedVad class (src-tauri/resources/firered_vad.py) on libqasr (HIP).

Same constructor / options / methods as the reference:
    FireRedVad(model_path=None, cmvn_path=None, options=None)      # firered_vad.py:41-85
    .probabilities(audio) -> np.ndarray[T] float32                 # :106-111
    .warmup()                                                      # :113-114
    .speech_timestamps(audio) -> [{"start", "end"}]                # :116-119
    ._timestamps_from_probabilities(probs, audio_length_samples)   # :121-191
model_path may be the repo's .qvad container (tools/convert_vad.py); cmvn_path is accepted for API parity
(the container carries the CMVN statistics).  The segmenter runs in libqasr (host code) so the
post-processing is the same function the native engine uses.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import Segment, VadOptions, check

SAMPLE_RATE = 16_000
FRAME_SHIFT_SAMPLES = 160
FRAME_LENGTH_SAMPLES = 400


@dataclass(frozen=True)
class FireRedVadOptions:
    threshold: float = 0.5
    smooth_window_frames: int = 5
    min_speech_duration_ms: int = 150
    min_silence_duration_ms: int = 300
    speech_pad_ms: int = 120


def _opts(o: FireRedVadOptions) -> VadOptions:
    return VadOptions(float(o.threshold), int(o.smooth_window_frames), int(o.min_speech_duration_ms),
                      int(o.min_silence_duration_ms), int(o.speech_pad_ms))


def timestamps_from_probabilities(probs, audio_length_samples: int, options: FireRedVadOptions | None = None):
    p = np.ascontiguousarray(np.asarray(probs, dtype=np.float32).reshape(-1))
    cap = max(1, p.size)
    segs = (Segment * cap)()
    n = C.c_size_t()
    check(_lib.load().qasr_vad_timestamps_from_probabilities(p.ctypes.data_as(C.c_void_p), p.size,
                                                             int(audio_length_samples),
                                                             C.byref(_opts(options or FireRedVadOptions())), segs,
                                                             cap, C.byref(n)))
    return [{"start": int(segs[i].start), "end": int(segs[i].end)} for i in range(n.value)]


class FireRedVad:
    def __init__(self, model_path=None, cmvn_path=None, options: FireRedVadOptions | None = None):
        self.options = options or FireRedVadOptions()
        self.model_path = str(model_path) if model_path else _lib.VAD_ASSET
        self.cmvn_path = cmvn_path
        self._h = C.c_void_p()
        check(_lib.load().qasr_vad_open(self.model_path.encode(), C.byref(self._h)))

    def features(self, audio) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(audio, dtype=np.float32).reshape(-1))
        t = 1 + (a.size - 400) // 160 if a.size >= 400 else 0
        out = np.empty((t, 80), np.float32)
        n = C.c_size_t()
        check(_lib.load().qasr_vad_features(self._h, a.ctypes.data_as(C.c_void_p), a.size,
                                            out.ctypes.data_as(C.c_void_p), t, C.byref(n)))
        return out[: n.value]

    def probabilities(self, audio) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(audio, dtype=np.float32).reshape(-1))
        t = 1 + (a.size - 400) // 160 if a.size >= 400 else 0
        out = np.empty(t, np.float32)
        n = C.c_size_t()
        check(_lib.load().qasr_vad_probabilities(self._h, a.ctypes.data_as(C.c_void_p), a.size,
                                                 out.ctypes.data_as(C.c_void_p), t, C.byref(n)))
        return out[: n.value]

    def warmup(self) -> None:
        self.probabilities(np.zeros(SAMPLE_RATE, dtype=np.float32))

    def speech_timestamps(self, audio):
        samples = np.asarray(audio, dtype=np.float32).reshape(-1)
        return self._timestamps_from_probabilities(self.probabilities(samples), len(samples))

    def _timestamps_from_probabilities(self, raw_probabilities, audio_length_samples: int):
        return timestamps_from_probabilities(raw_probabilities, audio_length_samples, self.options)

    def close(self):
        if self._h:
            _lib.load().qasr_vad_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
