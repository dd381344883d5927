"""qasr — host-side Python mirror of the light-whisper local ASR plugin interface over libqasr (HIP).

Modules:
  _lib          ctypes binding of include/qasr.h (fails loudly when libqasr.so is absent)
  transcribe_cpp  drop-in for the `transcribe_cpp` API the reference server binds (Model/session/run/close)
  firered_vad   drop-in for the reference FireRedVad class (probabilities / speech_timestamps)
"""
from ._lib import load, check, QasrError  # noqa: F401
