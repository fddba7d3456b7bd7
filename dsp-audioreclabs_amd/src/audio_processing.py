"""Drop-in for the reference's src/audio_processing.py on MI355X.

Same function names, arguments, return types and error behaviour as the reference
(Hypersonic-cpu/DSP-AudioRecLabs src/audio_processing.py).  WAV decoding is host I/O
(as in the reference); everything from preprocessing on runs in HIP kernels
(csrc/extract.hip, csrc/primitives.hip) -- there is no CPU fallback.
"""
import wave

import numpy as np

from . import _hip
from .pipeline import create_window  # noqa: F401  (re-exported: src/audio_processing.py:278-296)


# ---------------------------------------------------------------- WAV decoding (host I/O)
def decode_pcm_bytes(raw, sample_width, n_channels):
    """Bytes of a WAV data chunk -> (float64 audio, integer samples, scale).

    float64 audio is exactly what the reference's load_wav returns
    (src/audio_processing.py:31-44), including its uint8 arithmetic: for 8-bit files
    ``frombuffer(uint8) - 128`` stays uint8 under numpy's casting rules, i.e. it wraps to
    ``(u8 - 128) mod 256``.  ``audio == ints * scale`` exactly, and ``ints`` is what the GPU
    path consumes (any power-of-two scale cancels in preprocess()).
    """
    if sample_width == 1:
        u = np.frombuffer(raw, dtype=np.uint8)
        ints = (u ^ 0x80).astype(np.int32)  # == (u - 128) mod 256
        scale = 1.0 / 128.0
    elif sample_width == 2:
        ints = np.frombuffer(raw, dtype=np.int16).astype(np.int32)
        scale = 1.0 / 32768.0
    else:
        raise ValueError(f"不支持的采样位数: {sample_width}")
    if n_channels == 2:
        ints = ints.reshape(-1, 2).sum(axis=1)  # mean of two channels = sum * scale / 2
        scale = scale / 2.0
    audio = ints.astype(np.float64) * scale
    return audio, ints, scale


def _read_wav(filepath):
    with wave.open(filepath, "rb") as w:
        n_channels = w.getnchannels()
        sample_width = w.getsampwidth()
        sample_rate = w.getframerate()
        raw = w.readframes(w.getnframes())
    return raw, sample_width, n_channels, sample_rate


def load_wav(filepath):
    """src/audio_processing.py:9-46 -> (audio float64 in [-1, 1], sample_rate)."""
    raw, sw, ch, sr = _read_wav(filepath)
    audio, _, _ = decode_pcm_bytes(raw, sw, ch)
    return audio, sr


def load_wav_pcm(filepath):
    """GPU-path form of load_wav: (int16 samples, sample_rate).

    16-bit mono and 8-bit mono/stereo fit int16 exactly; 16-bit stereo (sums up to 17 bits)
    raises ValueError for now."""
    raw, sw, ch, sr = _read_wav(filepath)
    _, ints, _ = decode_pcm_bytes(raw, sw, ch)
    if ints.size and (ints.max() > 32767 or ints.min() < -32768):
        raise ValueError("16-bit stereo needs the int32 sample path (not built yet)")
    return ints.astype(np.int16), sr
