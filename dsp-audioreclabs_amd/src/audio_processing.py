"""Drop-in for the reference's src/audio_processing.py on MI355X.

Same function names, arguments, return types and error behaviour as the reference
(Hypersonic-cpu/DSP-AudioRecLabs src/audio_processing.py).  WAV decoding is host file I/O, as
in the reference.  ``process_audio_file`` -- the function the reference's callers use
(experiments/run_experiments.py:90-99) -- runs the fused gfx950 kernel (csrc/extract.hip) for
preprocess + endpoint detection + framing + E/M/ZCR in one launch and returns the frames as a
``DeviceFrames`` object that ``feature_extraction.extract_features_from_frames`` consumes
without recomputing anything.  The per-array helpers (remove_dc ... frame_signal) are kept for
callers that use them directly (plots, notebooks); they run as float64 torch ops on the HIP
device.  There is no CPU fallback: without a GPU every entry point raises ``HipError``.
"""
import wave

import numpy as np

from . import _hip
from .pipeline import FeatureExtractor, create_window  # noqa: F401  (create_window: :278-296)


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


def _read_wav_module(filepath):
    """The reference's reader (src/audio_processing.py:20-28): Python's wave module."""
    with wave.open(filepath, "rb") as w:
        n_channels = w.getnchannels()
        sample_width = w.getsampwidth()
        sample_rate = w.getframerate()
        raw = w.readframes(w.getnframes())
    return raw, sample_width, n_channels, sample_rate


def _parse_riff(buf):
    """The data bytes and format of a well-formed PCM WAV image, exactly what wave.open +
    readframes(getnframes()) return for it (RIFF/WAVE header, chunks padded to even sizes, 'fmt '
    with WAVE_FORMAT_PCM before 'data', nframes = data size // frame size); None for anything
    else -- the caller then takes the wave module itself, errors and all.  The walk is bounded by
    the RIFF chunk as well as the file: wave reads every subchunk through the RIFF chunk, so a RIFF
    size below 4 is 'not a WAVE file' and a RIFF size ending inside the data truncates the samples;
    such files go to the wave module."""
    if len(buf) < 12 or buf[0:4] != b"RIFF" or buf[8:12] != b"WAVE":
        return None
    riff = int.from_bytes(buf[4:8], "little")
    if riff < 4:
        return None
    p, n, fmt = 12, min(len(buf), 8 + riff), None
    while p + 8 <= n:
        cid, size = buf[p:p + 4], int.from_bytes(buf[p + 4:p + 8], "little")
        body = p + 8
        if cid == b"fmt ":
            if size < 16 or body + 16 > n:
                return None
            tag, ch, sr = int.from_bytes(buf[body:body + 2], "little"), int.from_bytes(buf[body + 2:body + 4], "little"), \
                int.from_bytes(buf[body + 4:body + 8], "little")
            bits = int.from_bytes(buf[body + 14:body + 16], "little")
            if tag != 1 or ch == 0 or bits == 0:
                return None
            fmt = (ch, (bits + 7) // 8, sr)
        elif cid == b"data":
            if fmt is None:
                return None
            ch, sw, sr = fmt
            nbytes = (size // (ch * sw)) * ch * sw
            if body + nbytes > n:  # truncated file: the wave module's own behaviour
                return None
            return memoryview(buf)[body:body + nbytes], sw, ch, sr
        p = body + size + (size & 1)
    return None


def _read_wav(filepath):
    """(data bytes, sample width, channels, sample rate) of a WAV file: one read and a RIFF chunk
    walk for well-formed PCM files, the wave module (the reference's reader) for anything else."""
    with open(filepath, "rb") as f:
        buf = f.read()
    r = _parse_riff(buf)
    return r if r is not None else _read_wav_module(filepath)


def load_wav(filepath):
    """src/audio_processing.py:9-46 -> (audio float64 in [-1, 1], sample_rate)."""
    raw, sw, ch, sr = _read_wav(filepath)
    audio, _, _ = decode_pcm_bytes(raw, sw, ch)
    return audio, sr


def load_wav_pcm(filepath):
    """GPU-path form of load_wav: (integer samples, sample_rate).

    The samples are ``ints`` of decode_pcm_bytes (load_wav's audio up to a power-of-two scale,
    which preprocess cancels): int16 for 16-bit mono and 8-bit mono/stereo; for 16-bit stereo the
    channel sums, int16 when they fit and int32 otherwise (17 bits: dsp_extract_general)."""
    raw, sw, ch, sr = _read_wav(filepath)
    if sw == 2 and ch == 1:  # the common case: the payload itself, no conversion
        return np.frombuffer(raw, dtype=np.int16), sr
    _, ints, _ = decode_pcm_bytes(raw, sw, ch)
    if ints.size and (ints.max() > 32767 or ints.min() < -32768):
        return ints.astype(np.int32), sr
    return ints.astype(np.int16), sr


# ---------------------------------------------------------------- fused path
class DeviceFrames:
    """The windowed frames of one processed clip (frame_signal, :299-333), kept implicit.

    The fused kernel computed everything extract_features_from_frames needs; ``features``
    holds the per-frame (E, M, ZCR) sequences and ``vector`` the 15-d statistics.  Indexing,
    ``len`` and ``np.asarray`` behave like the reference's float64 [n_frames, frame_length]
    array; materialising it (rarely needed: plots) runs on the device.
    """

    def __init__(self, pcm, start, end, frame_length, frame_shift, window_type, features, vector):
        self._pcm = pcm  # int16 numpy, the whole clip
        self.start, self.end = int(start), int(end)
        self.frame_length, self.frame_shift = int(frame_length), int(frame_shift)
        self.window_type = window_type
        self.features = features  # dict energy / magnitude / zcr -> float64 [n_frames]
        self.vector = vector      # float64 [15]
        self.n_frames = len(features["energy"])

    def __len__(self):
        return self.n_frames

    @property
    def shape(self):
        return (self.n_frames, self.frame_length)

    def materialize(self):
        import torch
        d = _hip.require_device()
        k = torch.as_tensor(self._pcm.astype(np.float64), device=d)
        audio = preprocess(k)[self.start:self.end]
        return frame_signal(audio, self.frame_length, self.frame_shift, self.window_type).cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.materialize()
        return a if dtype is None else a.astype(dtype)

    def __getitem__(self, idx):
        return self.materialize()[idx]

    def __iter__(self):
        return iter(self.materialize())


_extractors = {}


def _extractor(frame_length, frame_shift, window_type, do_vad, hi, lo, zr):
    key = (frame_length, frame_shift, window_type, bool(do_vad), hi, lo, zr)
    if key not in _extractors:
        _extractors[key] = FeatureExtractor(frame_length, frame_shift, window_type, do_vad, hi, lo, zr,
                                            return_vad_lists=True, return_sequences=True)
    return _extractors[key]


_ERRORS = {
    _hip.CLIP_EMPTY: "zero-size array to reduction operation maximum which has no identity",
    _hip.CLIP_NO_AUDIO: "No audio remaining after preprocessing and endpoint detection.",
    _hip.CLIP_NO_FRAMES: "No frames provided for feature extraction.",
    _hip.CLIP_TOO_LONG: "clip longer than the device pipeline supports",
    _hip.CLIP_UNCERTIFIED: "endpoint decision could not be certified",
}


def _len_bucket(n, cap):
    """n rounded up to 1/8-octave steps; not past the fused plan's cap when n itself fits it."""
    step = 1 << max(0, int(n).bit_length() - 3)
    m = -(-int(n) // step) * step
    return min(m, cap) if n <= cap else m


def process_audio_file(filepath, frame_length, frame_shift,
                       window_type='hamming',
                       do_endpoint_detection=True,
                       energy_high_ratio=0.5,
                       energy_low_ratio=0.1,
                       zcr_threshold_ratio=1.5):
    """src/audio_processing.py:336-396 -> (frames, sample_rate, metadata), one fused launch.

    ``frames`` is a DeviceFrames (see above); ``metadata`` has the reference's keys
    (original_length, sample_rate, start_point, end_point, energy_list, zcr_list,
    segmented_length when endpoint detection is on, n_frames).  Errors raise ValueError with
    the reference's messages.
    """
    pcm, sr = load_wav_pcm(filepath)
    return process_pcm(pcm, sr, frame_length, frame_shift, window_type, do_endpoint_detection,
                       energy_high_ratio, energy_low_ratio, zcr_threshold_ratio)


def process_pcm(pcm, sample_rate, frame_length, frame_shift, window_type='hamming',
                do_endpoint_detection=True, energy_high_ratio=0.5, energy_low_ratio=0.1,
                zcr_threshold_ratio=1.5):
    """process_audio_file on integer samples already in memory (int16, or int32 for 16-bit
    stereo channel sums)."""
    if window_type not in ("rectangular", "hamming", "hanning"):
        create_window(window_type, 1)  # raises the reference's ValueError
    pcm = np.ascontiguousarray(pcm, dtype=np.int32 if np.asarray(pcm).dtype == np.int32 else np.int16)
    n = pcm.size
    if n == 0:
        raise ValueError(_ERRORS[_hip.CLIP_EMPTY])
    fx = _extractor(int(frame_length), int(frame_shift), window_type, do_endpoint_detection,
                    float(energy_high_ratio), float(energy_low_ratio), float(zcr_threshold_ratio))
    # the launch is sized for a length bucket (1/8 octave, clamped to the fused kernel's plan), so
    # a caller looping over files of similar lengths, as the reference's experiments do
    # (experiments/run_experiments.py:82-111), reuses one set of device output buffers
    out = {k: v.cpu().numpy() for k, v in fx(pcm.reshape(1, -1), max_len=_len_bucket(n, fx.fused_cap())).items()}
    st = int(out["status"][0]) & 0xFF
    if st:
        raise ValueError(_ERRORS.get(st, "clip rejected by the device path (status %d)" % st))
    start, end = (int(x) for x in out["start_end"][0])
    nf = int(out["n_frames"][0])
    seq = out["seq"][0, :nf].astype(np.float64)
    features = {"energy": seq[:, 0], "magnitude": seq[:, 1], "zcr": seq[:, 2]}
    frames = DeviceFrames(pcm, start, end, frame_length, frame_shift, window_type, features,
                          out["feat"][0].astype(np.float64))
    metadata = {"original_length": n, "sample_rate": sample_rate}
    if do_endpoint_detection:
        nv = (n - frame_length) // frame_shift + 1 if n >= frame_length else 0
        metadata.update({
            "start_point": start,
            "end_point": end,
            "energy_list": out["vad_energy"][0, :nv].astype(np.float64),
            "zcr_list": out["vad_zcr"][0, :nv].astype(np.float64),
            "segmented_length": end - start,
        })
    metadata["n_frames"] = nf
    return frames, sample_rate, metadata


# ---------------------------------------------------------------- per-array helpers (device)
# The reference's building blocks (:49-333) as float64 torch ops on the HIP device, for callers
# that use them one array at a time.  The fused kernel above is the hot path.
def _dev(x):
    import torch
    d = _hip.require_device()
    if isinstance(x, torch.Tensor):
        return x.to(device=d, dtype=torch.float64)
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=d)


def _out(t, like):
    import torch
    if isinstance(like, torch.Tensor):
        return t
    return t.cpu().numpy() if t.dim() else float(t.item())


def remove_dc(audio_data):
    """:49-59"""
    x = _dev(audio_data)
    return _out(x - x.mean(), audio_data)


def normalize_audio(audio_data):
    """:62-75"""
    x = _dev(audio_data)
    m = x.abs().max()
    return _out(x / m if m > 0 else x, audio_data)


def preprocess(audio_data):
    """:78-90"""
    return normalize_audio(remove_dc(audio_data))


def compute_short_time_energy(frame):
    """:93-103 (sum of squares)"""
    x = _dev(frame)
    return _out((x * x).sum(), frame)


def compute_short_time_magnitude(frame):
    """:106-116 (sum of |x|)"""
    x = _dev(frame)
    return _out(x.abs().sum(), frame)


def compute_zero_crossing_rate(frame):
    """:119-132 (sign with 0 -> -1, half the sum of |diff|)"""
    import torch
    x = _dev(frame)
    s = torch.where(x > 0, 1.0, -1.0).to(torch.float64)
    return _out((s[1:] - s[:-1]).abs().sum() / 2, frame)


def frame_signal(audio_data, frame_length, frame_shift, window_type='hamming'):
    """:299-333 -> windowed frames [n_frames, frame_length] (last frame zero-padded)."""
    import torch
    x = _dev(audio_data)
    n = x.numel()
    w = _dev(create_window(window_type, frame_length))
    if n == 0:
        return _out(torch.zeros((0, frame_length), dtype=torch.float64, device=x.device), audio_data)
    nf = 1 if n <= frame_length else int(np.ceil((n - frame_length) / frame_shift)) + 1
    need = (nf - 1) * frame_shift + frame_length
    xp = torch.cat([x, x.new_zeros(max(0, need - n))])
    frames = xp.unfold(0, frame_length, frame_shift)[:nf] * w
    return _out(frames, audio_data)


def endpoint_detection(audio_data, frame_length, frame_shift,
                       energy_high_ratio=0.5, energy_low_ratio=0.1, zcr_threshold_ratio=1.5):
    """:135-275 on a preprocessed float64 signal -> (start, end, energy_list, zcr_list).

    The fused kernel decides endpoints bit-exactly from the integer samples; this helper takes
    an arbitrary float64 signal, so its frame energies are device float64 sums (numpy sums in a
    different order: last-bit differences can only matter for a threshold tie)."""
    import torch
    x = _dev(audio_data)
    n = x.numel()
    if n < frame_length:
        return 0, n, np.array([]), np.array([])
    nfr = (n - frame_length) // frame_shift + 1
    fr = x.unfold(0, frame_length, frame_shift)[:nfr]
    E = (fr * fr).sum(dim=1).cpu().numpy()
    s = torch.where(fr > 0, 1.0, -1.0).to(torch.float64)
    Z = ((s[:, 1:] - s[:, :-1]).abs().sum(dim=1) / 2).cpu().numpy()
    k = min(5, nfr // 10)
    noise_e = np.mean(np.concatenate([E[:k], E[-k:]])) if k > 0 else np.min(E)
    speech_e = np.percentile(E, 90)
    t1 = speech_e * energy_high_ratio
    hi = np.nonzero(E > t1)[0]
    if hi.size == 0:
        return 0, n, E, Z
    n3, n4 = int(hi[0]), int(hi[-1])
    t2 = noise_e + (speech_e - noise_e) * energy_low_ratio
    n2 = 0
    for i in range(n3 - 1, -1, -1):
        if E[i] <= t2:
            n2 = i + 1
            break
    n5 = nfr - 1
    for i in range(n4 + 1, nfr):
        if E[i] <= t2:
            n5 = i - 1
            break
    noise_z = np.mean(np.concatenate([Z[:k], Z[-k:]])) if k > 0 else np.min(Z)
    tz = noise_z * zcr_threshold_ratio
    n1 = 0
    for i in range(n2 - 1, -1, -1):
        if Z[i] <= tz:
            n1 = i + 1
            break
    n6 = nfr - 1
    for i in range(n5 + 1, nfr):
        if Z[i] <= tz:
            n6 = i - 1
            break
    return n1 * frame_shift, min(n6 * frame_shift + frame_length, n), E, Z
