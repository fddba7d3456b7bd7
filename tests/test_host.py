"""Host-side logic of the drop-in layer: windows, WAV decoding, synthetic data, sharding."""
import io
import wave

import numpy as np
import pytest


def test_windows_match_numpy():
    from src.pipeline import create_window
    for L in (1, 2, 1024, 1102):
        assert np.array_equal(create_window("hamming", L), np.hamming(L))
        assert np.array_equal(create_window("hanning", L), np.hanning(L))
        assert np.array_equal(create_window("rectangular", L), np.ones(L))
    with pytest.raises(ValueError):
        create_window("kaiser", 16)


def _wav_bytes(data, width, channels, sr=44100):
    b = io.BytesIO()
    with wave.open(b, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes(data.tobytes())
    b.seek(0)
    return b


def test_decode_matches_reference_formula():
    """load_wav (src/audio_processing.py:31-44): 8-bit via uint8 arithmetic (wraps), 16-bit /32768,
    stereo = channel mean; the integer form times the scale is the float64 audio exactly."""
    from src.audio_processing import decode_pcm_bytes
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, 1000, dtype=np.uint8)
    a, ints, sc = decode_pcm_bytes(u8.tobytes(), 1, 1)
    assert np.array_equal(a, (u8 - 128).astype(np.float64) / 128.0)  # numpy uint8 wrap, as the reference
    assert np.array_equal(ints * sc, a)
    s16 = rng.integers(-32768, 32768, 2000, dtype=np.int16)
    a, ints, sc = decode_pcm_bytes(s16.tobytes(), 2, 2)
    ref = np.mean(s16.astype(np.float64).reshape(-1, 2) / 32768.0, axis=1)
    assert np.array_equal(a, ref)
    assert np.array_equal(ints * sc, a)
    with pytest.raises(ValueError):
        decode_pcm_bytes(b"\0" * 12, 3, 1)


def test_load_wav_pcm_roundtrip(tmp_path):
    from src.audio_processing import load_wav, load_wav_pcm
    x = (np.arange(-500, 500) * 31).astype(np.int16)
    p = tmp_path / "a.wav"
    p.write_bytes(_wav_bytes(x, 2, 1).read())
    pcm, sr = load_wav_pcm(str(p))
    a, sr2 = load_wav(str(p))
    assert sr == sr2 == 44100 and np.array_equal(pcm, x) and np.array_equal(a, x / 32768.0)


def test_synth_is_shardable():
    from src.synth import make_batch, make_clip
    full = make_batch(12, base_seed=5)
    part = make_batch(5, base_seed=5, start=7)
    assert np.array_equal(full[7:], part)
    assert np.array_equal(make_clip(5 + 3), full[3])
    x, y = make_batch(20, with_labels=True)
    assert np.array_equal(y, np.arange(20) % 10)


def test_shard_range_partitions():
    from src.distributed import shard_range
    for total in (0, 1, 7, 1000, 100000):
        for ws in (1, 2, 3, 8):
            spans = [shard_range(total, r, ws) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _riff(chunks):
    body = b"WAVE" + b"".join(cid + len(d).to_bytes(4, "little") + d + (b"\0" if len(d) & 1 else b"")
                              for cid, d in chunks)
    return b"RIFF" + len(body).to_bytes(4, "little") + body


def _riff_size(blob, size):
    """blob with its RIFF size field replaced (the wave module reads every chunk through it)"""
    return blob[:4] + int(size).to_bytes(4, "little") + blob[8:]


def _fmt(tag, ch, sr, bits):
    import struct
    return struct.pack("<HHLLHH", tag, ch, sr, sr * ch * ((bits + 7) // 8), ch * ((bits + 7) // 8), bits)


def test_riff_reader_equals_wave_module(tmp_path):
    """The one-read RIFF walk (load_wav_pcm's reader) returns exactly what the reference's
    wave.open + readframes(getnframes()) returns (src/audio_processing.py:20-28), and files it does
    not take (non-PCM, data before fmt, truncated) go to the wave module with its errors."""
    from src.audio_processing import _read_wav, _read_wav_module, load_wav_pcm
    rng = np.random.default_rng(1)
    pcm = rng.integers(-32768, 32768, 2001, dtype=np.int16).tobytes()
    cases = {
        "mono16": _riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]),
        "stereo16_partial_frame": _riff([(b"fmt ", _fmt(1, 2, 22050, 16)), (b"data", pcm)]),  # 4002 B: 1000 frames + 2
        "mono8_odd_list": _riff([(b"fmt ", _fmt(1, 1, 8000, 8)), (b"LIST", b"abc"), (b"data", pcm[:777])]),
        "fmt18": _riff([(b"fmt ", _fmt(1, 1, 44100, 16) + b"\0\0"), (b"data", pcm[:100])]),
        "float": _riff([(b"fmt ", _fmt(3, 1, 44100, 32)), (b"data", pcm[:400])]),
        "data_first": _riff([(b"data", pcm[:100]), (b"fmt ", _fmt(1, 1, 44100, 16))]),
        "truncated": _riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)])[:-500],
        "bits24": _riff([(b"fmt ", _fmt(1, 1, 44100, 24)), (b"data", pcm[:999])]),
        "not_riff": b"RIFX" + b"\0" * 40,
        # RIFF size field 0 / ending inside the data / ending inside the fmt chunk / too large
        "riff0": _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 0),
        "riff_short_data": _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 4 + 24 + 8 + 1001),
        "riff_short_fmt": _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 4 + 8 + 10),
        "riff_large": _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 1 << 30),
    }
    for name, blob in cases.items():
        p = tmp_path / (name + ".wav")
        p.write_bytes(blob)
        try:
            want = _read_wav_module(str(p))
        except Exception as e:  # noqa: BLE001
            with pytest.raises(type(e)):
                _read_wav(str(p))
            continue
        got = _read_wav(str(p))
        assert bytes(got[0]) == bytes(want[0]) and tuple(got[1:]) == tuple(want[1:]), name
    x = np.frombuffer(pcm, np.int16)
    got, sr = load_wav_pcm(str(tmp_path / "mono16.wav"))
    assert sr == 44100 and got.dtype == np.int16 and np.array_equal(got, x)


def test_native_wav_reader_equals_python_reader(tmp_path):
    """The library's batch reader (dsp_wav_scan / dsp_wav_read, host only: no GPU) takes exactly
    the mono 8/16-bit PCM files the RIFF walk takes and yields load_wav_pcm's samples for them;
    everything else goes to the Python reader, so read_packed's kept files, skip reasons and
    packed samples equal those of the pure-Python path (native=False)."""
    from src import _hip
    from src.audio_processing import load_wav_pcm
    from src.dataset import read_packed
    rng = np.random.default_rng(3)
    pcm = rng.integers(-32768, 32768, 4001, dtype=np.int16).tobytes()
    u8 = rng.integers(0, 256, 3333, dtype=np.uint8).tobytes()
    cases = [
        ("mono16", _riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)])),
        ("mono16_odd_bytes", _riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm[:1001])])),
        ("mono8_odd_list", _riff([(b"fmt ", _fmt(1, 1, 8000, 8)), (b"LIST", b"abc"), (b"data", u8)])),
        ("stereo16", _riff([(b"fmt ", _fmt(1, 2, 22050, 16)), (b"data", pcm)])),
        ("stereo8", _riff([(b"fmt ", _fmt(1, 2, 8000, 8)), (b"data", u8[:3332])])),
        ("fmt18", _riff([(b"fmt ", _fmt(1, 1, 44100, 16) + b"\0\0"), (b"data", pcm[:100])])),
        ("float", _riff([(b"fmt ", _fmt(3, 1, 44100, 32)), (b"data", pcm[:400])])),
        ("data_first", _riff([(b"data", pcm[:100]), (b"fmt ", _fmt(1, 1, 44100, 16))])),
        ("truncated", _riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)])[:-500]),
        ("empty", _riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", b"")])),
        ("not_riff", b"RIFX" + b"\0" * 40),
        ("riff0", _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 0)),
        ("riff_short_data", _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 4 + 24 + 8 + 1001)),
        ("riff_large", _riff_size(_riff([(b"fmt ", _fmt(1, 1, 44100, 16)), (b"data", pcm)]), 1 << 30)),
    ]
    paths = []
    for name, blob in cases * 3:  # repeated: several threads, chunks of 8 files
        p = tmp_path / ("%s_%d.wav" % (name, len(paths)))
        p.write_bytes(blob)
        paths.append(str(p))
    L = _hip.load_library()
    n = len(paths)
    kind, ns, off = np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64)
    from src.dataset import _cpaths
    assert L.dsp_wav_scan(_cpaths(paths), n, 4, kind.ctypes.data, ns.ctypes.data, off.ctypes.data) == 0
    native = {"mono16": 1, "mono16_odd_bytes": 1, "mono8_odd_list": 2, "fmt18": 1, "empty": 1, "riff_large": 1}
    for p, k, m in zip(paths, kind, ns):
        name = p.rsplit("/", 1)[1].rsplit("_", 1)[0]
        assert k == native.get(name, 0), name
        if k:
            assert m == load_wav_pcm(p)[0].size, name
    a = read_packed(paths, 4, pinned=False)
    b = read_packed(paths, 1, pinned=False, native=False)
    assert a[0] == b[0] and a[1] == b[1]
    assert len(a[2]) == len(b[2]) == 2  # int16 clips, then the int32 stereo sums
    for (pa, ba, oa), (pb, bb, ob) in zip(a[2], b[2]):
        assert np.array_equal(pa, pb) and np.array_equal(oa, ob) and torch_equal(ba, bb)
    for q, i in enumerate(a[0]):  # every kept clip's samples equal load_wav_pcm's
        for pos, buf, o in a[2]:
            j = np.nonzero(pos == q)[0]
            if j.size:
                got = buf.numpy()[o[j[0]]:o[j[0] + 1]]
                want = load_wav_pcm(paths[i])[0]
                assert np.array_equal(got.astype(np.int64), want.astype(np.int64)), paths[i]


def torch_equal(x, y):
    return x.dtype == y.dtype and bool((x == y).all())
