"""GPU parity of the general path (csrc/general.hip, dsp_extract_general): clips longer than the
fused kernel's on-chip plan and 16-bit stereo clips whose channel sums need int32 (the reference
processes both: src/audio_processing.py:35-44, :336-396), checked against the C oracle and the
reference-generated WAV goldens.  Tolerances as in test_gpu_extract.py."""
import ctypes
import wave

import numpy as np
import pytest

import oracle
from test_gpu_extract import feat_close

pytestmark = pytest.mark.gpu


def _write_wav(path, data, width=2, channels=1, sr=44100):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes(np.ascontiguousarray(data).tobytes())


def _check_clip(out, i, clip, L, S, win, vad=True, exact_se=True):
    from src.pipeline import create_window
    r = oracle.process_clip(clip if clip.dtype == np.int16 else clip.astype(np.float64), L, S,
                            create_window(win, L), do_vad=vad)
    assert (out["status"][i] & 0xFF) == r["status"], (i, out["status"][i], r["status"])
    if r["status"]:
        return r
    assert tuple(out["start_end"][i]) == (r["start"], r["end"]), (i, out["start_end"][i], r["start"], r["end"])
    assert out["n_frames"][i] == r["n_frames"], i
    assert not feat_close(out["feat"][i], r["feat"]).any(), (i, out["feat"][i], r["feat"])
    return r


def test_long_clips_mixed_with_short():
    """1 s, 3 s, 10 s and 30 s clips in one batch: the short ones on the fused kernel, the ones
    past its on-chip plan on the general kernel, in stream order, no host round trip between."""
    import torch
    from src.pipeline import FeatureExtractor
    from src.synth import make_clip
    sr = 44100
    lens = [sr, 10 * sr, 3 * sr, sr + 17, 30 * sr, 5000, 0, 10 * sr + 3]
    clips = [make_clip(900 + i, n) if n else np.zeros(0, np.int16) for i, n in enumerate(lens)]
    off = np.zeros(len(clips) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    pcm = np.concatenate(clips + [np.zeros(8, np.int16)])
    for vad in (True, False):
        fx = FeatureExtractor(1102, 441, "hamming", vad, return_vad_lists=True, return_sequences=True)
        assert 3 * sr <= fx.fused_cap() < 10 * sr
        out = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm).cuda(), off).items()}
        for i, c in enumerate(clips):
            r = _check_clip(out, i, c, 1102, 441, "hamming", vad)
            if r["status"] == 0:
                F = r["n_frames"]
                np.testing.assert_array_equal(out["seq"][i, :F, 2], r["seq"][:, 2])
                np.testing.assert_allclose(out["seq"][i, :F, 0], r["seq"][:, 0], rtol=1e-5, atol=1e-30)
                if vad:
                    nv = len(r["vad_energy"])
                    np.testing.assert_array_equal(out["vad_zcr"][i, :nv], r["vad_zcr"])
                    np.testing.assert_allclose(out["vad_energy"][i, :nv], r["vad_energy"], rtol=1e-12, atol=0)


def _general(pcm, off, L, S, win, vad=True, sample_bytes=2, nv_ld=None):
    """dsp_extract_general over every clip (min_len 0), straight through the C ABI."""
    import torch
    from src import _hip
    from src.pipeline import create_window
    lib = _hip.lib()
    B = len(off) - 1
    lens = np.diff(off)
    ml = int(lens.max())
    d = torch.device("cuda")
    t = torch.as_tensor(pcm).to(d)
    o = torch.as_tensor(off).to(d)
    w = torch.as_tensor(create_window(win, L)).to(d)
    ld = max(1, (ml - L) // S + 1) if ml >= L else 1
    out = dict(feat=torch.empty((B, 15), dtype=torch.float32, device=d),
               start_end=torch.empty((B, 2), dtype=torch.int32, device=d),
               n_frames=torch.empty(B, dtype=torch.int32, device=d),
               status=torch.empty(B, dtype=torch.int32, device=d),
               vad_energy=torch.zeros((B, ld), dtype=torch.float64, device=d),
               vad_zcr=torch.zeros((B, ld), dtype=torch.int32, device=d))
    ldf = 1 if ml <= L else (ml - L + S - 1) // S + 1
    out["seq"] = torch.zeros((B, ldf, 3), dtype=torch.float32, device=d)
    nb = lib.dsp_extract_general_workspace_bytes(B, ml, L, S)
    ws = torch.empty(nb, dtype=torch.uint8, device=d)
    P = _hip.ptr
    rc = lib.dsp_extract_general(P(t), sample_bytes, P(o), None, B, 0, ml, L, S, P(w), int(vad), 0.5, 0.1, 1.5,
                                 P(out["feat"]), P(out["start_end"]), P(out["n_frames"]), P(out["status"]), 0,
                                 P(out["vad_energy"]), P(out["vad_zcr"]), ld, P(out["seq"]), ldf, P(ws), nb,
                                 _hip.stream_handle(d))
    _hip.check(rc, "dsp_extract_general")
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("L,S,win", [(1102, 441, "hamming"), (1024, 512, "hanning"), (882, 220, "rectangular"),
                                     (2205, 441, "hamming")])
def test_general_kernel_vs_oracle_and_fused(L, S, win):
    """The general kernel on ordinary clips (ragged, short, silent, near-tie) equals the oracle,
    and the fused kernel on the same batch."""
    import torch
    from src.pipeline import FeatureExtractor
    from src.synth import make_clip
    from test_gpu_production import near_tie_clip
    lens = [44100, 1, 1101, 1102, 1103, 20000, 57000, 5, 44100, 44100]
    clips = [make_clip(70 + i, n) for i, n in enumerate(lens)]
    clips[8] = np.zeros(44100, np.int16)
    clips[9] = near_tie_clip()
    off = np.zeros(len(clips) + 1, np.int64)
    off[1:] = np.cumsum([c.size for c in clips])
    pcm = np.concatenate(clips + [np.zeros(8, np.int16)])
    g = _general(pcm, off, L, S, win)
    for i, c in enumerate(clips):
        r = _check_clip(g, i, c, L, S, win)
        if r["status"] == 0 and len(r["vad_energy"]):
            nv = len(r["vad_energy"])
            np.testing.assert_allclose(g["vad_energy"][i, :nv], r["vad_energy"], rtol=1e-12, atol=0)
            np.testing.assert_array_equal(g["vad_zcr"][i, :nv], r["vad_zcr"])
    fx = FeatureExtractor(L, S, win, True)
    f = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm).cuda(), off).items()}
    assert np.array_equal(f["start_end"], g["start_end"]) and np.array_equal(f["n_frames"], g["n_frames"])
    assert np.array_equal(f["status"] & 0xFF, g["status"] & 0xFF)
    if (L, S) == (1102, 441):
        assert g["status"][9] & 0x100  # the near tie was redone in numpy's exact order


def test_int32_stereo_sums_vs_oracle():
    """17-bit clips (sums of two int16 channels, beyond int16) on the int32 path."""
    import torch
    from src.pipeline import FeatureExtractor
    from src.synth import make_clip
    clips = []
    for i in range(6):
        a = make_clip(300 + i, 44100 - 500 * i).astype(np.int32)
        clips.append(a + np.roll(a, 11 + i))  # |sum| up to ~2 x 0.6 FS: 17 bits
    assert max(np.abs(c).max() for c in clips) > 32767
    off = np.zeros(len(clips) + 1, np.int64)
    off[1:] = np.cumsum([c.size for c in clips])
    pcm = np.concatenate(clips + [np.zeros(8, np.int32)])
    fx = FeatureExtractor(1102, 441, "hamming", True)
    out = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm).cuda(), off).items()}
    for i, c in enumerate(clips):
        _check_clip(out, i, c, 1102, 441, "hamming")


def test_clips_past_explicit_max_len_report_too_long():
    """An explicit max_len caps the clips processed: on the general-only paths (an int32 batch, and
    an int16 batch at a frame length the fused plan cannot hold) a longer clip reports
    DSP_CLIP_TOO_LONG with NaN features instead of leaving its outputs unwritten."""
    import torch
    from src.pipeline import FeatureExtractor
    from src.synth import make_clip
    for dtype, L, S in ((np.int32, 1102, 441), (np.int16, 40000, 441)):
        clips = [make_clip(900 + i, n).astype(dtype) for i, n in enumerate((30000, 200000, 44100))]
        off = np.zeros(len(clips) + 1, np.int64)
        off[1:] = np.cumsum([c.size for c in clips])
        pcm = np.concatenate(clips + [np.zeros(8, dtype)])
        fx = FeatureExtractor(L, S, "hamming", True)
        if dtype == np.int16:
            assert fx.fused_cap() == 0
        for o in fx._outputs(len(clips), 50000).values():  # stale contents must not survive
            o.fill_(7)
        out = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm).cuda(), off, max_len=50000).items()}
        assert out["status"][1] & 0xFF == 4, out["status"]  # DSP_CLIP_TOO_LONG
        assert np.isnan(out["feat"][1]).all()
        assert out["n_frames"][1] == 0 and (out["start_end"][1] == 0).all()
        assert (out["status"][[0, 2]] & 0xFF == 0).all()
        if dtype == np.int32:
            for i in (0, 2):
                _check_clip(out, i, clips[i], L, S, "hamming")


def test_s16_stereo_golden_through_process_audio_file(golden, tmp_path):
    """The reference-generated 16-bit stereo WAV (tests/golden: wav/s16_stereo_clip) through the
    drop-in process_audio_file: endpoints exact, 15-d vector within tolerance."""
    from src.audio_processing import load_wav_pcm, process_audio_file, process_pcm
    from src.feature_extraction import extract_features_from_frames
    raw = golden["wav/s16_stereo_clip/raw"]
    _write_wav(tmp_path / "st.wav", raw, channels=2)
    frames, sr, md = process_audio_file(str(tmp_path / "st.wav"), 1102, 441)
    assert (md["start_point"], md["end_point"]) == tuple(golden["wav/s16_stereo_clip/start_end"])
    vec, _ = extract_features_from_frames(frames, "statistical")
    assert not feat_close(vec, golden["wav/s16_stereo_clip/feat"]).any()
    # the same clip on the int32 (channel-sum) path: identical reference results
    pcm, _ = load_wav_pcm(str(tmp_path / "st.wav"))
    frames, sr, md = process_pcm(pcm.astype(np.int32), sr, 1102, 441)
    assert (md["start_point"], md["end_point"]) == tuple(golden["wav/s16_stereo_clip/start_end"])
    vec, _ = extract_features_from_frames(frames, "statistical")
    assert not feat_close(vec, golden["wav/s16_stereo_clip/feat"]).any()


def test_dataset_with_stereo_and_long_files(tmp_path):
    """PCMDataset with a 16-bit stereo file (int32 part) and a 12 s file (general kernel) among
    ordinary ones: every file kept and equal to the oracle, in dataset order."""
    from src.audio_processing import load_wav_pcm
    from src.dataset import PCMDataset
    from src.pipeline import create_window
    from src.synth import make_clip
    for c in range(2):
        d = tmp_path / ("c%d" % c)
        d.mkdir()
        for j in range(3):
            _write_wav(d / ("s%d.wav" % j), make_clip(4000 + 10 * c + j, 40000 + 777 * j))
    a = make_clip(4100).astype(np.int32)
    st = np.stack([a, np.roll(a, 5)], axis=1).reshape(-1).astype(np.int16)
    _write_wav(tmp_path / "c0" / "st.wav", st, channels=2)
    _write_wav(tmp_path / "c1" / "long.wav", make_clip(4200, 12 * 44100))
    ds = PCMDataset(str(tmp_path))
    assert len(ds) == 8 and not ds.skipped
    X, y, ok = ds.extract(1102, 441, "hamming")
    assert ok.all()
    w = create_window("hamming", 1102)
    for row, (f, _) in zip(X, ds.files):
        pcm = load_wav_pcm(f)[0]
        r = oracle.process_clip(pcm if pcm.dtype == np.int16 else pcm.astype(np.float64), 1102, 441, w)
        assert not feat_close(row, r["feat"]).any(), f
