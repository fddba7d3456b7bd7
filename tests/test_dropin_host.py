"""Host-side parts of the drop-in layer (no GPU): configuration, dataset listing, argument errors."""
import os
import wave

import numpy as np
import pytest


def test_config_matches_reference_constants():
    import config
    assert (config.SAMPLE_RATE, config.FRAME_LENGTH, config.FRAME_SHIFT) == (44100, 1102, 441)
    assert (config.ENERGY_HIGH_RATIO, config.ENERGY_LOW_RATIO, config.ZCR_THRESHOLD_RATIO) == (0.5, 0.1, 1.5)
    assert config.WINDOW_TYPES == ['rectangular', 'hamming', 'hanning']
    assert (config.KNN_N_NEIGHBORS, config.TEST_SIZE, config.RANDOM_SEED) == (3, 0.2, 42)
    assert not os.path.exists(config.RESULTS_DIR) or os.path.isdir(config.RESULTS_DIR)


def test_pad_or_truncate():
    from src.feature_extraction import pad_or_truncate_sequence
    s = np.arange(12.0).reshape(4, 3)
    assert pad_or_truncate_sequence(s, 6).shape == (6, 3)
    assert np.array_equal(pad_or_truncate_sequence(s, 6)[4:], np.zeros((2, 3)))
    assert np.array_equal(pad_or_truncate_sequence(s, 2), s[:2])


def test_errors_match_reference():
    from src.feature_extraction import extract_features_from_frames
    from src.models import create_classifier
    with pytest.raises(ValueError):
        extract_features_from_frames(np.zeros((3, 8)), method='bogus')
    with pytest.raises(ValueError):
        create_classifier('perceptron')
    with pytest.raises(NotImplementedError):
        create_classifier('mlp')
    clf = create_classifier('naive_bayes')  # scikit-learn model, as in the reference
    clf.fit(np.random.default_rng(0).normal(size=(20, 3)), np.arange(20) % 2)


def _write_wav(path, data, width=2, channels=1, sr=44100):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes(np.ascontiguousarray(data).tobytes())


def test_dataset_listing_order(tmp_path):
    from experiments.run_experiments import list_dataset
    for c in ("b", "a", ".hidden"):
        (tmp_path / c).mkdir()
    _write_wav(tmp_path / "a" / "x.wav", np.zeros(10, np.int16))
    _write_wav(tmp_path / "b" / "y.wav", np.zeros(10, np.int16))
    files, classes = list_dataset(str(tmp_path))
    assert classes == ["a", "b"]
    assert [(os.path.basename(f), c) for f, c in files] == [("x.wav", 0), ("y.wav", 1)]


def test_dataset_listing_and_packing(tmp_path):
    """src/dataset.py host side: class = sorted sub-directory index, glob order, packed buffer
    with an 8-sample tail and int64 offsets."""
    from src.dataset import list_dataset, pack_clips
    for name in ("b", "a", ".hidden"):
        (tmp_path / name).mkdir()
    (tmp_path / "a" / "x.wav").write_bytes(b"")
    (tmp_path / "b" / "y.wav").write_bytes(b"")
    (tmp_path / "b" / "notes.txt").write_bytes(b"")
    files, classes = list_dataset(str(tmp_path))
    assert classes == ["a", "b"] and [(os.path.basename(f), c) for f, c in files] == [("x.wav", 0), ("y.wav", 1)]
    clips = [np.arange(5, dtype=np.int16), np.arange(3, dtype=np.int16) + 100]
    pcm, off = pack_clips(clips)
    assert list(off) == [0, 5, 8] and pcm.size == 16 and list(pcm[5:8]) == [100, 101, 102] and not pcm[8:].any()
