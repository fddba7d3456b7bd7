"""Drop-in for the reference's src/feature_extraction.py on MI355X.

``extract_features_from_frames`` (fe.py:91-132) on the ``DeviceFrames`` that
``audio_processing.process_audio_file`` returns hands back what the fused gfx950 kernel already
computed (per-frame E / M / ZCR and the 15-d statistics): no second pass.  Plain frame arrays
(callers that build frames themselves) are reduced on the HIP device.  ``normalize_features``
runs the z-score kernels (csrc/knn.hip: dsp_zscore_fit / dsp_zscore_apply).
"""
import numpy as np

from . import _hip
from .audio_processing import DeviceFrames
from .pipeline import FEATURE_NAMES, zscore_apply, zscore_fit


def extract_frame_features(frames):
    """fe.py:12-43 -> {'energy', 'magnitude', 'zcr'}: float64 [n_frames] each."""
    if isinstance(frames, DeviceFrames):
        if len(frames) == 0:
            raise ValueError("No frames provided for feature extraction.")
        return {k: v.copy() for k, v in frames.features.items()}
    import torch
    d = _hip.require_device()
    f = frames if isinstance(frames, torch.Tensor) else torch.as_tensor(np.asarray(frames, dtype=np.float64))
    f = f.to(device=d, dtype=torch.float64)
    if f.dim() != 2 or f.shape[0] == 0:
        raise ValueError("No frames provided for feature extraction.")
    s = torch.where(f > 0, 1.0, -1.0).to(torch.float64)
    return {
        "energy": (f * f).sum(dim=1).cpu().numpy(),
        "magnitude": f.abs().sum(dim=1).cpu().numpy(),
        "zcr": ((s[:, 1:] - s[:, :-1]).abs().sum(dim=1) / 2).cpu().numpy(),
    }


def compute_statistics(sequence):
    """fe.py:46-62 -> {'mean', 'std', 'max', 'min', 'median'} (population std)."""
    import torch
    d = _hip.require_device()
    x = torch.as_tensor(np.asarray(sequence, dtype=np.float64), device=d)
    if x.numel() == 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    xs = torch.sort(x).values
    n = xs.numel()
    med = xs[n // 2] if n % 2 else (xs[n // 2 - 1] + xs[n // 2]) / 2
    return {"mean": float(x.mean()), "std": float(x.std(unbiased=False)), "max": float(xs[-1]),
            "min": float(xs[0]), "median": float(med)}


def extract_statistical_features(frame_features):
    """fe.py:65-88 -> (float64 [15], names) in the order energy, magnitude, zcr x stats."""
    vec = []
    for ft in ("energy", "magnitude", "zcr"):
        st = compute_statistics(frame_features[ft])
        vec += [st[k] for k in ("mean", "std", "max", "min", "median")]
    return np.array(vec), list(FEATURE_NAMES)


def extract_features_from_frames(frames, method='statistical', use_only_energy_zcr=False):
    """fe.py:91-132: 'statistical' -> ([15], names); 'sequence' -> ([n, 3] or [n, 2], None)."""
    if method not in ("statistical", "sequence"):
        raise ValueError(f"不支持的特征提取方法: {method}")
    if method == "statistical" and isinstance(frames, DeviceFrames):
        if len(frames) == 0:
            raise ValueError("No frames provided for feature extraction.")
        return frames.vector.copy(), list(FEATURE_NAMES)
    ff = extract_frame_features(frames)
    if method == "statistical":
        return extract_statistical_features(ff)
    cols = ["energy", "zcr"] if use_only_energy_zcr else ["energy", "magnitude", "zcr"]
    return np.stack([ff[c] for c in cols], axis=1), None


def pad_or_truncate_sequence(sequence, target_length):
    """fe.py:135-154: zero-pad or cut [n, d] to [target_length, d]."""
    sequence = np.asarray(sequence)
    if len(sequence) < target_length:
        pad = np.zeros((target_length - len(sequence), sequence.shape[1]))
        return np.vstack([sequence, pad])
    return sequence[:target_length]


def normalize_features(features, mean=None, std=None):
    """fe.py:157-181 -> (normalized, mean, std); std == 0 -> 1; float64 on the device.

    2-D input: column statistics in numpy's axis-0 order (bit-exact).  1-D input (a single
    vector, scalar statistics): numpy sums it pairwise, the device sequentially -- equal to a
    few ulps."""
    X = np.asarray(features, dtype=np.float64)
    one = X.ndim == 1
    X2 = X.reshape(-1, 1) if one else X
    if mean is None or std is None:
        m_d, s_d = zscore_fit(X2)
        m_fit, s_fit = m_d.cpu().numpy(), s_d.cpu().numpy()
    mean = m_fit if mean is None else np.asarray(mean, dtype=np.float64)
    std = s_fit if std is None else np.asarray(std, dtype=np.float64)  # s_fit: 0 -> 1 already
    std = np.where(std == 0, 1.0, std)
    cols = X2.shape[1]
    out = zscore_apply(X2, np.broadcast_to(mean, (cols,)), np.broadcast_to(std, (cols,))).cpu().numpy()
    if one:
        return out.reshape(-1), mean.reshape(-1)[0] if mean.size == 1 else mean, \
            std.reshape(-1)[0] if std.size == 1 else std
    return out, mean, std
