"""Seeded synthetic isolated-word utterances (int16 PCM, 44.1 kHz).

There is no dataset on this machine (the reference reads ~/Downloads/speech_data_*,
config.py:16-19), so every test and benchmark uses clips made here.  Clip ``i``
is generated from ``numpy.random.default_rng(base_seed + i)`` alone, so any
shard of a batch can be produced independently and reproducibly.

Content of one clip: a Gaussian noise floor (sigma ~0.003 FS),
a 50 ms fricative burst (sigma ~0.05 FS) just before the onset, and one voiced
segment (f0 in [100, 250] Hz, 5 harmonics, Hanning envelope, 0.3-0.5 s long,
onset 0.15-0.35 s).  With ``n_classes`` set, f0 and duration depend on the
class label so that a KNN on the 15-d features has something to learn.
"""
import numpy as np

SAMPLE_RATE = 44100


def make_clip(seed, n_samples=SAMPLE_RATE, label=None, n_classes=10, sr=SAMPLE_RATE):
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples) / sr
    x = rng.standard_normal(n_samples) * 0.003
    if label is None:
        f0 = rng.uniform(100.0, 250.0)
        dur = rng.uniform(0.3, 0.5)
    else:
        frac = (label + rng.uniform(0.1, 0.9)) / n_classes
        f0 = 100.0 + 150.0 * frac
        dur = 0.3 + 0.2 * ((label * 7) % n_classes + rng.uniform(0.0, 1.0)) / n_classes
    onset = rng.uniform(0.15, 0.35)
    amp = rng.uniform(0.2, 0.6)
    scale = min(1.0, n_samples / float(sr))  # shorter clips: shrink the layout
    i0 = int(onset * scale * sr)
    i1 = min(n_samples, i0 + int(dur * scale * sr))
    seg = np.zeros(i1 - i0)
    ts = t[i0:i1]
    for h in range(1, 6):
        seg += np.sin(2 * np.pi * f0 * h * ts + rng.uniform(0, 2 * np.pi)) / h
    seg *= np.hanning(seg.size) * amp / 1.5
    x[i0:i1] += seg
    b1 = max(0, i0 - int(0.05 * scale * sr))
    x[b1:i0] += rng.standard_normal(i0 - b1) * 0.05
    return np.clip(np.round(x * 32767.0), -32768, 32767).astype(np.int16)


def make_batch(n_clips, base_seed=0, n_samples=SAMPLE_RATE, start=0, with_labels=False, n_classes=10):
    """Clips ``start .. start+n_clips-1`` of the stream seeded at ``base_seed``.

    Returns int16 [n_clips, n_samples] (and int32 labels when ``with_labels``).
    """
    out = np.empty((n_clips, n_samples), np.int16)
    labels = np.empty(n_clips, np.int32)
    for j in range(n_clips):
        g = start + j
        lab = g % n_classes if with_labels else None
        out[j] = make_clip(base_seed + g, n_samples, label=lab, n_classes=n_classes)
        labels[j] = -1 if lab is None else lab
    if with_labels:
        return out, labels
    return out


def make_batch_device(n_clips, device, base_seed=0, n_samples=SAMPLE_RATE, start=0, chunk=2048):
    """The same utterance recipe generated on the device (torch RNG, float32): for batches too
    large to synthesise on the host (100 k clips = 8.8 GB).  Clips ``start .. start+n_clips-1``;
    chunk ``c`` of ``chunk`` clips is drawn from a generator seeded with (base_seed, c), so a
    shard that starts on a chunk boundary is reproducible on its own.  Returns int16
    [n_clips, n_samples] on ``device``."""
    import torch
    out = torch.empty((n_clips, n_samples), dtype=torch.int16, device=device)
    t = torch.arange(n_samples, device=device, dtype=torch.float32) / SAMPLE_RATE
    idx = torch.arange(n_samples, device=device)
    scale = min(1.0, n_samples / float(SAMPLE_RATE))
    lo = 0
    while lo < n_clips:
        c = (start + lo) // chunk
        hi = min(n_clips, (c + 1) * chunk - start)
        m = hi - lo
        g = torch.Generator(device=device)
        g.manual_seed(int(base_seed) * 1000003 + c)
        u = torch.rand((m, 9), generator=g, device=device)
        f0 = 100.0 + 150.0 * u[:, 0:1]
        dur = 0.3 + 0.2 * u[:, 1:2]
        onset = 0.15 + 0.2 * u[:, 2:3]
        amp = 0.2 + 0.4 * u[:, 3:4]
        i0 = (onset * scale * SAMPLE_RATE).long()
        i1 = torch.clamp(i0 + (dur * scale * SAMPLE_RATE).long(), max=n_samples)
        x = torch.randn((m, n_samples), generator=g, device=device) * 0.003
        seg = torch.zeros((m, n_samples), device=device)
        for h in range(1, 6):
            seg += torch.sin(2 * torch.pi * f0 * h * t + 2 * torch.pi * u[:, 3 + h:4 + h]) / h
        inside = (idx >= i0) & (idx < i1)
        seglen = (i1 - i0).clamp(min=2).float()
        env = 0.5 - 0.5 * torch.cos(2 * torch.pi * (idx - i0).float() / (seglen - 1))
        x += torch.where(inside, seg * env * amp / 1.5, 0.0)
        b1 = torch.clamp(i0 - int(0.05 * scale * SAMPLE_RATE), min=0)
        burst = (idx >= b1) & (idx < i0)
        x += torch.where(burst, torch.randn((m, n_samples), generator=g, device=device) * 0.05, 0.0)
        out[lo:hi] = torch.clamp(torch.round(x * 32767.0), -32768, 32767).to(torch.int16)
        lo = hi
    return out
