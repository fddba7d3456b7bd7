"""Dataset side of the hot path: WAV decoding off the Python
per-file loop, one pinned host->device upload, and every (frame length, frame shift, window)
configuration extracted from the same HBM-resident PCM.

The reference decodes and processes one file per loop iteration for every configuration it
evaluates (train_model.py:21-110 inside ablation_study.py:146-163, 230-247;
experiments/run_experiments.py:78-111 once per window type).  Here a dataset is decoded once --
the mono 8/16-bit PCM files by the library's native reader (dsp_wav_scan / dsp_wav_read: threads
without the interpreter lock, samples written straight into one pinned int16 buffer at their
packed offsets), every other file by the Python reader (``load_wav_pcm``) -- uploaded once, and
each configuration is one fused kernel launch over all clips (``FeatureExtractor``).  ``iter_device_batches`` is the
streaming form for file lists larger than host or device memory: batch k+1 is decoded and copied
on a side stream while batch k is being processed.
"""
import ctypes
import os
from concurrent.futures import ThreadPoolExecutor
from glob import glob

import numpy as np

from .audio_processing import load_wav_pcm
from .pipeline import FeatureExtractor


def list_dataset(data_dir):
    """[(path, class_index)] and the class names, in the reference's order: class = index of the
    sorted sub-directory name, files in glob order (run_experiments.py:64-82, train_model.py:56-71)."""
    classes = sorted(d for d in os.listdir(data_dir)
                     if os.path.isdir(os.path.join(data_dir, d)) and not d.startswith('.'))
    files = []
    for ci, name in enumerate(classes):
        for f in glob(os.path.join(data_dir, name, '*.wav')):
            files.append((f, ci))
    return files, classes


def _decode(paths, n_threads):
    """[(int16 pcm or None, error or None)] in input order."""
    def one(p):
        try:
            return load_wav_pcm(p)[0], None
        except Exception as e:  # the reference skips files it cannot process (:109-111)
            return None, str(e)
    if n_threads <= 1 or len(paths) < 2:
        return [one(p) for p in paths]
    with ThreadPoolExecutor(max_workers=n_threads) as ex:
        return list(ex.map(one, paths))


def pack_clips(clips):
    """integer clips -> (packed [sum + 8], offsets int64 [B+1]); int16, or int32 when any clip
    holds 16-bit stereo channel sums; the 8-sample tail keeps the last clip's 16-B vectors
    inside the buffer."""
    dt = np.int32 if any(c.dtype == np.int32 for c in clips) else np.int16
    lens = np.array([c.size for c in clips], dtype=np.int64)
    off = np.zeros(len(clips) + 1, dtype=np.int64)
    off[1:] = np.cumsum(lens)
    return np.concatenate([c.astype(dt, copy=False) for c in clips] + [np.zeros(8, dt)]), off


def _upload(pcm, off, device, stream=None):
    """Pinned staging + asynchronous copy on ``stream`` (current stream if None); ``pcm`` a numpy
    array or an already pinned host tensor."""
    import torch
    hp = pcm if isinstance(pcm, torch.Tensor) and pcm.is_pinned() else torch.from_numpy(np.asarray(pcm)).pin_memory()
    ho = torch.from_numpy(off).pin_memory()
    if stream is None:
        return hp.to(device, non_blocking=True), ho.to(device, non_blocking=True), (hp, ho)
    with torch.cuda.stream(stream):
        return hp.to(device, non_blocking=True), ho.to(device, non_blocking=True), (hp, ho)


def _native_reader():
    """The library with the batch WAV reader, or None (an older A/B variant library)."""
    from . import _hip
    L = _hip.load_library()
    return L if hasattr(L, "dsp_wav_scan") else None


def _cpaths(paths):
    return (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])


def read_packed(paths, n_threads=None, pinned=True, native=True):
    """A file list decoded and packed for one upload per sample type.

    -> (kept, skipped, groups): ``kept`` the indices into ``paths`` of the decoded, non-empty files
    in order; ``skipped`` [(path, reason)] (the reference skips what it cannot process,
    run_experiments.py:109-111); ``groups`` [(pos, pcm, offsets)] -- int16 clips first, then the
    int32 ones (16-bit stereo sums beyond int16) -- with ``pos`` the int64 positions in ``kept``,
    ``pcm`` a host tensor [total + 8] (pinned when ``pinned``; the 8-sample tail keeps the last
    clip's 16-B vectors inside the buffer) and ``offsets`` int64 [len(pos) + 1]."""
    import torch
    from . import _hip
    n, nt = len(paths), _threads(n_threads)
    kind, ns, doff = np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64)
    L = _native_reader() if native else None
    if L is not None and n:
        _hip.check(L.dsp_wav_scan(_cpaths(paths), n, nt, kind.ctypes.data, ns.ctypes.data, doff.ctypes.data),
                   "dsp_wav_scan")
    py = np.nonzero(kind == _hip.DSP_WAV_OTHER)[0].tolist()
    dec = dict(zip(py, _decode([paths[i] for i in py], nt)))
    kept, skipped, wide = [], [], []
    for i in range(n):
        if kind[i] != _hip.DSP_WAV_OTHER:
            pcm, err, size = None, None, int(ns[i])
        else:
            pcm, err = dec[i]
            size = 0 if pcm is None else pcm.size
        if size == 0:
            skipped.append((paths[i], err or "empty file"))
            continue
        kept.append(i)
        wide.append(pcm is not None and pcm.dtype == np.int32)
    groups = []
    for w in (False, True):
        pos = np.array([j for j, x in enumerate(wide) if x == w], dtype=np.int64)
        if pos.size == 0:
            continue
        files = [kept[j] for j in pos]
        lens = np.array([ns[i] if kind[i] else dec[i][0].size for i in files], dtype=np.int64)
        off = np.zeros(len(files) + 1, dtype=np.int64)
        off[1:] = np.cumsum(lens)
        buf = torch.empty(int(off[-1]) + 8, dtype=torch.int32 if w else torch.int16, pin_memory=pinned)
        hv = buf.numpy()
        hv[int(off[-1]):] = 0
        nat = [j for j, i in enumerate(files) if kind[i] != _hip.DSP_WAV_OTHER]
        if nat:
            sel = [files[j] for j in nat]
            k2 = np.ascontiguousarray(kind[sel])
            n2, d2, o2 = (np.ascontiguousarray(a) for a in (ns[sel], doff[sel], off[nat]))
            _hip.check(L.dsp_wav_read(_cpaths([paths[i] for i in sel]), len(sel), nt, k2.ctypes.data, n2.ctypes.data,
                                      d2.ctypes.data, o2.ctypes.data, buf.data_ptr()), "dsp_wav_read")
            if (k2 == _hip.DSP_WAV_OTHER).any():  # a file changed since the scan: all through Python
                return read_packed(paths, n_threads, pinned, native=False)
        for j, i in enumerate(files):
            if kind[i] == _hip.DSP_WAV_OTHER:
                hv[off[j]:off[j + 1]] = dec[i][0]
        groups.append((pos, buf, off))
    return kept, skipped, groups


def upload_groups(groups, device):
    """read_packed's groups -> ([(pos, device pcm, device offsets, longest clip)], the pinned
    host buffers, to be kept alive until the asynchronous copies have run)."""
    import torch
    parts, pinned = [], []
    for pos, buf, off in groups:
        ho = torch.from_numpy(off).pin_memory()
        parts.append((pos, buf.to(device, non_blocking=True), ho.to(device, non_blocking=True), int(np.diff(off).max())))
        pinned.append((buf, ho))
    return parts, pinned


def _threads(n_threads):
    if n_threads:
        return int(n_threads)
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


class PCMDataset:
    """A directory of class sub-directories of WAV files, decoded once and resident in HBM.

    Attributes: ``labels`` int array, ``files`` [(path, class)] of the kept clips, ``skipped``
    [(path, reason)], ``class_names``; ``parts``: the device-resident PCM as (clip numbers,
    packed pcm, int64 offsets, longest clip) groups -- int16 clips in one, and 16-bit stereo
    clips whose channel sums need int32 in another (dsp_extract_general).
    """

    def __init__(self, data_dir, n_threads=None, device=None):
        from . import _hip
        self.device = device or _hip.require_device()
        files, self.class_names = list_dataset(data_dir)
        kept, self.skipped, groups = read_packed([f for f, _ in files], n_threads)
        if not kept:
            raise ValueError("no readable WAV files under %s" % data_dir)
        self.files = [files[i] for i in kept]
        self.labels = np.array([ci for _, ci in self.files], dtype=np.int64)
        self.parts, self._pinned = upload_groups(groups, self.device)
        self.max_len = max(p_[3] for p_ in self.parts)

    def _run(self, fx):
        """Every part through ``fx`` -> per-clip host arrays in dataset order (per-frame arrays
        zero-padded to the widest part)."""
        n = len(self.files)
        got = []
        for idx, dp, do, ml in self.parts:
            got.append((idx, {k: v.cpu().numpy() for k, v in fx(dp, do, max_len=ml).items()}))
        res = {}
        for k in got[0][1]:
            width = max(o[k].shape[1] for _, o in got) if got[0][1][k].ndim > 1 else None
            a0 = got[0][1][k]
            shape = (n,) if width is None else (n, width) + a0.shape[2:]
            res[k] = np.zeros(shape, dtype=a0.dtype)
            for idx, o in got:
                if width is None:
                    res[k][idx] = o[k]
                else:
                    res[k][idx, :o[k].shape[1]] = o[k]
        return res

    def __len__(self):
        return len(self.files)

    def extract(self, frame_length, frame_shift, window_type='hamming', do_endpoint_detection=True,
                energy_high_ratio=0.5, energy_low_ratio=0.1, zcr_threshold_ratio=1.5):
        """One fused launch over every clip -> (X float64 [n_ok, 15], y [n_ok], ok mask [n]).

        Clips whose processing the reference would abandon with a ValueError (status & 0xFF != 0)
        are dropped, as the reference's loaders skip them (train_model.py:91-94)."""
        fx = FeatureExtractor(frame_length, frame_shift, window_type, do_endpoint_detection,
                              energy_high_ratio, energy_low_ratio, zcr_threshold_ratio, device=self.device)
        out = self._run(fx)
        feat = out["feat"].astype(np.float64)
        ok = (out["status"] & 0xFF) == 0
        return feat[ok], self.labels[ok], ok

    def extract_both(self, frame_length, frame_shift, window_type='hamming', do_endpoint_detection=True,
                     use_only_energy_zcr=True, energy_high_ratio=0.5, energy_low_ratio=0.1,
                     zcr_threshold_ratio=1.5):
        """compare_feature_methods.py:43-115 in one fused launch: the statistical matrix and the
        padded sequence tensor of the same clips.

        -> (X_stat float64 [n_ok, 15], y [n_ok], X_seq float64 [n_ok, max_frames, 2|3], lengths
        [n_ok]).  The kernel writes each clip's per-frame (E, M, ZCR) rows into a zeroed
        [B, ld, 3] buffer, so cutting it at the batch's longest sequence is exactly
        ``pad_or_truncate_sequence(seq, max(lengths))`` (fe.py:135-154) for every clip; the
        columns are (E, ZCR) with ``use_only_energy_zcr`` (fe.py:124-128)."""
        fx = FeatureExtractor(frame_length, frame_shift, window_type, do_endpoint_detection,
                              energy_high_ratio, energy_low_ratio, zcr_threshold_ratio,
                              return_sequences=True, device=self.device)
        out = self._run(fx)
        ok = (out["status"] & 0xFF) == 0
        lengths = out["n_frames"].astype(np.int64)[ok]
        width = int(lengths.max()) if lengths.size else 0
        cols = [0, 2] if use_only_energy_zcr else [0, 1, 2]
        seq = out["seq"][ok][:, :width][:, :, cols].astype(np.float64)
        feat = out["feat"].astype(np.float64)[ok]
        return feat, self.labels[ok], seq, lengths

    def sweep(self, configs, **kw):
        """Feature matrices for several (frame_length, frame_shift, window_type) configurations
        over the same resident PCM: {config: (X, y, ok)}."""
        return {tuple(c): self.extract(*c, **kw) for c in configs}


def iter_device_batches(paths, batch_clips, n_threads=None, device=None):
    """Stream a file list through the device in batches: yields (pcm, offsets, max_len, index
    list, skipped) with the device tensors of batch k ready while batch k+1 is decoded on host
    threads and copied on a side stream (the consumer's launches on the current stream overlap
    the next copy).  Paths that fail to decode are reported in ``skipped`` and not in the batch."""
    import torch
    from . import _hip
    device = device or _hip.require_device()
    copy_stream = torch.cuda.Stream(device)
    nt = _threads(n_threads)
    pool = ThreadPoolExecutor(max_workers=1)

    def prepare(lo):
        idx = list(range(lo, min(lo + batch_clips, len(paths))))
        kept, skipped, groups = read_packed([paths[i] for i in idx], nt)
        if not kept:
            return None, [], skipped
        if len(groups) == 1:
            pcm, off = groups[0][1], groups[0][2]
        else:  # int16 and int32 clips in one batch: one int32 buffer in file order
            byp = {}
            for pos, buf, goff in groups:
                for j, q in enumerate(pos):
                    byp[int(q)] = buf.numpy()[goff[j]:goff[j + 1]]
            pcm, off = pack_clips([byp[q] for q in range(len(kept))])
        dp, do, pin = _upload(pcm, off, device, copy_stream)
        ev = torch.cuda.Event()
        ev.record(copy_stream)
        return (dp, do, int(np.diff(off).max()), ev, pin), [idx[k] for k in kept], skipped

    try:
        fut = pool.submit(prepare, 0)
        for lo in range(0, len(paths), batch_clips):
            cur, idx, skipped = fut.result()
            if lo + batch_clips < len(paths):
                fut = pool.submit(prepare, lo + batch_clips)
            if cur is None:
                yield None, None, 0, idx, skipped
                continue
            dp, do, ml, ev, _pin = cur
            cs = torch.cuda.current_stream(device)
            cs.wait_event(ev)
            dp.record_stream(cs)  # allocated on the copy stream, used on this one
            do.record_stream(cs)
            yield dp, do, ml, idx, skipped
    finally:
        pool.shutdown(wait=True)
