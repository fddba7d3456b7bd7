"""Batched device API of the hot path (PyTorch-ROCm tensors in, tensors out).

This is what the reference's per-file loop becomes (experiments/run_experiments.py:78-111):
a batch of int16 clips resident in HBM goes through one fused HIP launch
(``dsp_extract_features``) and a 15-d feature matrix comes back, then
``knn_classify`` runs KNeighborsClassifier's exact k-NN + vote on the device.
"""
import numpy as np

from . import _hip

FEATURE_NAMES = ["%s_%s" % (f, s) for f in ("energy", "magnitude", "zcr")
                 for s in ("mean", "std", "max", "min", "median")]


def create_window(window_type, length):
    """src/audio_processing.py:278-296 -- host-side coefficients, exactly numpy's."""
    if window_type == "rectangular":
        return np.ones(length)
    if window_type == "hamming":
        return np.hamming(length)
    if window_type == "hanning":
        return np.hanning(length)
    raise ValueError("不支持的窗函数类型: %s" % window_type)


def _as_device(x, dtype, device):
    import torch
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.array(x, copy=True, order="C")).to(device=device, dtype=dtype).contiguous()


class FeatureExtractor:
    """Reusable launch plan for ``dsp_extract_features`` (outputs preallocated per batch size).

    Parameters mirror process_audio_file (src/audio_processing.py:336-341) with frame sizes
    in samples, as the reference's callers pass them (experiments/run_experiments.py:90-99).
    """

    def __init__(self, frame_length, frame_shift, window_type="hamming", do_endpoint_detection=True,
                 energy_high_ratio=0.5, energy_low_ratio=0.1, zcr_threshold_ratio=1.5,
                 return_vad_lists=False, return_sequences=False, device=None):
        import torch
        self.device = device or _hip.require_device()
        self.L, self.S = int(frame_length), int(frame_shift)
        if self.L < 1 or self.S < 1:
            raise ValueError("frame_length and frame_shift must be positive")
        self.window_type = window_type
        self.window = torch.as_tensor(create_window(window_type, self.L), dtype=torch.float64).to(self.device)
        self.do_vad = bool(do_endpoint_detection)
        self.ratios = (float(energy_high_ratio), float(energy_low_ratio), float(zcr_threshold_ratio))
        self.return_vad_lists = return_vad_lists
        self.return_sequences = return_sequences
        self._bufs = {}

    def _queue_ws(self):
        """The zeroed DSP_QUEUE_WS_BYTES scratch of this extractor's launches on the CURRENT
        stream.  Launches on one stream are ordered, so they share one buffer (each launch leaves
        it zeroed); a launch on another stream -- including a HIP-graph capture, whose replays
        may overlap eager calls -- gets its own, so two launches can never claim chunks from the
        same counters."""
        import torch
        qs = self.__dict__.setdefault("_queues", {})
        key = torch.cuda.current_stream(self.device).cuda_stream
        q = qs.get(key)
        if q is None:
            q = qs[key] = torch.zeros(_hip.QUEUE_WS_BYTES // 4, dtype=torch.int32, device=self.device)
        return q

    def lds_bytes(self, max_len):
        return _hip.lib().dsp_extract_lds_bytes(int(max_len), self.L, self.S)

    def _outputs(self, B, max_len):
        import torch
        key = (B, max_len)
        if key not in self._bufs:
            d = self.device
            # one packed row per clip (DSP_OUT_ROW_WORDS int32 words: feat[15] as f32 bits, start,
            # end, n_frames, status), written by the kernels with out_stride = 19; the four result
            # arrays are strided views of it, and "rows" travels in one collective unpacked
            rows = torch.empty((B, _hip.OUT_ROW_WORDS), dtype=torch.int32, device=d)
            o = dict(rows=rows, feat=rows.view(torch.float32)[:, :15], start_end=rows[:, 15:17],
                     n_frames=rows[:, 17], status=rows[:, 18])
            if self.return_vad_lists:
                ld = max(1, (max_len - self.L) // self.S + 1) if max_len >= self.L else 1
                o["vad_energy"] = torch.zeros((B, ld), dtype=torch.float64, device=d)
                o["vad_zcr"] = torch.zeros((B, ld), dtype=torch.int32, device=d)
            if self.return_sequences:
                ld = 1 if max_len <= self.L else (max_len - self.L + self.S - 1) // self.S + 1
                o["seq"] = torch.zeros((B, ld, 3), dtype=torch.float32, device=d)
            self._bufs = {key: o}  # keep one shape alive
        return self._bufs[key]

    def fused_cap(self):
        """Longest clip (samples) the fused kernel's on-chip plan holds at this (L, S)."""
        if not hasattr(self, "_fcap"):
            lib, lo, hi = _hip.lib(), 0, 1 << 24
            while lo < hi:  # dsp_extract_lds_bytes is non-zero exactly for n <= cap
                mid = (lo + hi + 1) // 2
                if lib.dsp_extract_lds_bytes(mid, self.L, self.S) > 0:
                    lo = mid
                else:
                    hi = mid - 1
            self._fcap = lo
        return self._fcap

    def __call__(self, pcm, offsets=None, max_len=None):
        """pcm: int16 or int32 [B, N] (uniform clips) or packed 1-D with int64 offsets [B+1].

        int16 clips that fit the fused kernel's on-chip plan run in one fused launch; longer
        clips, and int32 samples (16-bit stereo channel sums), run on dsp_extract_general in the
        same stream order.  An explicit ``max_len`` caps the clips processed (longer ones report
        DSP_CLIP_TOO_LONG); without it, device-tensor offsets cost one host sync (the longest
        clip sizes the launch), so pass ``max_len`` to capture the call in a HIP graph.  Returns a
        dict of device tensors: feat [B,15] f32, start_end [B,2] i32, n_frames [B] i32, status
        [B] i32 -- strided views of ``rows`` [B,19] i32, each clip's packed 76-B record -- (+
        vad_energy/vad_zcr, seq when requested).  The tensors are reused by the next call with the
        same shape.
        """
        import torch
        d = self.device
        wide = str(getattr(pcm, "dtype", "")) in ("int32", "torch.int32")
        pcm = _as_device(pcm, torch.int32 if wide else torch.int16, d)
        if offsets is None:
            if pcm.dim() != 2:
                raise ValueError("1-D packed pcm needs offsets")
            B, N = pcm.shape
            key = ("uni", B, N)
            if key not in self._bufs:
                self._bufs[key] = torch.arange(B + 1, dtype=torch.int64, device=d) * N
            off = self._bufs[key]
            true_max = N
        else:
            if isinstance(offsets, np.ndarray) or not isinstance(offsets, torch.Tensor):
                lens = np.diff(np.asarray(offsets, dtype=np.int64))
                true_max = int(lens.max()) if lens.size else 1
            else:
                true_max = None
            off = _as_device(offsets, torch.int64, d)
            B = off.numel() - 1
            if true_max is None:
                true_max = int(torch.max(off[1:] - off[:-1]).item()) if B > 0 else 1
        if max_len is None:
            max_len = true_max
        pcm = pcm.reshape(-1)
        max_len = max(int(max_len), 1)
        out = self._outputs(B, max_len)
        hi, lo, zr = self.ratios
        ve, vz, ldv = out.get("vad_energy"), out.get("vad_zcr"), 0
        if ve is not None:
            ldv = ve.shape[1]
        sq, lds_ = out.get("seq"), 0
        if sq is not None:
            lds_ = sq.shape[1]
        args = (int(self.do_vad), hi, lo, zr, _hip.ptr(out["feat"]), _hip.ptr(out["start_end"]),
                _hip.ptr(out["n_frames"]), _hip.ptr(out["status"]), _hip.OUT_ROW_WORDS, _hip.ptr(ve),
                _hip.ptr(vz), ldv, _hip.ptr(sq), lds_)
        cap = 0 if wide else self.fused_cap()
        if not wide and B > 0 and cap > 0:
            # the clip-queue scratch: zeroed once, and every launch leaves it zeroed again (the
            # last workgroup out of each kernel resets its counters), so the launches of this
            # extractor on its stream reuse one buffer without a fill kernel per call
            queue = self._queue_ws()
            rc = _hip.lib().dsp_extract_features(
                _hip.ptr(pcm), _hip.ptr(off), B, min(max_len, cap), self.L, self.S,
                _hip.ptr(self.window), *args, _hip.ptr(queue), _hip.stream_handle(d))
            _hip.check(rc, "dsp_extract_features")
        if B > 0 and (wide or max_len > cap):
            # the clips the fused kernel cannot hold (longer than cap, or every clip of an int32
            # batch, or all of them when the fused plan holds none at this frame length): the
            # general kernel over the whole batch, its length window [cap + 1, max_len] selecting
            # them on the device -- no host round trip, so the call stays graph-capturable
            nbytes = _hip.lib().dsp_extract_general_workspace_bytes(B, max_len, self.L, self.S)
            ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=d)
            rc = _hip.lib().dsp_extract_general(
                _hip.ptr(pcm), 4 if wide else 2, _hip.ptr(off), None, B, cap, max_len, self.L, self.S,
                _hip.ptr(self.window), *args, _hip.ptr(ws), nbytes, _hip.stream_handle(d))
            _hip.check(rc, "dsp_extract_general")
            self._keep = ws  # stream-ordered use: the caching allocator reuses it only after the launch
        return out


def process_audio_batch(pcm, offsets=None, frame_length=1102, frame_shift=441, window_type="hamming",
                        do_endpoint_detection=True, energy_high_ratio=0.5, energy_low_ratio=0.1,
                        zcr_threshold_ratio=1.5, return_vad_lists=False, return_sequences=False,
                        max_len=None):
    """One-shot batched form of process_audio_file + extract_features_from_frames."""
    fx = FeatureExtractor(frame_length, frame_shift, window_type, do_endpoint_detection,
                          energy_high_ratio, energy_low_ratio, zcr_threshold_ratio,
                          return_vad_lists, return_sequences)
    return dict(fx(pcm, offsets, max_len))


class KnnIndex:
    """A reference set prepared for ``dsp_knn_classify`` -- KNeighborsClassifier.fit's side
    (src/models.py:52-55): the first query converts the rows for the screen into this index's
    workspace, and every later query against the same set skips that step (DSP_KNN_REF_READY).
    ``query`` is predict / kneighbors.  One query at a time per index (a workspace is a launch's
    scratch); the workspace grows to the largest query batch seen."""

    def __init__(self, ref, ref_labels, k, n_classes=None, with_pred=True):
        import torch
        self.device = _hip.require_device()
        self.ref = _as_device(ref, torch.float64, self.device)
        self.Nr, self.D = self.ref.shape
        self.k = int(k)
        self.labels = _as_device(ref_labels, torch.int32, self.device) if (ref_labels is not None and with_pred) else None
        self.n_classes = int(n_classes or 0)
        self._ws, self._ready = None, False

    def query(self, query, self_offset=-1, stats=None):
        """(idx int32 [Nq,k], dist float64 [Nq,k], pred int32 [Nq] or None); a dict passed as
        ``stats`` receives "fallbacks" (queries answered by the exhaustive fp64 scan; one host sync)."""
        import torch
        d, k = self.device, self.k
        q = _as_device(query, torch.float64, d)
        Nq = q.shape[0]
        ws_bytes = _hip.lib().dsp_knn_workspace_bytes(self.Nr, Nq, self.D, k)
        if ws_bytes == 0 and Nq > 0:
            raise ValueError("unsupported KNN shape (1 <= D <= 4096, 1 <= k <= 32)")
        if self._ws is None or self._ws.numel() < ws_bytes:
            self._ws, self._ready = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=d), False
        idx = torch.empty((Nq, k), dtype=torch.int32, device=d)
        dist = torch.empty((Nq, k), dtype=torch.float64, device=d)
        pred = torch.empty(Nq, dtype=torch.int32, device=d) if self.labels is not None else None
        flags = _hip.KNN_REF_READY if self._ready else 0
        rc = _hip.lib().dsp_knn_classify(_hip.ptr(self.ref), _hip.ptr(self.labels), self.Nr, _hip.ptr(q), Nq,
                                         self.D, k, int(self_offset), self.n_classes, _hip.ptr(idx),
                                         _hip.ptr(dist), _hip.ptr(pred), _hip.ptr(self._ws), self._ws.numel(),
                                         flags, _hip.stream_handle(d))
        _hip.check(rc, "dsp_knn_classify")
        self._ready = self._ready or (Nq > 0 and self.Nr > 0)
        if stats is not None and Nq > 0:
            off = _hip.lib().dsp_knn_workspace_fallbacks_offset(self.Nr, Nq, self.D, k)
            stats["fallbacks"] = int(self._ws[off:off + 4].view(torch.int32).item())
        return idx, dist, pred


def knn_classify(ref, ref_labels, query, k, self_offset=-1, n_classes=None, with_pred=True, stats=None):
    """Exact k-NN (KNeighborsClassifier semantics) on the device, one-shot (``KnnIndex`` keeps the
    prepared reference set across queries).

    ref [Nr, D] / query [Nq, D] float64 (cast if needed), ref_labels int [Nr].
    Returns (idx int32 [Nq,k], dist float64 [Nq,k], pred int32 [Nq] or None).  A dict passed as
    ``stats`` receives "fallbacks": the queries answered by the exhaustive fp64 fallback (one host
    sync).
    """
    return KnnIndex(ref, ref_labels, k, n_classes, with_pred).query(query, self_offset, stats)


def zscore_fit(X):
    """normalize_features' mean/std (src/feature_extraction.py:171-177) on the device."""
    import torch
    d = _hip.require_device()
    X = _as_device(X, torch.float64, d)
    N, D = X.shape
    mean = torch.empty(D, dtype=torch.float64, device=d)
    std = torch.empty(D, dtype=torch.float64, device=d)
    _hip.check(_hip.lib().dsp_zscore_fit(_hip.ptr(X), N, D, _hip.ptr(mean), _hip.ptr(std),
                                         _hip.stream_handle(d)), "dsp_zscore_fit")
    return mean, std


def zscore_apply(X, mean, std):
    import torch
    d = _hip.require_device()
    X = _as_device(X, torch.float64, d)
    mean = _as_device(mean, torch.float64, d)
    # a private float64 copy: std may be a read-only (e.g. broadcast) numpy view
    std = _as_device(std, torch.float64, d)
    std = torch.where(std == 0, torch.ones_like(std), std)
    out = torch.empty_like(X)
    N, D = X.shape
    _hip.check(_hip.lib().dsp_zscore_apply(_hip.ptr(X), N, D, _hip.ptr(mean), _hip.ptr(std), _hip.ptr(out),
                                           _hip.stream_handle(d)), "dsp_zscore_apply")
    return out
