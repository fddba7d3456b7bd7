"""ctypes front end of the C oracle (oracle/dsp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg, never by the product package.  It is the
checker the HIP path is compared against; see dsp_oracle.c for what it
restates and how it is pinned to the reference.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libdsp_oracle.so")
_lib = None

_D = ctypes.POINTER(ctypes.c_double)
_I64 = ctypes.POINTER(ctypes.c_int64)
_I32 = ctypes.POINTER(ctypes.c_int32)
_I16 = ctypes.POINTER(ctypes.c_int16)
_i64 = ctypes.c_int64
_dbl = ctypes.c_double


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "dsp_oracle.c")
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.ora_np_sum.restype = ctypes.c_double
        L.ora_np_sum.argtypes = [_D, _i64]
        L.ora_compute_statistics.argtypes = [_D, _i64, _D]
        L.ora_preprocess.argtypes = [_D, _i64, _D]
        L.ora_endpoint_detection.restype = _i64
        L.ora_endpoint_detection.argtypes = [_D, _i64, _i64, _i64, _dbl, _dbl, _dbl, _I64, _I64, _D, _D]
        L.ora_frame_count.restype = _i64
        L.ora_frame_count.argtypes = [_i64, _i64, _i64]
        L.ora_vad_frame_count.restype = _i64
        L.ora_vad_frame_count.argtypes = [_i64, _i64, _i64]
        L.ora_frame_features.restype = _i64
        L.ora_frame_features.argtypes = [_D, _i64, _i64, _i64, _D, _D, _D, _D]
        proc = [_i64, _i64, _i64, _D, ctypes.c_int, _dbl, _dbl, _dbl, _D, _I64, _I64, _D, _D, _I64, _D, _i64]
        L.ora_process_pcm_i16.argtypes = [_I16] + proc
        L.ora_process_f64.argtypes = [_D] + proc
        L.ora_process_batch_i16.argtypes = [_I16, _I64, _i64, _i64, _i64, _D, ctypes.c_int, _dbl, _dbl, _dbl,
                                            _D, _I64, _I64, _I32, ctypes.c_int]
        L.ora_zscore_fit.argtypes = [_D, _i64, ctypes.c_int, _D, _D]
        L.ora_knn.argtypes = [_D, _I32, _i64, _D, _i64, ctypes.c_int, ctypes.c_int, _i64, ctypes.c_int,
                              _I32, _D, _I32]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def np_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().ora_np_sum(_p(a, _D), a.size)


def compute_statistics(seq):
    a = np.ascontiguousarray(seq, dtype=np.float64)
    out = np.zeros(5)
    lib().ora_compute_statistics(_p(a, _D), a.size, _p(out, _D))
    return out


def preprocess(x):
    a = np.array(x, dtype=np.float64)
    if lib().ora_preprocess(_p(a, _D), a.size, _p(a, _D)):
        raise ValueError("zero-size array")
    return a


def endpoint_detection(x, L, S, hi=0.5, lo=0.1, zr=1.5):
    a = np.ascontiguousarray(x, dtype=np.float64)
    nv = lib().ora_vad_frame_count(a.size, L, S)
    E = np.zeros(max(nv, 1))
    Z = np.zeros(max(nv, 1))
    st, en = ctypes.c_int64(), ctypes.c_int64()
    n = lib().ora_endpoint_detection(_p(a, _D), a.size, L, S, hi, lo, zr, ctypes.byref(st), ctypes.byref(en),
                                     _p(E, _D), _p(Z, _D))
    return st.value, en.value, E[:n], Z[:n]


def frame_features(x, L, S, window):
    a = np.ascontiguousarray(x, dtype=np.float64)
    w = np.ascontiguousarray(window, dtype=np.float64)
    F = lib().ora_frame_count(a.size, L, S)
    E, M, Z = np.zeros(max(F, 1)), np.zeros(max(F, 1)), np.zeros(max(F, 1))
    lib().ora_frame_features(_p(a, _D), a.size, L, S, _p(w, _D), _p(E, _D), _p(M, _D), _p(Z, _D))
    return E[:F], M[:F], Z[:F]


def process_clip(pcm, L, S, window, do_vad=True, hi=0.5, lo=0.1, zr=1.5):
    """Whole per-clip pipeline on int16 PCM (or float64 audio).

    Returns dict(status, feat[15], start, end, n_frames, vad_energy, vad_zcr, seq[F,3]).
    """
    pcm = np.ascontiguousarray(pcm)
    w = np.ascontiguousarray(window, dtype=np.float64)
    n = pcm.size
    nv = lib().ora_vad_frame_count(n, L, S)
    cap = lib().ora_frame_count(n, L, S) + 1
    feat = np.zeros(15)
    se = np.zeros(2, np.int64)
    nf = ctypes.c_int64(0)
    nvo = ctypes.c_int64(0)
    E = np.zeros(max(nv, 1))
    Z = np.zeros(max(nv, 1))
    seq = np.zeros((cap, 3))
    args = (n, L, S, _p(w, _D), int(do_vad), hi, lo, zr, _p(feat, _D), _p(se, _I64), ctypes.byref(nf),
            _p(E, _D), _p(Z, _D), ctypes.byref(nvo), _p(seq, _D), cap)
    if pcm.dtype == np.int16:
        rc = lib().ora_process_pcm_i16(_p(pcm, _I16), *args)
    else:
        a = np.ascontiguousarray(pcm, dtype=np.float64)
        rc = lib().ora_process_f64(_p(a, _D), *args)
    F = nf.value
    return dict(status=rc, feat=feat, start=int(se[0]), end=int(se[1]), n_frames=F,
                vad_energy=E[:nvo.value], vad_zcr=Z[:nvo.value], seq=seq[:F])


def process_batch(pcm, offsets, L, S, window, do_vad=True, hi=0.5, lo=0.1, zr=1.5, nthreads=1):
    """Batched driver (used as the CPU baseline): int16 packed clips + int64 offsets[B+1]."""
    pcm = np.ascontiguousarray(pcm, dtype=np.int16)
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    w = np.ascontiguousarray(window, dtype=np.float64)
    B = off.size - 1
    feat = np.zeros((B, 15))
    se = np.zeros((B, 2), np.int64)
    nf = np.zeros(B, np.int64)
    st = np.zeros(B, np.int32)
    lib().ora_process_batch_i16(_p(pcm, _I16), _p(off, _I64), B, L, S, _p(w, _D), int(do_vad), hi, lo, zr,
                                _p(feat, _D), _p(se, _I64), _p(nf, _I64), _p(st, _I32), int(nthreads))
    return dict(feat=feat, start_end=se, n_frames=nf, status=st)


def zscore_fit(X):
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    mean, std = np.zeros(d), np.zeros(d)
    lib().ora_zscore_fit(_p(X, _D), n, d, _p(mean, _D), _p(std, _D))
    return mean, std


def knn(ref, ref_labels, query, k, n_classes=None, self_offset=-1, nthreads=1):
    """sklearn KNeighborsClassifier(k) kneighbors + predict, restated (dsp_oracle.c ora_knn).
    With nthreads > 1 the queries are split into contiguous blocks answered on that many host
    threads (ctypes releases the GIL); self_offset follows each block."""
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    q = np.ascontiguousarray(query, dtype=np.float64)
    lbl = np.ascontiguousarray(ref_labels, dtype=np.int32)
    if n_classes is None:
        n_classes = int(lbl.max()) + 1 if lbl.size else 1
    Nr, D = ref.shape
    Nq = q.shape[0]
    idx = np.zeros((Nq, k), np.int32)
    dist = np.zeros((Nq, k))
    pred = np.zeros(Nq, np.int32)
    L = lib()

    def run(a, b):
        if b <= a:
            return
        L.ora_knn(_p(ref, _D), _p(lbl, _I32), Nr, _p(q[a:b], _D), b - a, D, k,
                  self_offset + a if self_offset >= 0 else -1, n_classes,
                  _p(idx[a:b], _I32), _p(dist[a:b], _D), _p(pred[a:b], _I32))

    nthreads = max(1, min(int(nthreads), Nq))
    if nthreads == 1:
        run(0, Nq)
    else:
        from concurrent.futures import ThreadPoolExecutor
        cuts = [Nq * t // nthreads for t in range(nthreads + 1)]
        with ThreadPoolExecutor(nthreads) as ex:
            list(ex.map(lambda t: run(cuts[t], cuts[t + 1]), range(nthreads)))
    return idx, dist, pred
