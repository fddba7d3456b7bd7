#!/usr/bin/env python3
"""Row f4: where the end-to-end time of ``run.py --experiment classifier``
goes, on a synthetic isolated-word dataset (--files WAVs, 10 classes, 16-bit mono 44.1 kHz,
0.7-1.4 s, written into a temporary directory, so the page cache is warm).

Three measurements, one JSON line:

* ``user_wall_s``: ``python run.py --experiment classifier`` as a user starts it (a fresh process,
  interpreter start and every import included), timed from outside.
* ``cold`` / ``warm``: the same ``run.main`` in a fresh instrumented process, twice.  The
  instrumentation wraps the functions the run calls -- file listing, ``read_packed`` (the native
  batch reader into one pinned buffer, the Python reader for any other file), ``upload_groups``,
  device initialisation, ``PCMDataset.extract`` (FeatureExtractor + fused launch +
  device->host copy), ``train_test_split``, the z-score, each classifier's fit + evaluate, the
  result file -- and ``builtins.__import__`` (time spent importing modules, charged to the stage
  that triggered it).  ``unattributed_s`` = run.main's time minus every stage and every import
  outside a stage; ``imports_before_main_s`` is the process's import of the instrumented modules.
  The first pass pays the one-off costs (imports, HIP context, code-object loads); the second is
  the steady state.
* ``decode``: the decode stage alone over the same files -- files/s and MB/s -- for the native
  reader (``read_packed``: dsp_wav_scan + dsp_wav_read into a pinned buffer) on the default thread
  count and on 1 thread, and for the Python readers it replaced (``_decode``: the RIFF walk of
  ``_read_wav`` and the ``wave`` module), 1 thread and the pool.

Needs the GPU (extraction and KNN run there).

    python tools/f4_breakdown.py [--files 2000]
"""
import argparse
import builtins
import json
import os
import subprocess
import sys
import tempfile
import time
import wave

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dsp-audioreclabs_amd")
sys.path.insert(0, PKG)


def write_dataset(root, n_files, n_classes=10):
    from src.synth import make_clip
    rng = np.random.default_rng(0)
    for c in range(n_classes):
        os.makedirs(os.path.join(root, "class_%02d" % c), exist_ok=True)
    for i in range(n_files):
        c = i % n_classes
        n = int(rng.integers(30000, 60000))  # 0.7-1.4 s
        pcm = make_clip(10000 + i, n, label=c, n_classes=n_classes)
        with wave.open(os.path.join(root, "class_%02d" % c, "u%05d.wav" % i), "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(44100)
            w.writeframes(pcm.tobytes())


class Clock:
    """Stage timers (inclusive, non-overlapping by construction) plus import time charged to the
    open stage."""

    def __init__(self):
        self.stages, self.stage_imports, self.open, self.imports_outside = {}, {}, None, 0.0
        self.depth = 0
        self.sync = None

    def wrap(self, name, fn, sync=False):
        clock = self

        def timed(*a, **k):
            if clock.open is not None:  # nested call of a wrapped function: the outer stage owns it
                return fn(*a, **k)
            if sync and clock.sync:
                clock.sync()
            clock.open = name
            t = time.perf_counter()
            try:
                out = fn(*a, **k)
                if sync and clock.sync:
                    clock.sync()
                return out
            finally:
                clock.stages[name] = clock.stages.get(name, 0.0) + time.perf_counter() - t
                clock.open = None
        return timed

    def install_import_timer(self):
        orig = builtins.__import__
        clock = self

        def timed_import(*a, **k):
            if clock.depth:
                return orig(*a, **k)
            clock.depth = 1
            t = time.perf_counter()
            try:
                return orig(*a, **k)
            finally:
                dt = time.perf_counter() - t
                clock.depth = 0
                if clock.open is None:
                    clock.imports_outside += dt
                else:
                    clock.stage_imports[clock.open] = clock.stage_imports.get(clock.open, 0.0) + dt
        builtins.__import__ = timed_import

    def reset(self):
        self.stages, self.stage_imports, self.imports_outside = {}, {}, 0.0


def instrumented(data, res):
    """Child process: run.main twice under the stage clock; prints one JSON line."""
    t_proc = time.perf_counter()
    clock = Clock()
    clock.install_import_timer()
    import run  # noqa: F401  (run.py's own module-level imports)
    import src.dataset as ds
    import src._hip as hip
    import experiments.run_experiments as rx
    import sklearn.model_selection as ms
    imports_before = time.perf_counter() - t_proc
    clock.imports_outside = 0.0

    ds.list_dataset = clock.wrap("list_files", ds.list_dataset)
    ds.read_packed = clock.wrap("decode", ds.read_packed)
    ds.upload_groups = clock.wrap("upload", ds.upload_groups, sync=True)
    hip.require_device = clock.wrap("device_init", hip.require_device)
    ds.PCMDataset.extract = clock.wrap("extraction", ds.PCMDataset.extract, sync=True)
    ms.train_test_split = clock.wrap("split", ms.train_test_split)
    rx.normalize_features = clock.wrap("zscore", rx.normalize_features, sync=True)
    orig_te = rx.SpeechRecognitionExperiment.train_and_evaluate_classifier

    def te(self, kind, *a, **k):
        return clock.wrap("fit_evaluate_" + kind, orig_te, sync=True)(self, kind, *a, **k)
    rx.SpeechRecognitionExperiment.train_and_evaluate_classifier = te
    rx.SpeechRecognitionExperiment._save = clock.wrap("save_results", rx.SpeechRecognitionExperiment._save)

    passes = []
    for p in range(2):
        clock.reset()
        if p == 1 or "torch" in sys.modules:
            import torch
            clock.sync = torch.cuda.synchronize if torch.cuda.is_initialized() else None
        t = time.perf_counter()
        rc = run.main(["--data-dir", data, "--results-dir", res, "--experiment", "classifier"])
        if clock.sync is None:
            import torch
            torch.cuda.synchronize()
        total = time.perf_counter() - t
        assert rc == 0
        staged = sum(clock.stages.values())
        passes.append({
            "run_main_s": round(total, 4),
            "stages_s": {k: round(v, 5) for k, v in clock.stages.items()},
            "of_which_imports_s": {k: round(v, 5) for k, v in clock.stage_imports.items()},
            "imports_outside_stages_s": round(clock.imports_outside, 5),
            "unattributed_s": round(total - staged - clock.imports_outside, 5),
            "attributed_frac": round((staged + clock.imports_outside) / total, 4),
            "share": {k: round(v / total, 4) for k, v in clock.stages.items()},
        })
    print(json.dumps({"imports_before_main_s": round(imports_before, 4), "cold": passes[0], "warm": passes[1]}),
          flush=True)


def decode_bench(data):
    """_decode alone: files/s and MB/s for the RIFF reader and the wave module, 1 thread and the pool."""
    import src.audio_processing as ap
    import src.dataset as ds
    files, _ = ds.list_dataset(data)
    paths = [f for f, _ in files]
    mb = sum(os.path.getsize(p) for p in paths) / 1e6
    out = {"files": len(paths), "MB": round(mb, 2), "pool_threads": ds._threads(None)}
    for nt in (ds._threads(None), 1):
        ds.read_packed(paths[:64], nt)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            kept, _, groups = ds.read_packed(paths, nt)
            best = min(best, time.perf_counter() - t)
        assert len(kept) == len(paths)
        out["native_%dthr" % nt] = {"s": round(best, 4), "files_per_s": round(len(paths) / best, 1),
                                    "MB_per_s": round(mb / best, 1), "includes": "scan + read into pinned buffer"}
    riff = ap._read_wav
    for reader in ("riff", "wave_module"):
        ap._read_wav = riff if reader == "riff" else (lambda f: ap._read_wav_module(f))
        for nt in (1, ds._threads(None)):
            ds._decode(paths[:64], nt)
            best = 1e9
            for _ in range(3):
                t = time.perf_counter()
                r = ds._decode(paths, nt)
                best = min(best, time.perf_counter() - t)
            assert all(p is not None for p, _ in r)
            out["%s_%dthr" % (reader, nt)] = {"s": round(best, 4), "files_per_s": round(len(paths) / best, 1),
                                              "MB_per_s": round(mb / best, 1)}
    ap._read_wav = riff
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=2000)
    ap.add_argument("--instrumented", nargs=2, metavar=("DATA", "RESULTS"), help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.instrumented:
        return instrumented(*args.instrumented)
    tmp = tempfile.mkdtemp(prefix="f4_")
    data = os.path.join(tmp, "data")
    write_dataset(data, args.files)

    # as a user runs it: a fresh interpreter, every import included
    t = time.perf_counter()
    subprocess.run([sys.executable, os.path.join(PKG, "run.py"), "--data-dir", data, "--results-dir",
                    os.path.join(tmp, "r0"), "--experiment", "classifier"], check=True, stdout=subprocess.DEVNULL)
    user_wall = time.perf_counter() - t

    t = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--instrumented", data, os.path.join(tmp, "r1")],
                       check=True, capture_output=True, text=True)
    child_wall = time.perf_counter() - t
    inst = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    dec = decode_bench(data)
    cold = inst["cold"]
    print(json.dumps({
        "what": "run.py --experiment classifier, %d synthetic WAVs (10 classes, 0.7-1.4 s, 16-bit mono, page cache "
                "warm)" % args.files,
        "user_wall_s": round(user_wall, 4),
        "interpreter_and_imports_s": round(user_wall - cold["run_main_s"], 4),
        "instrumented_process_wall_s": round(child_wall, 4),
        **inst,
        "decode": dec,
        "decode_share_of_user_wall": round(cold["stages_s"].get("decode", 0.0) / user_wall, 4),
    }), flush=True)


if __name__ == "__main__":
    main()
