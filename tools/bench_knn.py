#!/usr/bin/env python3
"""KNN leg of the hot path (BASELINE.json configs[4]): exact k-NN of 15-d feature vectors,
KNeighborsClassifier semantics (src/models.py:18-72), on one GPU.

The 8-GPU config shards 100 000 queries over the ranks against the full, replicated 100 000-row
reference set, so one rank's work is --queries 12500 against --ref 100000; the
default runs that shard.  Inputs are synthetic z-scored 15-d vectors drawn around 10 class
centres (no dataset here), resident in HBM; the query block is a slice of the reference set and
excludes itself (kneighbors(X=None) semantics, self_offset).

Prints one JSON line: pairs/s, achieved fp32 TFLOP/s at 45 flop per pair (15 sub + 15 fma) against
the 157.3 TF fp32 peak (matrix cores and VALU alike: the screen runs v_mfma_f32_16x16x4_f32), and the C oracle's exhaustive
single-thread rate on a bounded query sample, run on this host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dsp-audioreclabs_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

VALU_PEAK_TFS = 157.3  # MI355X fp32, vector and f32-in MFMA alike (MI355X_MICROARCH.md)
FLOP_PER_PAIR = 45     # D = 15: 15 subtractions + 15 fused multiply-adds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", type=int, default=100000)
    ap.add_argument("--queries", type=int, default=12500)
    ap.add_argument("--dim", type=int, default=15)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-queries", type=int, default=200)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--graph", action="store_true", help="also time the query job replayed from a HIP graph")
    ap.add_argument("--data", choices=("extracted", "synthetic"), default="extracted",
                    help="extracted: the z-scored 15-d features of --ref synthetic utterances (BASELINE "
                         "configs[4]); synthetic: Gaussian vectors around 10 class centres (rounds 1-5)")
    a = ap.parse_args()
    import torch
    from src.pipeline import FeatureExtractor, KnnIndex, zscore_apply, zscore_fit

    dev = torch.device("cuda", 0)
    if a.data == "extracted":
        from src.synth import make_batch_device
        a.dim = 15
        out = FeatureExtractor(1102, 441, "hamming", True, device=dev)(make_batch_device(a.ref, dev, base_seed=0))
        assert not (out["status"] & 0xFF).any().item()
        feat = out["feat"].to(torch.float64)
        mu, sd = zscore_fit(feat)
        Xd = zscore_apply(feat, mu, sd)
        yd = (torch.arange(a.ref, device=dev) % 10).to(torch.int32)
        X, y = Xd.cpu().numpy(), yd.cpu().numpy()
    else:
        rng = np.random.default_rng(0)
        centres = rng.standard_normal((10, a.dim)) * 1.5
        y = rng.integers(0, 10, a.ref).astype(np.int32)
        X = centres[y] + rng.standard_normal((a.ref, a.dim))
        X = (X - X.mean(0)) / X.std(0)
        Xd = torch.as_tensor(X, device=dev)
        yd = torch.as_tensor(y, device=dev)
    q0 = 0
    Qd = Xd[q0:q0 + a.queries]
    index = KnnIndex(Xd, yd, a.k, n_classes=10)
    index.query(Qd, self_offset=q0)  # fit (the reference set converted) + warm-up (code objects)
    torch.cuda.synchronize()
    times = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        idx, dist, pred = index.query(Qd, self_offset=q0)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / 1e3)
    st = {}  # the fallback count reads the workspace (a host sync): one untimed call
    index.query(Qd, self_offset=q0, stats=st)
    t_graph = None
    if a.graph:  # the same query job captured once and replayed (launch gaps gone: serving use)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            index.query(Qd, self_offset=q0)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            gi, gd, gp = index.query(Qd, self_offset=q0)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(gi, idx) and torch.equal(gd, dist) and (gp is None or torch.equal(gp, pred))
        gt = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            gt.append(e0.elapsed_time(e1) / 1e3)
        t_graph = float(np.median(gt))
    t = float(np.median(times))
    pairs = float(a.ref) * a.queries
    res = {"metric": "k-NN pairs/s (15-d, exact, KNeighborsClassifier semantics)",
           "value": round(pairs / t, 1), "unit": "pairs/s", "ms": round(t * 1e3, 4),
           "fallbacks": st.get("fallbacks"),
           "ms_graph_replay": None if t_graph is None else round(t_graph * 1e3, 4),
           "config": {"ref": a.ref, "queries": a.queries, "dim": a.dim, "k": a.k, "self_query": True,
                      "data": ("z-scored 15-d features of %d synthetic utterances (fused extraction + "
                               "normalize_features on the device), labels i mod 10" % a.ref)
                      if a.data == "extracted" else "synthetic z-scored 15-d vectors around 10 class centres",
                      "timed": "queries against the prepared reference set (KnnIndex: the fp32 conversion "
                               "is the fit, done once)"},
           "roofline": {"bound": "mfma-f32", "achieved": round(pairs * FLOP_PER_PAIR / t / 1e12, 2),
                        "peak": VALU_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": round(pairs * FLOP_PER_PAIR / t / 1e12 / VALU_PEAK_TFS, 4),
                        "flop_per_pair": FLOP_PER_PAIR}}
    if not a.no_cpu:
        import oracle
        nq = min(a.cpu_queries, a.queries)
        t0 = time.perf_counter()
        i0, d0, p0 = oracle.knn(X, y, X[q0:q0 + nq], a.k, n_classes=10, self_offset=q0)
        tc = time.perf_counter() - t0
        ok = bool(np.array_equal(idx[:nq].cpu().numpy(), i0) and np.array_equal(dist[:nq].cpu().numpy(), d0)
                  and np.array_equal(pred[:nq].cpu().numpy(), p0))
        res["cpu_baseline"] = {"value": round(nq * float(a.ref) / tc, 1), "unit": "pairs/s", "cores": 1,
                               "kind": "port",
                               "sample": "%d queries x %d rows exhaustive fp64 (oracle/dsp_oracle.c ora_knn), %.2f s"
                                         % (nq, a.ref, tc)}
        res["parity_on_sample"] = ok
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
