#!/usr/bin/env python3
"""Headline benchmark: frames/s of framing + window + E/M/ZCR (+ double-threshold VAD) on
1 s 44.1 kHz clips (BASELINE.json "metric"), one process per GPU.

Workload at N=1 is BASELINE.json configs[1]: 1000 synthetic 1 s utterances per GPU, Hamming
window, all three features + VAD (reference defaults L=1102, S=441, config.py:39-40).  A
"step" is one pass of the fused HIP kernel over one 1000-clip batch that is already resident
in HBM; steps rotate over a pool of batches larger than the 256 MiB Infinity Cache so every
step streams its input from HBM.  Frames counted per clip = VAD frames (98) + frames after the
endpoint crop (data dependent), the same frames the reference computes E/ZCR on.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dsp-audioreclabs_amd"))

METRIC = "frames/sec (framing+window+E/M/ZCR) on 1 s 44.1 kHz clips; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
OUT_BYTES_PER_CLIP = 15 * 4 + 2 * 4 + 4 + 4  # feat f32[15] + start/end + n_frames + status


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clips", type=int, default=1000, help="clips per GPU per step")
    ap.add_argument("--pool", type=int, default=4, help="distinct resident batches per GPU")
    ap.add_argument("--frame-length", type=int, default=1102)
    ap.add_argument("--frame-shift", type=int, default=441)
    ap.add_argument("--window", default="hamming")
    ap.add_argument("--no-vad", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step from Python instead of replaying a captured HIP graph")
    ap.add_argument("--knn-ref", type=int, default=100000,
                    help="KNN leg (BASELINE configs[4]): reference rows, all of them queried (0: skip)")
    ap.add_argument("--knn-k", type=int, default=5)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from src.pipeline import FeatureExtractor
    from src.synth import make_batch

    C, P, N = args.clips, args.pool, 44100
    L, S = args.frame_length, args.frame_shift
    vad = not args.no_vad
    # each rank generates its own contiguous slice of the global clip stream (seed = index)
    host = make_batch(P * C, base_seed=0, start=rank * P * C).reshape(P, C, N)
    pool = torch.as_tensor(host).to(dev)
    fx = FeatureExtractor(L, S, args.window, vad, device=dev)
    stream = torch.cuda.current_stream(dev)

    # frames per batch (VAD frames + feature frames), counted from the kernel's own outputs
    frames = []
    for p in range(P):
        out = fx(pool[p])
        nf = out["n_frames"].to(torch.int64).sum().item()
        nv = C * ((N - L) // S + 1) if (vad and N >= L) else 0
        frames.append(nf + nv)
        st = out["status"].cpu().numpy() & 0xFF
        assert not st.any(), "clip errors in benchmark batch"
    for i in range(args.warmup):
        fx(pool[i % P])
    torch.cuda.synchronize(dev)

    K = args.steps
    # per-launch kernel time on the launch stream (HIP events), for the roofline
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for i in range(K):
        ev[i][0].record(stream)
        fx(pool[i % P])
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    # the timed steps: the K launches captured once into a HIP graph and replayed, so the host's
    # per-call overhead (ctypes, Python) does not throttle a 60 us kernel; --no-graph launches
    # each step from Python
    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=torch.cuda.Stream(dev)):
            for i in range(K):
                fx(pool[i % P])
        graph.replay()
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graph is not None:
        graph.replay()
    else:
        for i in range(K):
            fx(pool[i % P])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    my_frames = float(sum(frames[i % P] for i in range(K)))
    if world > 1:
        t = torch.tensor([elapsed, my_frames, kern_ms], dtype=torch.float64, device=dev)
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, total_frames, kern_ms = tmax[0].item(), tsum[1].item(), tmax[2].item()
        # the exchange step before KNN (not part of the metric): all-gather of the 15-d vectors
        from src.distributed import all_gather_rows
        feat = fx(pool[0])["feat"]
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        all_gather_rows(feat, total=C * world)
        torch.cuda.synchronize(dev)
        ag_ms = (time.perf_counter() - g0) * 1e3
    else:
        total_frames = my_frames
        ag_ms = None
    knn = knn_leg(args, dev, world) if args.knn_ref > 0 else None

    result = None
    if rank == 0:
        bytes_per_launch = C * (2 * N + OUT_BYTES_PER_CLIP)
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "dsp::extract_kernel", "kernel_avg_ms": round(kern_ms, 5),
                "algorithmic_bytes_per_launch": bytes_per_launch}
        pmc = os.path.join(REPO, "profiles", "pmc_extract.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                pm = json.load(f)
            key = "%d_%d_%d_%s_%d" % (C, L, S, args.window, int(vad))
            if key in pm:
                roof["traffic"] = pm[key]["hbm_bytes_per_launch"]
                roof["traffic_source"] = pm[key]["source"]
        result = {
            "metric": METRIC,
            "value": round(total_frames / elapsed, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (seeded 1 s int16 utterances: noise floor + fricative burst + voiced segment)",
            "config": {"workload": "BASELINE configs[1]: %d x 1 s 44.1 kHz utterances per GPU, %s window, "
                                   "E/M/ZCR + %s" % (C, args.window, "double-threshold VAD" if vad else "no VAD"),
                       "clips_per_gpu": C, "samples_per_clip": N, "frame_length": L, "frame_shift": S,
                       "window": args.window, "vad": vad, "input": "int16 PCM resident in HBM",
                       "frames_per_step_per_gpu": round(my_frames / K, 1),
                       "parallelism": "dp%d (clips sharded, no collective in the step)" % world,
                       "launch": "hip graph of the %d steps" % K if graph is not None else "python loop"},
            "roofline": roof,
        }
        if ag_ms is not None:
            result["allgather_feat_ms"] = round(ag_ms, 4)
        if knn is not None:
            result["knn"] = knn
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(host[0], L, S, args.window, vad, args.cpu_seconds)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


def knn_leg(args, dev, world):
    """BASELINE configs[4] beside the headline metric: exact k-NN (KNeighborsClassifier
    semantics) of every one of --knn-ref synthetic z-scored 15-d vectors against all of them
    (self excluded), queries sharded over the ranks, results gathered (RCCL all-gather).  Not
    part of ``value``; reported as its own object with its VALU roofline (45 flop per pair)."""
    import torch
    import torch.distributed as dist
    from src.distributed import knn_sharded
    from src.pipeline import knn_classify
    rng = np.random.default_rng(0)  # same reference set on every rank
    n, dim = args.knn_ref, 15
    centres = rng.standard_normal((10, dim)) * 1.5
    y = rng.integers(0, 10, n).astype(np.int32)
    X = centres[y] + rng.standard_normal((n, dim))
    X = (X - X.mean(0)) / X.std(0)
    Xd, yd = torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)
    knn_sharded(knn_classify, Xd, yd, Xd, args.knn_k, self_query=True)  # warm-up
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(3):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        idx, dd, pred = knn_sharded(knn_classify, Xd, yd, Xd, args.knn_k, self_query=True)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = tt.item()
    pairs = float(n) * n
    tf = pairs * 45 / t / 1e12
    return {"metric": "k-NN pairs/s (15-d, exact, k=%d, self-query, gathered)" % args.knn_k,
            "value": round(pairs / t, 1), "unit": "pairs/s", "ms": round(t * 1e3, 4),
            "ref": n, "queries": n, "queries_per_rank": -(-n // world),
            "roofline": {"bound": "valu", "achieved": round(tf, 2), "peak": 157.3 * world, "unit": "TFLOP/s",
                         "frac": round(tf / (157.3 * world), 4), "flop_per_pair": 45,
                         "note": "whole-job wall time incl. conversion, merge and the result all-gather"},
            "data": "synthetic z-scored 15-d vectors around 10 class centres"}


def cpu_baseline(batch, L, S, window, vad, budget_s):
    """The C oracle (a restatement of the reference's numpy pipeline, oracle/) on the host
    cores of this box, on a bounded sample of the same clips."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from src.pipeline import create_window
    w = create_window(window, L)
    C, N = batch.shape
    flat = np.ascontiguousarray(batch.reshape(-1))
    off = np.arange(C + 1, dtype=np.int64) * N
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    nv = (N - L) // S + 1 if (vad and N >= L) else 0

    def run(nt, clips):
        o = off[:clips + 1]
        t = time.perf_counter()
        r = oracle.process_batch(flat[:o[-1]], o, L, S, w, do_vad=vad, nthreads=nt)
        dt = time.perf_counter() - t
        return (nv * clips + int(r["n_frames"].sum())) / dt, dt

    run(threads, min(C, 64 * threads))  # warm-up (thread arenas, page faults, clocks)
    rate, dt = run(threads, C)
    reps = 1
    total_frames, total_t = rate * dt, dt
    while total_t < budget_s and reps < 5000:
        r2, d2 = run(threads, C)
        total_frames += r2 * d2
        total_t += d2
        reps += 1
    one, d1 = run(1, min(C, 200))
    return {"value": round(total_frames / total_t, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": "%d passes over %d of the benchmark's clips (%.1f s), C restatement of the reference "
                      "numpy pipeline (oracle/dsp_oracle.c), %d threads; 1 thread: %.4g frames/s"
                      % (reps, C, total_t, threads, one)}


if __name__ == "__main__":
    main()
