#!/usr/bin/env python3
"""Headline benchmark: frames/s of framing + window + E/M/ZCR (+ double-threshold VAD) on
1 s 44.1 kHz clips (BASELINE.json "metric"), one process per GPU.

Workload: the north-star batch, 100 000 synthetic 1 s utterances (BASELINE.json north_star and
configs[3]; 8.8 GB of int16 PCM, which fits one GPU), Hamming window, all three features +
VAD, reference defaults L=1102, S=441 (config.py:39-40).  The batch is sharded over the ranks
(rank r holds shard_range(clips, r, N), generated on its own device), so N=8 is exactly
configs[3] and the scaling is strong.  A "step" is one pass of the fused HIP kernel over the
rank's whole shard, already resident in HBM.  Frames counted per clip = VAD frames (98) +
frames after the endpoint crop (data dependent), the frames the reference computes E/ZCR on.

Beside the metric (not part of ``value``):
  * ``window_sweep`` -- configs[2]: 10 000 clips x {rectangular, hamming, hanning};
  * ``allgather`` (N > 1) -- the one exchange step, all per-clip results in one RCCL all-gather;
  * ``knn`` -- configs[4]: exact k=5 self-query over 100 000 15-d vectors, queries sharded;
  * ``configs0`` -- configs[0]'s frame sizes (Hamming, 1024 / 512 samples) on the same clips,
    GPU frames/s beside its own CPU baseline (N = 1);
  * ``configs1`` -- configs[1]: 1 000 clips, one launch (the latency-dominated small batch);
  * ``cpu_baseline`` (N = 1) -- the C restatement of the reference on this box's host cores,
    on a bounded sample of the same clips, whose outputs are also compared with the GPU's.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Without a launcher (no WORLD_SIZE in the environment) ``--gpus N`` > 1 starts the N ranks itself,
as a child torch.distributed.run, before anything touches the GPU; under a launcher WORLD_SIZE must
equal --gpus.  DSP_BENCH_ONE_DEVICE=1 (every rank on cuda:0) with DSP_BENCH_BACKEND=gloo rehearses
the multi-rank path on a one-GPU box: the line then says ``rehearsal``, the backend and the number
of physical GPUs, and is not a scaling measurement.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dsp-audioreclabs_amd"))

METRIC = "frames/sec (framing+window+E/M/ZCR) on 1 s 44.1 kHz clips; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
OUT_BYTES_PER_CLIP = 15 * 4 + 2 * 4 + 4 + 4  # feat f32[15] + start/end + n_frames + status
LLC_BYTES = 256 << 20  # MI355X Infinity Cache


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=100000, help="clips of the whole job (sharded over ranks)")
    ap.add_argument("--frame-length", type=int, default=1102)
    ap.add_argument("--frame-shift", type=int, default=441)
    ap.add_argument("--window", default="hamming")
    ap.add_argument("--no-vad", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step from Python instead of replaying a captured HIP graph")
    ap.add_argument("--sweep-clips", type=int, default=10000, help="window-sweep leg, configs[2] (0: skip)")
    ap.add_argument("--knn-ref", type=int, default=100000,
                    help="KNN leg (BASELINE configs[4]): reference rows, all of them queried (0: skip)")
    ap.add_argument("--knn-k", type=int, default=5)
    ap.add_argument("--small-clips", type=int, default=1000, help="configs[1] leg: clips of one launch (0: skip)")
    ap.add_argument("--cfg0", action=argparse.BooleanOptionalAction, default=True,
                    help="configs[0] leg: 1024 / 512-sample frames")
    ap.add_argument("--check-launch", action="store_true",
                    help="start the ranks and report the world size the process group saw (no GPU work)")
    return ap.parse_args(argv)


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(args):
    """--gpus N > 1 without a launcher: run this script under torch.distributed.run with N ranks
    (a child process; this one has not touched the GPU) and exit with its status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def check_launch(args, world, rank, backend):
    """--check-launch: the rank count the process group saw, without GPU work (CPU-testable)."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo" if backend != "nccl" else "nccl")
        seen = dist.get_world_size()
        dist.barrier()
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"check_launch": True, "gpus_flag": args.gpus, "world_size_env": world,
                          "ranks_seen": seen, "backend": backend if world > 1 else None}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def timed_launches(fn, n, stream):
    """Mean duration (ms) of n launches of fn() by HIP events recorded on the launch stream."""
    import torch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def assemble_result(args, world, ranks_seen, rehearsal, backend_name, C, total_frames, elapsed_x, elapsed_g,
                    kern_ms, kern_ms_iso=None, elapsed_gs=None, elapsed_gp=None, xchk=None):
    """The bench line (rank 0).  world > 1: ``value`` is the K steps of extraction + all-gather
    (configs[3] as BASELINE defines it), ``elapsed_g`` the faster of the serial loop (``elapsed_gs``)
    and the pipelined one (``elapsed_gp``: each step's gather beside the next step's extraction);
    ``value_extract_only`` the same steps without the exchange."""
    N = 44100
    L, S, vad = args.frame_length, args.frame_shift, not args.no_vad
    K = args.steps
    bytes_per_launch = C * (2 * N + OUT_BYTES_PER_CLIP)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "dsp::extract_kernel", "kernel_avg_ms": round(kern_ms, 5),
            "kernel_avg_source": "HIP events on the launch stream around the %d timed steps, / %d (per step: "
                                 "extract_kernel + extract_exact_kernel's early exit + launch gap)" % (args.steps, args.steps),
            "kernel_avg_ms_isolated_launches": None if kern_ms_iso is None else round(kern_ms_iso, 5),
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "per_unit": "2*44100 B in + 76 B out per clip"}
    pmc = os.path.join(REPO, "profiles", "pmc_extract.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            pm = json.load(f)
        key = "%d_%d_%d_%s_%d" % (C, L, S, args.window, int(vad))
        if key in pm:
            roof["traffic"] = pm[key]["hbm_bytes_per_launch"]
            roof["traffic_source"] = pm[key]["source"]
    elapsed = elapsed_g if elapsed_g is not None else elapsed_x
    result = {
        "metric": METRIC,
        "value": round(total_frames / elapsed, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "ranks_seen": ranks_seen,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded 1 s int16 utterances generated on the device: noise floor + "
                "fricative burst + voiced segment)",
        "config": {"workload": "north star / BASELINE configs[3] batch: %d x 1 s 44.1 kHz utterances "
                               "sharded over %d GPU(s), %s window, E/M/ZCR + %s"
                               % (args.clips, world, args.window, "double-threshold VAD" if vad else "no VAD"),
                   "clips": args.clips, "clips_per_gpu": C, "samples_per_clip": N, "frame_length": L,
                   "frame_shift": S, "window": args.window, "vad": vad, "input": "int16 PCM resident in HBM",
                   "frames_per_step": round(total_frames / K, 1),
                   "parallelism": ("dp%d (clips sharded; each step = extraction + one packed %s all-gather "
                                   "of the per-clip results)" % (world, backend_name)) if world > 1 else
                                  "dp1 (no collective)",
                   "launch": ("python loop of the %d steps (%s extraction + all-gather%s)"
                              % (K, "eager" if args.no_graph else "graph-replayed",
                                 ", pipelined" if elapsed_gp is not None and elapsed_gp <= elapsed_gs else ""))
                             if world > 1 else
                             ("hip graph of the %d steps" % K if not args.no_graph else "python loop")},
        "roofline": roof,
    }
    if world > 1:
        # the same K steps without the exchange (hip graph): what the kernel alone scales to
        result["value_extract_only"] = round(total_frames / elapsed_x, 1)
        result["ms_per_step_extract_only"] = round(elapsed_x / K * 1e3, 5)
        if elapsed_gs is not None:
            result["value_serial_exchange"] = round(total_frames / elapsed_gs, 1)
            result["ms_per_step_serial_exchange"] = round(elapsed_gs / K * 1e3, 5)
        if elapsed_gp is not None:
            result["value_pipelined_exchange"] = round(total_frames / elapsed_gp, 1)
            result["ms_per_step_pipelined_exchange"] = round(elapsed_gp / K * 1e3, 5)
            result["exchange"] = ("value = the faster of two step loops, both measured in this run: serial "
                                  "(each all-gather right after its extraction) and pipelined (step i's all-gather "
                                  "on a second stream beside step i+1's extraction, two output buffers); both "
                                  "extract every batch whole and gather all its rows inside the timed region")
        if xchk is not None:
            result["exchange_own_block_equal"] = xchk
    if rehearsal:
        result["rehearsal"] = True
        result["backend"] = backend_name
        result["physical_gpus"] = 1
        result["note"] = ("rehearsal of the multi-rank code path: %d ranks share cuda:0 over %s; not a "
                          "scaling measurement" % (world, backend_name))
    elif world > 1:
        result["backend"] = backend_name
    return result


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args)  # before any GPU call
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        return 2
    # rehearsal of the multi-rank path on a one-GPU box (not a measurement): DSP_BENCH_ONE_DEVICE=1
    # puts every rank on cuda:0 and DSP_BENCH_BACKEND=gloo replaces RCCL, which needs one GPU per rank
    rehearsal = os.environ.get("DSP_BENCH_ONE_DEVICE") == "1"
    if rehearsal:
        local = 0
    backend = os.environ.get("DSP_BENCH_BACKEND", "nccl")
    if args.check_launch:
        return check_launch(args, world, rank, backend)
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    ranks_seen = dist.get_world_size() if world > 1 else 1
    if ranks_seen != world:
        print("bench.py: process group has %d ranks, WORLD_SIZE %d" % (ranks_seen, world), file=sys.stderr)
        return 2
    backend_name = ("RCCL" if backend == "nccl" else backend) if world > 1 else None
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from src.distributed import gather_rows, gather_rows_async, shard_range
    from src.pipeline import FeatureExtractor
    from src.synth import make_batch_device

    N = 44100
    L, S = args.frame_length, args.frame_shift
    vad = not args.no_vad
    lo, hi = shard_range(args.clips, rank, world)
    C = hi - lo
    # a shard smaller than the Infinity Cache is rotated over distinct copies so that every step
    # streams its input from HBM
    P = max(1, math.ceil(2 * LLC_BYTES / max(1, C * 2 * N)))
    pool = [make_batch_device(C, dev, base_seed=p, start=lo) for p in range(P)]
    fx = FeatureExtractor(L, S, args.window, vad, device=dev)
    stream = torch.cuda.current_stream(dev)

    # frames per batch (VAD frames + feature frames), counted from the kernel's own outputs
    nv = ((N - L) // S + 1) if (vad and N >= L) else 0
    frames = []
    for p in range(P):
        out = fx(pool[p])
        frames.append(out["n_frames"].to(torch.int64).sum().item() + nv * C)
        st = out["status"].cpu().numpy() & 0xFF
        assert not st.any(), "clip errors in benchmark batch"
    for i in range(args.warmup):
        fx(pool[i % P])
    torch.cuda.synchronize(dev)

    K = args.steps
    # isolated launches, each bracketed by HIP events: reported beside the timed region's figure;
    # after the host-side syncs above the GPU has idled and its clock ramps back up over the first
    # few launches (round 6 kernel trace: 2.75 -> 2.45 ms), so these read high
    kern_ms_iso = timed_launches(lambda: fx(pool[0]), max(3, min(K, 10)), stream) if P == 1 else \
        float(np.mean([timed_launches(lambda: fx(pool[p]), 2, stream) for p in range(P)]))
    # the timed steps: captured once into a HIP graph and replayed, so host overhead (ctypes,
    # Python) does not throttle short launches; --no-graph launches each step from Python
    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(dev)
        with torch.cuda.stream(cs):  # the capture stream's own clip-queue scratch, outside the graph
            fx(pool[0])
        cs.synchronize()
        with torch.cuda.graph(graph, stream=cs):
            for i in range(K):
                fx(pool[i % P])
        graph.replay()
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for i in range(K):
            fx(pool[i % P])
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed_x = time.perf_counter() - t0  # extraction only
    # the roofline's per-launch time: HIP events on the launch stream around the K timed steps, / K
    # (each step = extract_kernel + extract_exact_kernel's early exit + the gap between launches)
    kern_ms = ev0.elapsed_time(ev1) / K
    my_frames = float(sum(frames[i % P] for i in range(K)))
    # the timed steps checked: the last replayed step's outputs (still in the extractor's buffers)
    # against one eager launch of the same batch into fresh buffers, bit for bit
    timed_ok = None
    if graph is not None:
        got = fx._outputs(C, N)["rows"].clone()
        fresh = FeatureExtractor(L, S, args.window, vad, device=dev)
        ref = fresh(pool[(K - 1) % P])["rows"]
        torch.cuda.synchronize(dev)
        timed_ok = bool(torch.equal(got, ref))
        del fresh, ref, got
    del graph

    # N > 1: configs[3] as BASELINE defines it -- every step is the rank's extraction followed by
    # the exchange, ONE packed all-gather of every per-clip result (76 B/clip) over RCCL; launched
    # from Python (the collective is not captured), K steps between barriers
    elapsed_g, elapsed_gs, elapsed_gp, ag, xchk = None, None, None, None, None
    if world > 1:
        def one_step_graphs(f):
            """ext(i): step i's extraction by f on pool[i % P] -- a replay of a one-launch HIP graph
            per batch (eager launches leave ~15 us of idle GPU per step at 12.5k clips,
            profiles/r06z_eager_step.txt), eager with --no-graph; returns f's output rows."""
            if args.no_graph:
                return lambda i: f(pool[i % P])["rows"]
            gs, rows = [], None
            cs = torch.cuda.Stream(dev)
            for b in pool:
                with torch.cuda.stream(cs):  # the capture stream's own clip-queue scratch, outside the graph
                    f(b)
                cs.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cs):
                    rows = f(b)["rows"]
                gs.append(g)
            torch.cuda.synchronize(dev)

            def ext(i):
                gs[i % P].replay()
                return rows
            return ext

        ext0 = one_step_graphs(fx)

        def step(i):
            return gather_rows(ext0(i), args.clips)
        step(0)
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(K):
            step(i)
        torch.cuda.synchronize(dev)
        dist.barrier()
        elapsed_gs = time.perf_counter() - t0  # serial: each gather waits for its extraction
        # pipelined (RCCL, equal blocks: every bench configuration): step i's all-gather runs on a
        # second stream beside step i + 1's extraction; two output buffers (two extractors), and an
        # extraction waits (on the device) for the gather that last read its buffer.  Every step
        # still extracts its whole batch and exchanges all of its rows inside the timed region.
        # (gloo, the one-GPU rehearsal's backend, blocks the host in every wait: serial only, unless
        # DSP_BENCH_PIPELINE=1 rehearses the pipelined loop too.)
        blocks = {hi - lo for lo, hi in (shard_range(args.clips, r, world) for r in range(world))}
        if len(blocks) == 1 and (backend == "nccl" or os.environ.get("DSP_BENCH_PIPELINE") == "1"):
            fx2 = FeatureExtractor(L, S, args.window, vad, device=dev)
            exts = (ext0, one_step_graphs(fx2))
            outs = [torch.empty((world * C, 19), dtype=torch.int32, device=dev) for _ in range(2)]
            comm = torch.cuda.Stream(dev)
            works = [None, None]

            def step_ov(i):
                j = i & 1
                if works[j] is not None:
                    works[j].wait()  # the extraction stream waits for gather i - 2 (no host sync)
                rows = exts[j](i)
                comm.wait_stream(stream)
                with torch.cuda.stream(comm):
                    works[j] = gather_rows_async(rows, outs[j])
                return rows

            step_ov(0)
            step_ov(1)
            torch.cuda.synchronize(dev)
            works = [None, None]
            dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(K):
                last = step_ov(i)
            torch.cuda.synchronize(dev)
            dist.barrier()
            elapsed_gp = time.perf_counter() - t0
            # the last step's gathered rows hold this rank's block as extracted
            xchk = bool(torch.equal(outs[(K - 1) & 1][rank * C:(rank + 1) * C], last))
            del exts, fx2, outs
        # the all-gather alone (median of 5), for the record
        rows = fx(pool[0])["rows"]
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(5):
            dist.barrier()
            g0 = time.perf_counter()
            gather_rows(rows, args.clips)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - g0)
        ag = {"ms": round(float(np.median(ts)) * 1e3, 4), "bytes": args.clips * OUT_BYTES_PER_CLIP,
              "collectives": 1, "backend": backend_name,
              "what": "every clip's packed 76-B result row (feat, start/end, n_frames, status) as written by "
                      "the kernel, one %s all_gather_into_tensor, no pack/unpack kernels" % backend_name}
    if world > 1:
        t = torch.tensor([elapsed_x, elapsed_gs, my_frames, kern_ms, kern_ms_iso,
                          -1.0 if elapsed_gp is None else elapsed_gp], dtype=torch.float64, device=dev)
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed_x, elapsed_gs, total_frames, kern_ms = tmax[0].item(), tmax[1].item(), tsum[2].item(), tmax[3].item()
        kern_ms_iso = tmax[4].item()
        elapsed_gp = tmax[5].item() if elapsed_gp is not None else None
        # value: the faster of the two step loops (both measured here, both in the line)
        elapsed_g = elapsed_gs if elapsed_gp is None else min(elapsed_gs, elapsed_gp)
        if xchk is not None:  # every rank's own block
            ok = torch.tensor([1 if xchk else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            xchk = bool(ok.item())
        if timed_ok is not None:  # every rank's last timed step
            ok = torch.tensor([1 if timed_ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            timed_ok = bool(ok.item())
    else:
        total_frames = my_frames

    peaks = measured_peaks(pool[0], dev)
    sweep = window_sweep(args, fx, pool[0], dev, world, rank) if args.sweep_clips > 0 else None
    cfg0 = configs0_leg(args, pool[0], dev, world) if args.cfg0 else None
    cfg1 = configs1_leg(args, fx, pool[0], dev, world) if args.small_clips > 0 else None
    knn = knn_leg(args, fx, pool[0], dev, world, rank) if args.knn_ref > 0 else None

    result = None
    if rank == 0:
        result = assemble_result(args, world, ranks_seen, rehearsal, backend_name, C, total_frames, elapsed_x,
                                 elapsed_g, kern_ms, kern_ms_iso, elapsed_gs, elapsed_gp, xchk)
        if peaks is not None:
            r = result["roofline"]
            r["measured_read_peak_gbs"] = peaks["read_gbs"]
            r["frac_of_measured_read"] = round(r["achieved"] / peaks["read_gbs"], 4)
            r["measured_copy_gbs"] = peaks["copy_gbs"]
            r["frac_of_measured_copy"] = round(r["achieved"] / peaks["copy_gbs"], 4)
            r["peaks_note"] = peaks["note"]
        result["timed_outputs_equal"] = timed_ok
        if timed_ok is not None:
            result["timed_outputs_check"] = ("the last replayed step's packed rows (feat, start/end, n_frames, "
                                             "status of all %d clips per rank) against one eager launch of the same "
                                             "batch into fresh buffers, bitwise" % C)
        if ag is not None:
            result["allgather"] = ag
        if cfg0 is not None:
            result["configs0"] = cfg0
        if cfg1 is not None:
            result["configs1"] = cfg1
        if sweep is not None:
            result["window_sweep"] = sweep
        if knn is not None:
            result["knn"] = knn
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(fx, pool[0], L, S, args.window, vad, args.cpu_seconds)
            result["cpu_baseline_reference_semantics"] = cpu_baseline_reference_semantics(
                pool[0], L, S, args.window, vad, args.cpu_seconds * 0.75)
            if cfg0 is not None:
                fx0 = FeatureExtractor(1024, 512, "hamming", True, device=dev)
                cfg0["cpu_baseline"] = cpu_baseline(fx0, pool[0], 1024, 512, "hamming", True, args.cpu_seconds / 2)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def measured_peaks(batch, dev, reps=5):
    """The HBM rates this box reaches on the benchmark's own resident batch (csrc/probe.hip,
    libdsp_probe.so): a streaming read of every byte with 16-B loads, and a copy of it (read +
    write bytes), median of ``reps`` launches each by HIP events.  None when the probe library is
    absent (it is built by the same Makefile)."""
    import ctypes
    import torch
    path = os.path.join(REPO, "dsp-audioreclabs_amd", "lib", "libdsp_probe.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.dsp_probe_read.argtypes = [vp, i64, vp, vp]
    L.dsp_probe_copy.argtypes = [vp, vp, i64, vp]
    src = batch.reshape(-1)
    nbytes = (src.numel() * src.element_size()) // 16 * 16
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream(dev)
    h = ctypes.c_void_p(st.cuda_stream)
    rd = timed_launches(lambda: L.dsp_probe_read(ctypes.c_void_p(src.data_ptr()), nbytes,
                                                 ctypes.c_void_p(out.data_ptr()), h), reps, st)
    cp = timed_launches(lambda: L.dsp_probe_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                                 nbytes, h), reps, st)
    del dst
    return {"read_gbs": round(nbytes / (rd * 1e-3) / 1e9, 1), "copy_gbs": round(2 * nbytes / (cp * 1e-3) / 1e9, 1),
            "note": "measured on this box over the %.2f GB resident batch (csrc/probe.hip): read = every byte once "
                    "with 16-B loads, copy = read + write bytes; HIP events, mean of %d launches" % (nbytes / 1e9, reps)}


def window_sweep(args, fx0, batch, dev, world, rank):
    """configs[2]: --sweep-clips clips (sharded over the ranks) x the three reference windows,
    one fused launch per window over the resident PCM (experiment_window_comparison,
    experiments/run_experiments.py:343-347).  Per-window frames/s from HIP-event launch times."""
    import torch
    import torch.distributed as dist
    from src.distributed import shard_range
    from src.pipeline import FeatureExtractor
    lo, hi = shard_range(min(args.sweep_clips, args.clips), rank, world)
    n = min(hi - lo, batch.shape[0])
    sub = batch[:n]
    stream = torch.cuda.current_stream(dev)
    res = {}
    for win in ("rectangular", "hamming", "hanning"):
        fx = FeatureExtractor(fx0.L, fx0.S, win, fx0.do_vad, device=dev)
        out = fx(sub)
        assert not (out["status"].cpu().numpy() & 0xFF).any()
        nv = ((sub.shape[1] - fx0.L) // fx0.S + 1) if fx0.do_vad else 0
        fr = out["n_frames"].to(torch.int64).sum().item() + nv * n
        ms = timed_launches(lambda: fx(sub), 5, stream)
        t = torch.tensor([ms, fr], dtype=torch.float64, device=dev)
        if world > 1:
            tm = t.clone()
            dist.all_reduce(tm, op=dist.ReduceOp.MAX)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            ms, fr = tm[0].item(), t[1].item()
        res[win] = {"frames_per_s": round(fr / (ms * 1e-3), 1), "kernel_ms": round(ms, 4)}
    return {"config": "BASELINE configs[2]: %d x 1 s clips per window" % min(args.sweep_clips, args.clips),
            "windows": res}


def configs0_leg(args, batch, dev, world):
    """BASELINE configs[0]'s frame sizes (run.py --experiment classifier with Hamming frames of
    1024 / 512 samples, /root/reference/config.py:35-40) on the rank's resident clips: GPU
    frames/s (VAD frames + feature frames) from HIP-event launch times."""
    import torch
    import torch.distributed as dist
    from src.pipeline import FeatureExtractor
    fx = FeatureExtractor(1024, 512, "hamming", True, device=dev)
    out = fx(batch)
    assert not (out["status"].cpu().numpy() & 0xFF).any()
    n, N = batch.shape
    fr = out["n_frames"].to(torch.int64).sum().item() + ((N - 1024) // 512 + 1) * n
    ms = timed_launches(lambda: fx(batch), 5, torch.cuda.current_stream(dev))
    t = torch.tensor([ms, fr], dtype=torch.float64, device=dev)
    if world > 1:
        tm = t.clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        ms, fr = tm[0].item(), t[1].item()
    byts = n * world * (2 * N + OUT_BYTES_PER_CLIP)
    return {"config": "BASELINE configs[0] frame sizes: Hamming, frame_length 1024, frame_shift 512 samples, "
                      "VAD on; %d x 1 s clips" % (n * world),
            "frames_per_s": round(fr / (ms * 1e-3), 1), "kernel_ms": round(ms, 4),
            "hbm_frac": round(byts / (ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4)}


def configs1_leg(args, fx, batch, dev, world):
    """BASELINE configs[1]: 1 000 synthetic 1 s clips (Hamming, all features + VAD) in ONE launch
    on one GPU -- a latency-dominated batch (about 2 clips per workgroup).  Reported per launch:
    the kernel time (HIP events) and the host wall time of a synchronised call."""
    import torch
    n = min(args.small_clips, batch.shape[0])
    sub = batch[:n]
    out = fx(sub)
    assert not (out["status"].cpu().numpy() & 0xFF).any()
    fr = out["n_frames"].to(torch.int64).sum().item() + ((sub.shape[1] - fx.L) // fx.S + 1) * n
    ms = timed_launches(lambda: fx(sub), 20, torch.cuda.current_stream(dev))
    walls = []
    for _ in range(20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fx(sub)
        torch.cuda.synchronize(dev)
        walls.append(time.perf_counter() - t0)
    return {"config": "BASELINE configs[1]: %d x 1 s clips, one launch, Hamming, E/M/ZCR + VAD (rank 0)" % n,
            "kernel_ms": round(ms, 4), "wall_ms_per_call": round(float(np.median(walls)) * 1e3, 4),
            "frames_per_s_kernel": round(fr / (ms * 1e-3), 1)}


def knn_leg(args, fx, batch, dev, world, rank):
    """BASELINE configs[4] beside the headline metric: exact k-NN (KNeighborsClassifier
    semantics) on the EXTRACTED feature vectors of the north-star batch, as the reference chains
    them (experiments/run_experiments.py:262-280, src/models.py:33-35): each rank's extraction of
    its shard -> one gather of the packed result rows (every rank holds every clip's 15-d vector)
    -> normalize_features on the device (dsp_zscore_fit / dsp_zscore_apply, fp64) -> the first
    --knn-ref vectors each queried against all of them (self excluded, k = --knn-k), queries
    sharded over the ranks, (idx, dist, pred) gathered in one collective.  Labels are clip index
    mod 10 (the synthetic batch has no classes; they only feed the vote).  Timed: the sharded
    search + its gather (median of 3).  Not part of ``value``; reported with its fp32 roofline:
    45 algorithmic flop per pair (15 sub + 15 mul + 15 add) against 157.3 TF/s, the fp32 peak of
    both the matrix cores (v_mfma_f32_16x16x4_f32, the screen's distances) and the VALU."""
    import torch
    import torch.distributed as dist
    from src.distributed import gather_rows, knn_sharded, result_views
    from src.pipeline import KnnIndex, zscore_apply, zscore_fit
    res = result_views(gather_rows(fx(batch)["rows"], args.clips))
    assert not (res["status"] & 0xFF).any().item()
    n = min(args.knn_ref, args.clips)
    feat = res["feat"][:n].to(torch.float64)
    torch.cuda.synchronize(dev)
    z0 = time.perf_counter()
    mu, sd = zscore_fit(feat)
    Xd = zscore_apply(feat, mu, sd)
    torch.cuda.synchronize(dev)
    zs_ms = (time.perf_counter() - z0) * 1e3
    yd = (torch.arange(n, device=dev) % 10).to(torch.int32)
    # fit: the reference set converted once (KnnIndex; every rank holds it), timed on its own
    index = KnnIndex(Xd, yd, args.knn_k, n_classes=10)
    from src.distributed import shard_range
    lo, hi = shard_range(n, rank, world)
    torch.cuda.synchronize(dev)
    f0 = time.perf_counter()
    index.query(Xd[lo:lo + 1], self_offset=lo)  # the first query prepares the reference set
    torch.cuda.synchronize(dev)
    fit_ms = (time.perf_counter() - f0) * 1e3

    def knn_fn(ref, lab, q, k, off):
        return index.query(q, self_offset=off)
    knn_sharded(knn_fn, Xd, yd, Xd, args.knn_k, self_query=True)  # warm-up
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(3):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        last = knn_sharded(knn_fn, Xd, yd, Xd, args.knn_k, self_query=True)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    # untimed: how many queries the fp32 screen could not certify (exhaustive fp64 fallback)
    st = {}
    index.query(Xd[lo:hi], self_offset=lo, stats=st)
    fb = torch.tensor([float(st.get("fallbacks", 0))], dtype=torch.float64, device=dev)
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = tt.item()
        dist.all_reduce(fb)
    X = Xd.cpu().numpy()
    y = yd.cpu().numpy()
    pairs = float(n) * n
    tf = pairs * 45 / t / 1e12
    cpu = None
    if rank == 0:
        # the C oracle (sklearn semantics, fp64) on a bounded sample of the same queries, timed on
        # the host cores; the answers of the last timed run for those queries must equal it bit
        # for bit
        idx, dist_, pred = last
        cpu = knn_cpu_baseline(X, y, args.knn_k, idx, dist_, pred)
    out = {"metric": "k-NN pairs/s (15-d, exact, k=%d, self-query, gathered)" % args.knn_k,
            "value": round(pairs / t, 1), "unit": "pairs/s", "ms": round(t * 1e3, 4),
            "ref": n, "queries": n, "queries_per_rank": -(-n // world),
            "roofline": {"bound": "mfma-f32", "achieved": round(tf, 2), "peak": 157.3 * world, "unit": "TFLOP/s",
                         "frac": round(tf / (157.3 * world), 4), "flop_per_pair": 45,
                         "note": "whole-job wall time of the queries (screen, merge, fallback, the result "
                                 "all-gather); the reference set's fp32 conversion is the index's fit, %.3f ms "
                                 "once (KNeighborsClassifier.fit's side)" % fit_ms},
            "data": "extracted features: the z-scored 15-d statistics the fused kernel produced for the first %d "
                    "clips of the north-star batch (gathered over %d rank(s), normalize_features on the device "
                    "%.2f ms); labels clip index mod 10" % (n, world, zs_ms),
            "fallbacks": int(fb.item()),
            "fallbacks_note": "queries the fp32 screen could not certify, answered by the exhaustive fp64 scan"}
    if cpu is not None:
        out["parity_on_sample"] = cpu.pop("parity_on_sample")
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu
    return out


def knn_cpu_baseline(X, y, k, idx, dist, pred, nq=1000):
    """oracle.knn (a C restatement of KNeighborsClassifier's exact search + vote) over the first
    nq self-queries on this box's host cores; parity of the GPU's answers on those queries."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    threads, _, _ = host_cores()
    t0 = time.perf_counter()
    i0, d0, p0 = oracle.knn(X, y, X[:nq], k, n_classes=10, self_offset=0, nthreads=threads)
    dt = time.perf_counter() - t0
    ok_i = bool(np.array_equal(idx[:nq].cpu().numpy(), i0))
    ok_d = bool(np.array_equal(dist[:nq].cpu().numpy(), d0))
    ok_p = bool(np.array_equal(pred[:nq].cpu().numpy(), p0))
    return {"value": round(nq * X.shape[0] / dt, 1), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": "%d self-queries x %d reference rows, C oracle (exact fp64 brute force, sklearn "
                      "semantics), %d threads" % (nq, X.shape[0], threads),
            "parity_on_sample": {"queries": nq, "idx_exact": ok_i, "dist_exact": ok_d, "pred_exact": ok_p}}


def host_cores():
    """(cores this process may use, CPUs visible): the affinity set, capped by the cgroup CPU
    quota when one is set (a GPU box shows the whole machine's CPUs but grants a share)."""
    vis = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return (min(vis, quota) if quota else vis), vis, quota


def cpu_baseline(fx, batch, L, S, window, vad, budget_s):
    """The C oracle (a restatement of the reference's numpy pipeline, oracle/) on the host
    cores of this box, on a bounded sample of the benchmark's own clips; its outputs on that
    sample are compared with the GPU's (endpoints and frame counts exact, features 1e-5)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from src.pipeline import create_window
    w = create_window(window, L)
    n_host = min(batch.shape[0], 2000)
    host = batch[:n_host].cpu().numpy()
    C, N = host.shape
    flat = np.ascontiguousarray(host.reshape(-1))
    off = np.arange(C + 1, dtype=np.int64) * N
    threads, visible, quota = host_cores()
    nv = (N - L) // S + 1 if (vad and N >= L) else 0

    def run(nt, clips):
        o = off[:clips + 1]
        t = time.perf_counter()
        r = oracle.process_batch(flat[:o[-1]], o, L, S, w, do_vad=vad, nthreads=nt)
        dt = time.perf_counter() - t
        return (nv * clips + int(r["n_frames"].sum())) / dt, dt, r

    run(threads, min(C, 64 * threads))  # warm-up (thread arenas, page faults, clocks)
    rate, dt, ref = run(threads, C)
    # parity spot check of the sample against the device results of the same clips
    got = {k: v[:C].cpu().numpy() for k, v in fx(batch[:C]).items()}
    se_ok = bool(np.array_equal(got["start_end"], ref["start_end"]))
    nf_ok = bool(np.array_equal(got["n_frames"], ref["n_frames"]))
    rel = np.abs(got["feat"] - ref["feat"]) / np.maximum(np.abs(ref["feat"]), 1e-30)
    reps = 1
    total_frames, total_t = rate * dt, dt
    while total_t < budget_s and reps < 5000:
        r2, d2, _ = run(threads, C)
        total_frames += r2 * d2
        total_t += d2
        reps += 1
    one, _, _ = run(1, min(C, 200))
    return {"value": round(total_frames / total_t, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "host_cpus_visible": visible, "cgroup_cpu_quota": quota,
            "sample": "%d passes over %d of the benchmark's clips (%.1f s), C restatement of the reference "
                      "numpy pipeline (oracle/dsp_oracle.c), %d threads (all usable cores: affinity %d, "
                      "cgroup quota %s); 1 thread: %.4g frames/s"
                      % (reps, C, total_t, threads, visible, quota, one),
            "parity_on_sample": {"clips": C, "start_end_exact": se_ok, "n_frames_exact": nf_ok,
                                 "feat_max_rel_err": float(np.nanmax(rel)),
                                 "feat_cells_over_1e-5_rel": int(np.nansum(rel > 1e-5))}}


def cpu_baseline_reference_semantics(batch, L, S, window, vad, budget_s, n_sample=1000):
    """SURVEY.md §8d's baseline as the reference runs it: its own numpy algorithm, one clip at a
    time with a Python loop over frames (oracle/np_reference.py, bit-exact against the reference's
    golden vectors), over a process pool of every usable host core, on a bounded sample of the
    benchmark's clips.  Its outputs on the sample are checked against the C oracle (start/end,
    frame counts and all 15 features bit for bit)."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import np_reference
    import oracle
    from src.pipeline import create_window
    w = create_window(window, L)
    host = batch[:n_sample].cpu().numpy()
    C, N = host.shape
    threads, visible, quota = host_cores()
    nv = (N - L) // S + 1 if (vad and N >= L) else 0
    per = -(-C // (4 * threads))  # ~4 tasks per worker
    tasks = [(host[a:a + per], L, S, w, vad) for a in range(0, C, per)]
    # spawned workers (fresh interpreters): nothing GPU-side is inherited by a fork
    with mp.get_context("spawn").Pool(threads) as pool:
        pool.map(np_reference.process_many, [(host[:2], L, S, w, vad)] * threads)  # start-up, imports
        passes, t_total, frames = 0, 0.0, 0
        first = None
        while passes == 0 or (t_total < budget_s and passes < 50):
            t0 = time.perf_counter()
            res = pool.map(np_reference.process_many, tasks)
            t_total += time.perf_counter() - t0
            passes += 1
            nf = np.concatenate([r[3] for r in res])
            frames += int(nf.sum()) + nv * C
            if first is None:
                first = res
    st = np.concatenate([r[0] for r in first])
    feat = np.concatenate([r[1] for r in first])
    se = np.concatenate([r[2] for r in first])
    nf = np.concatenate([r[3] for r in first])
    flat = np.ascontiguousarray(host.reshape(-1))
    ref = oracle.process_batch(flat, np.arange(C + 1, dtype=np.int64) * N, L, S, w, do_vad=vad, nthreads=threads)
    ok = ref["status"] == 0
    t1 = time.perf_counter()
    np_reference.process_many((host[:20], L, S, w, vad))  # one process, for the per-core rate
    one = (nv * 20 + int(nf[:20].sum())) / (time.perf_counter() - t1)
    return {"value": round(frames / t_total, 1), "unit": "frames/s", "cores": threads, "kind": "reference-semantics",
            "sample": "%d passes over %d of the benchmark's clips (%.1f s): the reference's numpy algorithm as it "
                      "runs (per-clip, per-frame Python loop; oracle/np_reference.py, bit-exact against the "
                      "reference's golden vectors) on a spawn pool of %d processes (all usable cores); 1 process: "
                      "%.4g frames/s" % (passes, C, t_total, threads, one),
            "parity_vs_c_oracle": {"clips": C, "status_equal": bool(np.array_equal(st, ref["status"])),
                                   "start_end_equal": bool(np.array_equal(se[ok], ref["start_end"][ok])),
                                   "n_frames_equal": bool(np.array_equal(nf[ok], ref["n_frames"][ok])),
                                   "feat_bit_exact": bool(np.array_equal(feat[ok], ref["feat"][ok]))}}


if __name__ == "__main__":
    sys.exit(main())
