#!/usr/bin/env python3
"""Are the extraction's re-reads HBM traffic?  

FETCH_SIZE counts Infinity-Cache hits as well as HBM reads (MI355X_MICROARCH.md), so the
extraction's 1.43x of algorithmic bytes does not say how much of it costs HBM time.  This probe
times, over the same resident batch of 1 s clips as bench.py: (a) a streaming read of every byte
once; (b) the same walk in 88 200-B clip blocks on the extraction's grid (3 workgroups per CU),
each block read whole and the previous block's middle 27 % (the size of a bench crop) read again
one block later -- the re-read shape of the extraction; (c) (b) with the whole previous block
re-read (2x bytes).  If the re-reads reached HBM, (b) would take ~1.27x and (c) ~2x of (a).
Run it under `rocprofv3 --pmc FETCH_SIZE` for the counter side.  Prints one JSON line.
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dsp-audioreclabs_amd"))


def main():
    import torch
    from src.synth import make_batch_device
    dev = torch.device("cuda", 0)
    clips = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    x = make_batch_device(clips, dev).reshape(-1)
    L = ctypes.CDLL(os.path.join(REPO, "dsp-audioreclabs_amd", "lib", "libdsp_probe.so"))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.dsp_probe_read.argtypes = [vp, i64, vp, vp]
    L.dsp_probe_reread.argtypes = [vp, i64, i64, i64, i64, ctypes.c_int, vp, vp]
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    h = ctypes.c_void_p(st.cuda_stream)
    blk = 88192  # 5 512 16-B vectors ~ one 1 s clip (88 200 B)
    nbytes = (x.numel() * 2) // blk * blk
    src = ctypes.c_void_p(x.data_ptr())
    o = ctypes.c_void_p(out.data_ptr())

    def timed(fn, n=5):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in ev:
            a.record(st)
            assert fn() == 0
            b.record(st)
        torch.cuda.synchronize()
        return sorted(a.elapsed_time(b) for a, b in ev)[n // 2]

    crop = (blk * 27 // 100) // 16 * 16
    off = ((blk - crop) // 2) // 16 * 16
    t_read = timed(lambda: L.dsp_probe_read(src, nbytes, o, h))
    t_block = timed(lambda: L.dsp_probe_reread(src, nbytes, blk, 0, 0, 0, o, h))
    t_crop = timed(lambda: L.dsp_probe_reread(src, nbytes, blk, off, crop, 0, o, h))
    t_all = timed(lambda: L.dsp_probe_reread(src, nbytes, blk, 0, blk, 0, o, h))
    r = {"bytes": nbytes, "read_once_ms": round(t_read, 4), "blocks_no_reread_ms": round(t_block, 4),
         "blocks_reread_crop27_ms": round(t_crop, 4), "blocks_reread_whole_ms": round(t_all, 4),
         "read_once_gbs": round(nbytes / t_read / 1e6, 1),
         "crop_reread_cost": round(t_crop / t_block, 4), "whole_reread_cost": round(t_all / t_block, 4),
         "note": "medians of 5 launches by HIP events; block = one 88 192-B clip, re-read one block later by the "
                 "same workgroup, 3 workgroups per CU"}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
