"""The multi-rank path with the HIP kernels in it: two processes on the one GPU of
the box, joined by gloo (RCCL needs one GPU per rank), each extracting its shard_range block with
the fused kernel and answering its block of KNN queries on the device, the results exchanged by
src/distributed.py's gather_rows (ONE all_gather_into_tensor of the kernel's packed 76-B result
rows; 3 001 clips = 1 501 + 1 500, so the ragged-block path) exactly as bench.py does over RCCL.  The gathered results
must equal one single-process launch bit for bit (features are position independent, so an odd
shard size changes nothing) and the oracle's KNN."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, L, S, K = 3001, 1102, 441, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, out_dir):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    from src import distributed as D
    from src.pipeline import FeatureExtractor, KnnIndex
    from src.synth import make_batch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        dev = torch.device("cuda", 0)
        fx = FeatureExtractor(L, S, "hamming", True, device=dev)

        def make_shard(lo, hi):
            return torch.as_tensor(make_batch(hi - lo, base_seed=21, start=lo)).to(dev)

        got = D.extract_sharded(fx, make_shard, B)  # FeatureExtractor's rows -> gather_rows
        assert got["rows"].shape == (B, 19)
        X = got["feat"].to(torch.float64)
        y = torch.arange(B, dtype=torch.int32, device=dev) % 4
        index = KnnIndex(X, y, K, n_classes=4)  # fit once on every rank, query the rank's block
        idx, dist_, pred = D.knn_sharded(lambda r, lab, q, k, so: index.query(q, self_offset=so),
                                         X, y, X, K, self_query=True)
        torch.cuda.synchronize(dev)
        if rank == 0:
            np.savez(os.path.join(out_dir, "gathered.npz"),
                     **{k: v.cpu().numpy() for k, v in got.items()},
                     idx=idx.cpu().numpy(), dist=dist_.cpu().numpy(), pred=pred.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo_on_one_gpu_equal_single_launch(tmp_path):
    import oracle
    from src.pipeline import FeatureExtractor
    from src.synth import make_batch

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    g = np.load(tmp_path / "gathered.npz")
    pcm = make_batch(B, base_seed=21)
    fx = FeatureExtractor(L, S, "hamming", True)
    one = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm, device="cuda:0")).items()}
    for k in ("feat", "start_end", "n_frames", "status"):
        assert np.array_equal(g[k], one[k]), k
    X = one["feat"].astype(np.float64)
    y = np.arange(B, dtype=np.int32) % 4
    i0, d0, p0 = oracle.knn(X, y, X, K, n_classes=4, self_offset=0)
    assert np.array_equal(g["idx"], i0) and np.array_equal(g["dist"], d0) and np.array_equal(g["pred"], p0)
