"""world_size-2 gloo run of the multi-GPU data flow on CPU: clip sharding with
no collective in the step, all-gather of the 15-d vectors, query-sharded KNN + gather.  The
per-shard compute here is the oracle (the HIP kernel needs the GPU); the product code under
test is src/distributed.py, which bench.py and the GPU path use unchanged."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, out_dir):
    import sys
    from conftest import PKG, REPO
    sys.path[:0] = [PKG, os.path.join(REPO, "oracle")]
    import torch.distributed as dist
    import oracle
    from src import distributed as D
    from src.pipeline import create_window
    from src.synth import make_batch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        B, L, S = 13, 1102, 441
        w = create_window("hamming", L)

        def make_shard(lo, hi):
            return make_batch(hi - lo, base_seed=11, start=lo, n_samples=8000)

        def extract(pcm):
            n, N = pcm.shape
            if n == 0:  # this rank's block is empty (total < world size)
                return {"feat": torch.zeros((0, 15), dtype=torch.float64),  # the oracle's dtypes
                        "start_end": torch.zeros((0, 2), dtype=torch.int64),
                        "n_frames": torch.zeros(0, dtype=torch.int64)}
            r = oracle.process_batch(pcm.reshape(-1), np.arange(n + 1, dtype=np.int64) * N, L, S, w)
            return {"feat": torch.as_tensor(r["feat"]), "start_end": torch.as_tensor(r["start_end"]),
                    "n_frames": torch.as_tensor(r["n_frames"])}

        def extract_rows(pcm):
            # FeatureExtractor's output layout: packed [n, 19] int32 rows and views of them
            r = extract(pcm)
            n = r["feat"].shape[0]
            rows = torch.zeros((n, 19), dtype=torch.int32)
            rows.view(torch.float32)[:, :15] = r["feat"].to(torch.float32)
            rows[:, 15:17] = r["start_end"].to(torch.int32)
            rows[:, 17] = r["n_frames"].to(torch.int32)
            return D.result_views(rows)

        got = D.extract_sharded(extract, make_shard, B)
        # packed rows: one all_gather_into_tensor, ragged (13 = 7 + 6), equal (16 = 8 + 8) and an
        # empty block (1 = 1 + 0)
        rows_r = {b: D.extract_sharded(extract_rows, make_shard, b) for b in (B, 16, 1)}
        labels = torch.arange(B, dtype=torch.int32) % 3
        X = got["feat"].to(torch.float64).numpy()

        def knn(ref, lab, q, k, self_off):
            if len(q) == 0:
                return (torch.zeros((0, k), dtype=torch.int32), torch.zeros((0, k), dtype=torch.float64),
                        torch.zeros(0, dtype=torch.int32))
            i, d, p = oracle.knn(ref, lab.numpy(), q, k, n_classes=3, self_offset=self_off)
            return torch.as_tensor(i), torch.as_tensor(d), torch.as_tensor(p)

        idx, dist_, pred = D.knn_sharded(knn, X, labels, X, 3, self_query=True)
        # one clip over two ranks: rank 1's block is empty and must still join the collectives
        one = D.extract_sharded(extract, make_shard, 1)
        i1, d1, p1 = D.knn_sharded(knn, X, labels, X[:1], 3, self_query=False)
        np.savez(os.path.join(out_dir, "rank%d.npz" % rank), feat=got["feat"].numpy(),
                 start_end=got["start_end"].numpy(), n_frames=got["n_frames"].numpy(),
                 idx=idx.numpy(), dist=dist_.numpy(), pred=pred.numpy(), one_feat=one["feat"].numpy(),
                 one_n=one["n_frames"].numpy(), i1=i1.numpy(), d1=d1.numpy(), p1=p1.numpy(),
                 **{"rows%d_%s" % (b, k): v.numpy() for b, g in rows_r.items() for k, v in g.items()})
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shard_gather(tmp_path):
    import oracle
    from src.pipeline import create_window
    from src.synth import make_batch
    ws = 2
    mp.spawn(_worker, args=(ws, _free_port(), str(tmp_path)), nprocs=ws, join=True)
    B, L, S = 13, 1102, 441
    pcm = make_batch(B, base_seed=11, n_samples=8000)
    full = oracle.process_batch(pcm.reshape(-1), np.arange(B + 1, dtype=np.int64) * 8000, L, S,
                                create_window("hamming", L))
    y = (np.arange(B) % 3).astype(np.int32)
    i0, d0, p0 = oracle.knn(full["feat"].astype(np.float64), y, full["feat"].astype(np.float64), 3,
                            n_classes=3, self_offset=0)
    for r in range(ws):
        got = np.load(tmp_path / ("rank%d.npz" % r))
        assert np.array_equal(got["feat"], full["feat"])  # every rank holds the whole matrix
        assert np.array_equal(got["start_end"], full["start_end"])
        assert np.array_equal(got["n_frames"], full["n_frames"])
        assert np.array_equal(got["idx"], i0) and np.array_equal(got["dist"], d0)
        assert np.array_equal(got["pred"], p0)
        assert np.array_equal(got["one_feat"], full["feat"][:1]) and np.array_equal(got["one_n"], full["n_frames"][:1])
        i1, d1, p1 = oracle.knn(full["feat"].astype(np.float64), y, full["feat"][:1].astype(np.float64), 3, n_classes=3)
        assert np.array_equal(got["i1"], i1) and np.array_equal(got["d1"], d1) and np.array_equal(got["p1"], p1)
        for b in (B, 16, 1):  # gather_rows: every rank holds every clip's packed row, in order
            fb = oracle.process_batch(make_batch(b, base_seed=11, n_samples=8000).reshape(-1),
                                      np.arange(b + 1, dtype=np.int64) * 8000, L, S, create_window("hamming", L))
            assert got["rows%d_rows" % b].shape == (b, 19)
            assert np.array_equal(got["rows%d_feat" % b], fb["feat"].astype(np.float32))
            assert np.array_equal(got["rows%d_start_end" % b], fb["start_end"])
            assert np.array_equal(got["rows%d_n_frames" % b], fb["n_frames"])
            assert not got["rows%d_status" % b].any()
