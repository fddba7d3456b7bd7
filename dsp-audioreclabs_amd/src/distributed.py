"""One process per GPU: clip sharding and the single exchange step.

Clips are independent, so rank r of P processes the contiguous block ``shard_range(B, r, P)``
with no collective inside the step.  The only exchange is before KNN: every rank needs the
whole [B, 15] feature matrix (and labels), gathered with ``all_gather`` -- RCCL over xGMI
with the "nccl" backend, gloo on CPU in the tests.  KNN then shards the queries and gathers
the per-query results the same way.
"""
import torch
import torch.distributed as dist


def world():
    """(rank, world_size) of the default group, (0, 1) when not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(total, rank, world_size):
    """Contiguous block [lo, hi) of ``total`` items owned by ``rank``: the first
    ``total % world_size`` ranks get one extra item."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("bad rank / world size")
    base, extra = divmod(int(total), world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def all_gather_rows(x, total=None, group=None):
    """Concatenate every rank's rows (in rank order) on every rank.

    Blocks may differ in length by the shard_range rule; they are padded to the largest block
    for the collective (all_gather needs equal shapes) and trimmed afterwards.
    """
    rank, ws = world()
    if ws == 1:
        return x
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    pad = x
    if x.shape[0] < m:
        pad = torch.cat([x, x.new_zeros((m - x.shape[0],) + tuple(x.shape[1:]))])
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad.contiguous(), group=group)
    out = torch.cat([p[:s] for p, s in zip(parts, sizes)])
    if total is not None and out.shape[0] != total:
        raise RuntimeError("gathered %d rows, expected %d" % (out.shape[0], total))
    return out


def extract_sharded(extract_fn, make_shard, total):
    """Run ``extract_fn(make_shard(lo, hi))`` on this rank's block and gather the results.

    ``extract_fn`` returns a dict of row-major tensors (feat, start_end, n_frames, status ...);
    every entry is all-gathered so each rank ends with the full-batch dict.
    """
    rank, ws = world()
    lo, hi = shard_range(total, rank, ws)
    out = extract_fn(make_shard(lo, hi))
    return {k: all_gather_rows(v, total) for k, v in out.items()}


def knn_sharded(knn_fn, ref, labels, queries, k, self_query=False):
    """Query-sharded KNN: the reference set is replicated (post-gather), rank r answers the
    queries of its shard_range block, and (idx, dist, pred) are gathered back.

    ``knn_fn(ref, labels, q, k, self_offset)`` -> (idx, dist, pred); with ``self_query`` the
    queries are the reference rows themselves and each excludes its own row.
    """
    rank, ws = world()
    lo, hi = shard_range(queries.shape[0], rank, ws)
    idx, d, pred = knn_fn(ref, labels, queries[lo:hi], k, lo if self_query else -1)
    n = queries.shape[0]
    return all_gather_rows(idx, n), all_gather_rows(d, n), all_gather_rows(pred, n)
