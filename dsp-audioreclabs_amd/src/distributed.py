"""One process per GPU: clip sharding and the single exchange step.

Clips are independent, so rank r of P processes the contiguous block ``shard_range(B, r, P)``
with no collective inside the step.  The only exchange is before KNN: every rank needs the
whole [B, 15] feature matrix (and the per-clip endpoints, frame counts, status).  The extraction
writes each clip's results as one packed 76-B row (``rows`` [B, 19] int32, ABI 6), so the exchange
is ONE ``all_gather_into_tensor`` of those rows (``gather_rows``) -- no pack, pad or unpack
kernels around it -- RCCL over xGMI with the "nccl" backend, gloo on CPU in the tests.  Block
sizes follow from ``shard_range`` on every rank, so no size exchange and no host sync precede the
collective.  KNN then shards the queries and gathers the per-query
results (idx, dist, pred) the same way, again as one collective.
"""
import math

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


def _pack_rows(tensors, rows):
    """dict of tensors with ``rows`` leading rows -> (uint8 [rows, row_bytes], layout)."""
    cols, layout = [], []
    for name, t in tensors.items():
        if t.shape[0] != rows:
            raise ValueError("%s has %d rows, expected %d" % (name, t.shape[0], rows))
        # explicit column count: an empty block (total < world size) still packs as [0, row_bytes]
        # and reaches the collective with the other ranks
        b = t.contiguous().reshape(rows, math.prod(t.shape[1:])).view(torch.uint8)
        layout.append((name, t.dtype, tuple(t.shape[1:]), b.shape[1]))
        cols.append(b)
    return torch.cat(cols, dim=1) if cols else None, layout


def _unpack_rows(packed, layout):
    out, c = {}, 0
    n = packed.shape[0]
    for name, dtype, tail, nb in layout:
        # clone, not contiguous(): a one-row slice is already "contiguous" at a byte offset that
        # need not be a multiple of the element size, and view(dtype) needs an aligned offset
        out[name] = packed[:, c:c + nb].clone().view(dtype).reshape((n,) + tail)
        c += nb
    return out


def gather_packed(tensors, total, group=None):
    """All-gather several row-aligned tensors (this rank's ``shard_range`` block of ``total``
    rows each) in rank order, as one collective over a packed byte matrix.

    Returns {name: tensor [total, ...]} on every rank.
    """
    rank, ws = world()
    if ws == 1:
        return dict(tensors)
    sizes = []
    for r in range(ws):
        lo, hi = shard_range(total, r, ws)
        sizes.append(hi - lo)
    rows = sizes[rank]
    packed, layout = _pack_rows(tensors, rows)
    m = max(sizes)
    if rows < m:
        packed = torch.cat([packed, packed.new_zeros((m - rows, packed.shape[1]))])
    parts = [torch.empty_like(packed) for _ in range(ws)]
    dist.all_gather(parts, packed, group=group)
    full = torch.cat([p[:s] for p, s in zip(parts, sizes)])
    return _unpack_rows(full, layout)


def gather_rows(rows, total, group=None):
    """All-gather this rank's ``shard_range`` block of ``total`` packed result rows (``rows``
    [n, W], contiguous) in rank order: ONE ``all_gather_into_tensor`` straight from the
    extraction's own output buffer.  Returns [total, W] on every rank -- the collective's output
    itself when the blocks are equal (every bench configuration: 100 000 clips over 1/2/4/8
    ranks); ragged blocks are padded to the largest and cut back (two copies, off the bench path).
    """
    import torch
    rank, ws = world()
    if ws == 1:
        return rows
    sizes = [shard_range(total, r, ws) for r in range(ws)]
    sizes = [hi - lo for lo, hi in sizes]
    if rows.shape[0] != sizes[rank]:
        raise ValueError("rank %d holds %d rows, its block is %d" % (rank, rows.shape[0], sizes[rank]))
    m = max(sizes)
    src = rows.contiguous()
    if src.shape[0] < m:
        src = torch.cat([src, src.new_zeros((m - src.shape[0],) + tuple(src.shape[1:]))])
    out = src.new_empty((ws * m,) + tuple(src.shape[1:]))
    dist.all_gather_into_tensor(out, src, group=group)
    if all(s_ == m for s_ in sizes):
        return out
    return torch.cat([out[r * m:r * m + sizes[r]] for r in range(ws)])


def gather_rows_async(rows, out, group=None):
    """``gather_rows`` for equal blocks into a caller-owned ``out`` [world * n, W], issued on the
    current stream without waiting: returns the collective's work handle (``work.wait()`` makes the
    caller's current stream wait for it).  With it the exchange of one batch can run beside the
    extraction of the next (bench.py's N > 1 step, two output buffers)."""
    rank, ws = world()
    if out.shape[0] != ws * rows.shape[0] or out.shape[1:] != rows.shape[1:]:
        raise ValueError("out must be [world * %d, ...] like rows" % rows.shape[0])
    if ws == 1:
        out.copy_(rows)
        return None
    return dist.all_gather_into_tensor(out, rows.contiguous(), group=group, async_op=True)


def result_views(rows):
    """The per-array results as views of packed rows [B, 19] (the layout of FeatureExtractor's
    ``rows``: feat[15] as f32 bits, start, end, n_frames, status)."""
    import torch
    return dict(rows=rows, feat=rows.view(torch.float32)[:, :15], start_end=rows[:, 15:17],
                n_frames=rows[:, 17], status=rows[:, 18])


def all_gather_rows(x, total=None, group=None):
    """Concatenate every rank's rows (in rank order) on every rank.

    With ``total`` the blocks are the ``shard_range`` blocks (one collective); without it the
    block sizes are exchanged first (blocks may be any size).
    """
    rank, ws = world()
    if ws == 1:
        return x
    if total is not None:
        return gather_packed({"x": x}, total, group)["x"]
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
    return torch.cat([p[:s] for p, s in zip(parts, sizes)])


def extract_sharded(extract_fn, make_shard, total):
    """Run ``extract_fn(make_shard(lo, hi))`` on this rank's block and gather the results.

    ``extract_fn`` returns FeatureExtractor's dict: its packed ``rows`` travel in one
    ``gather_rows`` collective and the per-array results come back as views of the gathered rows;
    any other row-major tensors (vad lists, sequences) in one more packed all-gather.
    """
    rank, ws = world()
    lo, hi = shard_range(total, rank, ws)
    out = extract_fn(make_shard(lo, hi))
    if "rows" not in out:
        return gather_packed(out, total)
    res = result_views(gather_rows(out["rows"], total))
    rest = {k: v for k, v in out.items() if k not in res}
    if rest:
        res.update(gather_packed(rest, total))
    return res


def knn_sharded(knn_fn, ref, labels, queries, k, self_query=False):
    """Query-sharded KNN: the reference set is replicated (post-gather), rank r answers the
    queries of its shard_range block, and (idx, dist, pred) are gathered back in one collective.

    ``knn_fn(ref, labels, q, k, self_offset)`` -> (idx, dist, pred); with ``self_query`` the
    queries are the reference rows themselves and each excludes its own row.
    """
    rank, ws = world()
    n = queries.shape[0]
    lo, hi = shard_range(n, rank, ws)
    idx, d, pred = knn_fn(ref, labels, queries[lo:hi], k, lo if self_query else -1)
    parts = {"idx": idx, "dist": d}
    if pred is not None:
        parts["pred"] = pred
    g = gather_packed(parts, n)
    return g["idx"], g["dist"], g.get("pred")
