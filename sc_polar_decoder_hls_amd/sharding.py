"""Multi-GPU layout of the decode: frames are independent, so a batch is split into
contiguous per-rank shards (one process per GPU) and every rank decodes its shard with no
data-path collective. Collectives appear only around the data path: a barrier + max-over-
ranks for timing, and an optional all-gather of the decoded words for verification.

The reference decodes one frame per top-level call (src/testbench/main.cpp:98-155 loops
frames through wrapper_in -> my_module -> wrapper_out); a batch of frames is the unit that
shards here.
"""

WAVE_FRAMES = 8   # frames per wave64 in the decode kernels; shard starts stay aligned to it


def shard_bounds(total, world, rank, align=WAVE_FRAMES):
    """Contiguous shard [start, start + count) of `total` frames for `rank` of `world`.

    Shards cover 0..total exactly once, differ in size by less than 2 `align` frames (one
    alignment unit plus the ragged tail), and start
    on multiples of `align` (so no wave straddles two ranks' halves of a batch)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %r / world %r" % (rank, world))
    if total < 0:
        raise ValueError("negative frame count")
    units = (total + align - 1) // align
    base, extra = divmod(units, world)
    u0 = rank * base + min(rank, extra)
    u1 = u0 + base + (1 if rank < extra else 0)
    start = min(total, u0 * align)
    end = min(total, u1 * align)
    return start, end - start


def frame_seed(base, rank):
    """Per-rank generator seed for synthetic frames (distinct streams per rank)."""
    return int(base) + 7919 * int(rank)


def max_over_ranks(values, dist=None, device=None):
    """Element-wise max of a list of floats over all ranks (timing aggregation)."""
    vals = [float(v) for v in values]
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return vals
    import torch
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def sum_over_ranks(counts, dist=None, device=None):
    """Error accounting over the whole job (the optional all-reduce of error
    counts; sc_error_counter.h:50-126 counts per stream): element-wise sum of an integer
    counter tensor over all ranks, in place on `device` (RCCL with the nccl backend). The
    per-frame sc_uint<10> wrap is applied before the sum, by polar_count_errors."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return counts
    t = counts.to(device) if device is not None else counts
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if t is not counts:
        counts.copy_(t.to(counts.device))
    return counts


def scatter_shards(full, total, frame_shape, dtype, dist=None, device=None):
    """Scatter a [total, *frame_shape] batch held by rank 0 into the per-rank shards of
    shard_bounds (RCCL over xGMI with the nccl backend). `full` is ignored on the other ranks
    (pass None); every rank knows the frame shape from its plan. Returns this rank's
    [count, *frame_shape] shard on `device`."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return full
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    spans = [shard_bounds(total, world, r) for r in range(world)]
    cap = max(c for _, c in spans)
    shape = (cap,) + tuple(frame_shape)
    out = torch.empty(shape, dtype=dtype, device=device)
    parts = None
    if rank == 0:
        parts = []
        for start, count in spans:   # equal-size (padded) chunks, as scatter requires
            buf = torch.zeros(shape, dtype=dtype, device=device)
            buf[:count] = full[start:start + count]
            parts.append(buf)
    dist.scatter(out, parts, src=0)
    return out[: spans[rank][1]]


def gather_shards(local, total, dist=None, device=None):
    """All-gather the per-rank decoded words [count, words] (int64 tensors) into the full
    [total, words] batch on every rank (verification, and the gather half of the C4
    scatter/gather mode of bench.py)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    import torch
    world = dist.get_world_size()
    counts = [shard_bounds(total, world, r)[1] for r in range(world)]
    cap = max(counts)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device if device is None else device)
    pad[: local.shape[0]] = local.to(pad.device)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)


def gather_to_root(local, total, dist=None, device=None):
    """Gather the per-rank [count, ...] results into [total, ...] on rank 0 (None elsewhere)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    counts = [shard_bounds(total, world, r)[1] for r in range(world)]
    cap = max(counts)
    dev = local.device if device is None else device
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[: local.shape[0]] = local.to(dev)
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, parts, dst=0)
    if rank != 0:
        return None
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
