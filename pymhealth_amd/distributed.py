"""Window sharding across the GPUs of a node (one process per GPU, torch.distributed).

Windows are independent (the reference's prange, src/mhealth/util/windows.py:70-71), so
the path shards with no data-path collective: rank r owns the contiguous global window
range ``shard_range(nw, r, world)`` and needs samples ``[w0*S, (w1-1)*S + W)`` — the
windows' own samples plus a (W - S)-sample halo when windows overlap. RCCL (backend
"nccl" on ROCm, over xGMI) is used only to move signal slices out of a rank that holds
the whole record (``scatter_signal``) and feature rows back (``gather_features``).

Every launch keeps GLOBAL window indices (``base_window``), so global window 0 keeps the
reference's serial row-0 numerics (windows.py:87) and a sharded run is bit-identical to
a single-GPU run.
"""
import torch
import torch.distributed as dist

from .engine import num_windows


def shard_range(nw, rank, world):
    """Contiguous window range [w0, w1) of ``rank`` (sizes differ by at most one)."""
    q, r = divmod(int(nw), int(world))
    w0 = rank * q + min(rank, r)
    return w0, w0 + q + (1 if rank < r else 0)


def sample_range(w0, w1, wsize, wstep):
    """Samples [s0, s1) that windows [w0, w1) read (empty range if no windows)."""
    if w1 <= w0:
        return w0 * wstep, w0 * wstep
    return w0 * wstep, (w1 - 1) * wstep + wsize


def _comm_device(t_device):
    """Where a collective's buffers live: RCCL ("nccl") moves device memory over xGMI;
    gloo (CPU tests, rehearsals) needs host tensors."""
    return torch.device("cpu") if dist.get_backend() == "gloo" else t_device


def scatter_signal(x, n_samples, wsize, wstep, *, src=0, group=None, device=None, channels=None,
                   dtype=torch.float32):
    """Send every rank the sample slice its windows need, from rank ``src``.

    x: the whole (N,) or (N, C) signal on rank ``src`` (None elsewhere; ``channels`` /
    ``dtype`` then give the slice's shape: C > 1 is an (n, C) slice). Returns
    (local_slice, w0, w1) on every rank, on ``device``; ``local_slice[0]`` is sample w0*S.
    Point-to-point sends (slices differ in length by the (W - S) halo of overlapping
    windows); one per rank, all in flight together.
    """
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    nw = num_windows(n_samples, wsize, wstep)
    w0, w1 = shard_range(nw, rank, world)
    s0, s1 = sample_range(w0, w1, wsize, wstep)
    if rank == src:
        comm = _comm_device(x.device)
        reqs = []
        for r in range(world):
            if r == src:
                continue
            a0, a1 = shard_range(nw, r, world)
            b0, b1 = sample_range(a0, a1, wsize, wstep)
            if b1 > b0:
                reqs.append(dist.isend(x[b0:b1].contiguous().to(comm), dst=r, group=group))
        for q in reqs:
            q.wait()
        local = x[s0:s1]
    else:
        if x is not None:
            channels, dtype = (1 if x.dim() == 1 else x.shape[1]), x.dtype
        C = channels or 1
        shape = (s1 - s0,) if C == 1 else (s1 - s0, C)
        dev = device if device is not None else torch.device("cpu")
        buf = torch.empty(shape, dtype=dtype, device=_comm_device(dev))
        if s1 > s0:
            dist.recv(buf, src=src, group=group)
        local = buf.to(dev)
    return local, w0, w1


def local_features(local, w0, w1, wsize, wstep, feature_ids, compute=None, **kw):
    """Features of global windows [w0, w1) from the local slice starting at sample w0*S.

    ``compute`` defaults to the MI355X engine (``engine.window_features``); tests inject
    the CPU oracle through it to check the sharding arithmetic without a GPU.
    """
    if compute is None:
        from .engine import window_features as compute
    return compute(local, wsize, wstep, feature_ids, first_window=w0, n_windows=w1 - w0,
                   base_window=w0, **kw)


# gather_features' padded send / receive buffers, one set per (shape, dtype, device, group
# layout): a timed loop of gathers (bench.py with_gather, --strong) times the collective,
# not the allocator. Only the padding columns are cleared between calls.
_GATHER_BUFS = {}


def _gather_buffers(C, F, width, dtype, comm, world, is_dst, group):
    key = (C, F, width, dtype, str(comm), world, is_dst, id(group))
    b = _GATHER_BUFS.get(key)
    if b is None:
        pad = torch.zeros((C, F, width), dtype=dtype, device=comm)
        recv = torch.empty((world, C, F, width), dtype=dtype, device=comm) if is_dst else None
        b = _GATHER_BUFS[key] = (pad, recv)
    return b


def gather_features(local_out, nw, *, dst=0, group=None):
    """Concatenate every rank's (C, F, n_local) rows along windows on rank ``dst``.

    Ranks' shards differ by at most one window: pad to the largest and use one
    ``dist.gather`` (RCCL over xGMI; host buffers under gloo). Returns the (C, F, nw)
    result on ``dst`` (on local_out's device) and None elsewhere. The padded buffers are
    allocated once per shape (``_GATHER_BUFS``).
    """
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    C, F, n = local_out.shape
    width = shard_range(nw, 0, world)[1]        # rank 0 has the largest shard
    comm = _comm_device(local_out.device)
    pad, recv = _gather_buffers(C, F, width, local_out.dtype, comm, world, rank == dst, group)
    pad[:, :, :n].copy_(local_out)
    if n < width:
        pad[:, :, n:].zero_()
    bufs = list(recv.unbind(0)) if rank == dst else None
    dist.gather(pad, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    parts = []
    for r in range(world):
        a0, a1 = shard_range(nw, r, world)
        parts.append(bufs[r][:, :, :a1 - a0])
    return torch.cat(parts, dim=2).to(local_out.device)


def sharded_features(x, n_samples, wsize, wstep, feature_ids, *, src=0, dst=0, group=None,
                     device=None, compute=None, channels=None, dtype=torch.float32, **kw):
    """Scatter -> per-rank fused features -> gather: the whole multi-GPU path (the
    strong-scaling step of ``bench.py --strong``)."""
    local, w0, w1 = scatter_signal(x, n_samples, wsize, wstep, src=src, group=group,
                                   device=device, channels=channels, dtype=dtype)
    nw = num_windows(n_samples, wsize, wstep)
    out = local_features(local, w0, w1, wsize, wstep, feature_ids, compute=compute, **kw)
    return gather_features(out, nw, dst=dst, group=group)
