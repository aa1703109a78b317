"""Sharding a frame batch over the GPUs of a node, and the one exchange step.

Frames are independent (a frame's key phase is the offset inside its own
payload), so encode and decode shard with no data-path collective: chunks
of `chunk` consecutive frames are dealt round-robin, chunk c to rank
c % world.  The only exchange is BASELINE config C5's gather
of every rank's framed output to one rank (`gather_frames`), a variable-size
point-to-point gather: over RCCL (torch.distributed backend "nccl") on the
MI355X node — each sender uses its own xGMI link into the root — and over
gloo on CPU in the tests.
"""
import numpy as np


def rank_frames(rank, world, n_total, chunk=1024):
    """Global indices of the frames rank `rank` owns, in local order."""
    n_chunks = (n_total + chunk - 1) // chunk
    mine = np.arange(rank, n_chunks, world, dtype=np.int64)
    idx = (mine[:, None] * chunk + np.arange(chunk, dtype=np.int64)[None, :]).reshape(-1)
    return idx[idx < n_total]


def gather_frames(wire, wire_off, dst=0, group=None):
    """Gather every rank's framed output to rank `dst` with torch.distributed
    (the gloo path of the CPU tests; the RCCL path of a deployment is the
    C-ABI's wsg_mgpu_encode_gather, cppserver_amd.MultiGPU).

    wire: uint8 tensor (this rank's encoded frames, back to back; at least
    wire_off[-1] bytes); wire_off: int64 tensor of n_local + 1 frame offsets.
    Returns on `dst` a list of (wire, wire_off) per rank (rank order), None
    elsewhere.  Sizes go first (all_gather), then one grouped batch of
    isend/irecv so all senders stream into the root concurrently.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = wire.device
    sizes = torch.stack([wire_off[-1].to(torch.int64), torch.tensor(wire_off.numel(), device=dev)])
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    all_sizes = torch.stack(all_sizes).cpu().tolist()   # one host sync for every rank's sizes
    nbytes = all_sizes[rank][0]

    if rank != dst:
        ops = [dist.P2POp(dist.isend, wire[:nbytes].contiguous(), dst, group=group),
               dist.P2POp(dist.isend, wire_off.contiguous(), dst, group=group)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return None

    out = [None] * world
    ops = []
    for r in range(world):
        nb, no = all_sizes[r]
        if r == dst:
            out[r] = (wire[:nb], wire_off)
            continue
        w = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)[:nb]
        o = torch.empty(no, dtype=torch.int64, device=dev)
        out[r] = (w, o)
        ops.append(dist.P2POp(dist.irecv, w, r, group=group))
        ops.append(dist.P2POp(dist.irecv, o, r, group=group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def reassemble(parts, n_total, chunk=1024):
    """Per-rank (wire, wire_off) -> the job's frames in global order (one
    concatenation of per-chunk slices).  Returns (wire, wire_off).  The
    offsets come to the host once per rank (no per-chunk device sync)."""
    import torch

    world = len(parts)
    n_chunks = (n_total + chunk - 1) // chunk
    offs = [off.cpu().numpy() for _, off in parts]
    slices, sizes = [], []
    for c in range(n_chunks):
        r, j = c % world, c // world
        w, _ = parts[r]
        off = offs[r]
        lo, hi = j * chunk, min((j + 1) * chunk, len(off) - 1)
        slices.append(w[int(off[lo]): int(off[hi])])
        sizes.append(np.diff(off[lo: hi + 1]))
    dev = parts[0][0].device
    wire = torch.cat(slices) if slices else torch.empty(0, dtype=torch.uint8, device=dev)
    wire_off = np.zeros(n_total + 1, dtype=np.int64)
    if sizes:
        wire_off[1:] = np.cumsum(np.concatenate(sizes))
    return wire, torch.from_numpy(wire_off).to(dev)
