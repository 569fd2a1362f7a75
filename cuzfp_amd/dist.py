"""Multi-GPU sharding of the fixed-rate codec (one process per GPU, RCCL over xGMI).

zfp blocks are independent and, in fixed-rate mode, sit at fixed stream
offsets: block b owns bits [b*maxbits, (b+1)*maxbits).  Splitting a 3D array
into z-slabs whose depth is a multiple of 4 therefore splits the stream into
contiguous segments: rank r's slab encodes to exactly bytes
[r*B*maxbits/8, (r+1)*B*maxbits/8) of the single-GPU stream (B = blocks per
slab), provided B*maxbits is a multiple of 64.  Encode and
decode need no communication at all; the one real exchange is the optional
all-gather that assembles the global compressed stream on every rank
(``torch.distributed.all_gather_into_tensor`` = ``ncclAllGather`` on RCCL).
2D arrays shard by 4-row y-slabs and 1D arrays by 4-value x-ranges the same way.
"""
from __future__ import annotations


def slab_extent(n_slow: int, world: int, rank: int) -> tuple[int, int]:
    """[start, stop) along the slowest axis for `rank`: whole 4-deep block slabs,
    split as evenly as possible (earlier ranks take the remainder)."""
    slabs = (n_slow + 3) // 4
    per, extra = divmod(slabs, world)
    s0 = rank * per + min(rank, extra)
    s1 = s0 + per + (1 if rank < extra else 0)
    return min(4 * s0, n_slow), min(4 * s1, n_slow)


def blocks_per_slab(shape) -> int:
    """zfp blocks in one 4-deep slab of the slowest axis."""
    shape = tuple(shape)
    if len(shape) == 1:
        return 1
    n = 1
    for s in shape[1:]:
        n *= (s + 3) // 4
    return n


def uniform_shard_ok(shape, world: int, maxbits: int) -> bool:
    """True when every rank's stream segment is whole 64-bit words and the same
    size, so one all-gather of equal chunks rebuilds the global stream."""
    slabs = (shape[0] + 3) // 4
    if slabs % world:
        return False
    seg_bits = (slabs // world) * blocks_per_slab(shape) * maxbits
    return seg_bits % 64 == 0 and shape[0] % 4 == 0


def segment_words(shape, world: int, maxbits: int) -> int:
    """64-bit words in each rank's stream segment under uniform sharding."""
    slabs = (shape[0] + 3) // 4
    return (slabs // world) * blocks_per_slab(shape) * maxbits // 64


def local_shape(shape, world: int, rank: int) -> tuple:
    z0, z1 = slab_extent(shape[0], world, rank)
    return (z1 - z0,) + tuple(shape[1:])


def allgather_stream(local_words, group=None):
    """Concatenate every rank's stream segment (int64 words, equal sizes) in rank
    order on every rank: one ``all_gather_into_tensor`` (RCCL ncclAllGather on
    GPU tensors, gloo on CPU tensors)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty(world * local_words.numel(), dtype=local_words.dtype,
                      device=local_words.device)
    if local_words.is_cuda:
        dist.all_gather_into_tensor(out, local_words, group=group)
    else:  # gloo has no all_gather_into_tensor on every build: use the list form
        parts = list(out.chunk(world))
        dist.all_gather(parts, local_words, group=group)
    return out


def stream_offset_words(shape, world: int, rank: int, maxbits: int) -> int:
    """Word offset of `rank`'s segment in the global stream (uniform sharding)."""
    return rank * segment_words(shape, world, maxbits)


__all__ = ["slab_extent", "blocks_per_slab", "uniform_shard_ok", "segment_words",
           "local_shape", "allgather_stream", "stream_offset_words"]
