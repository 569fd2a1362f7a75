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


class StrongShard:
    """Rank `rank`'s share of one E^3 array sharded over `world` ranks as z-slabs
    of E/world planes (BASELINE configs[4]: E = 1024, world = 8): its slab of
    the global array, the local shape and its word range in the global stream."""

    def __init__(self, edge: int, world: int, rank: int, maxbits: int):
        if edge % (4 * world):
            raise ValueError(f"edge {edge} is not a multiple of 4 * world ({world})")
        self.edge, self.world, self.rank, self.maxbits = edge, world, rank, maxbits
        self.global_shape = (edge, edge, edge)
        self.z0 = rank * edge // world
        self.z1 = (rank + 1) * edge // world
        self.shape = (self.z1 - self.z0, edge, edge)
        if not uniform_shard_ok(self.global_shape, world, maxbits):
            raise ValueError("segments are not whole 64-bit words")
        self.words = segment_words(self.global_shape, world, maxbits)
        self.word0 = stream_offset_words(self.global_shape, world, rank, maxbits)
        self.values = self.shape[0] * edge * edge


def sharded_summary(shard: "StrongShard", itemsize: int, step_s: float, enc_s: list, dec_s: list,
                    hbm_peak_GBps: float, allgather_s: float | None = None,
                    backend: str = "nccl (RCCL)") -> dict:
    """The bench line's record of one strong-scaled sharded run: `step_s` is the
    max over ranks of one encode+decode step, enc_s / dec_s the per-rank kernel
    times (seconds), allgather_s the max-over-ranks all-gather time."""
    g_in = shard.edge ** 3 * itemsize                 # global input bytes
    stream = shard.words * 8 * shard.world            # global stream bytes
    algo = 2 * (g_in + stream)                        # read + write, both kernels, all ranks
    out = {"workload": f"3d_float32_{shard.edge}^3_rate{shard.maxbits / 64:g}_zslab{shard.world}",
           "n_ranks": shard.world, "slab_shape": list(shard.shape), "global_shape": list(shard.global_shape),
           "maxbits": shard.maxbits, "step_ms": round(step_s * 1e3, 4),
           "value_GBps": round(g_in / step_s / 1e9, 2),
           "frac_of_aggregate_hbm": round(algo / step_s / 1e9 / (hbm_peak_GBps * shard.world), 4),
           "encode_ms_per_rank": [round(t * 1e3, 4) for t in enc_s],
           "decode_ms_per_rank": [round(t * 1e3, 4) for t in dec_s],
           "stream_bytes": stream}
    if allgather_s is not None:
        recv = stream - shard.words * 8               # bytes each rank receives
        out["allgather"] = {"ms": round(allgather_s * 1e3, 4), "bytes_in_per_rank": recv,
                            "GBps_in_per_rank": round(recv / allgather_s / 1e9, 2) if allgather_s > 0 else None,
                            "backend": backend}
    return out


__all__ = ["StrongShard", "sharded_summary", "slab_extent", "blocks_per_slab", "uniform_shard_ok", "segment_words",
           "local_shape", "allgather_stream", "stream_offset_words"]
