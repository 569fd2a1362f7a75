"""Benchmark: zfp fixed-rate encode+decode, device-resident, on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

With --gpus N > 1 and no launcher around it (WORLD_SIZE unset), bench.py
starts its N ranks itself through torch.distributed.run before touching the
GPU; a WORLD_SIZE that differs from --gpus is an error, so a run never
reports fewer ranks than it was asked for.  The line records what the ranks
saw (world_size_seen, backend, device_count, rank_devices).

A step is one pass of the hot path over one batch: encode the rank's array
into its fixed-rate stream, then decode the stream back, both on the GPU with
the data already in HBM.  Workload (BASELINE.json configs[1]): a 256^3 float32
array at 8 bits/value (maxbits 512) per GPU, filled with testzfp's polynomial
field (zfp-0.5.0/tests/testzfp.cpp:33-72).  With N GPUs every rank owns one
256^3 z-slab of a 256 x 256 x 256N array (weak scaling; blocks are independent,
so there is no collective on the data path).  The compressed-stream all-gather
over RCCL (the north star's exchange step) is timed separately, after the
timed region, and reported under "allgather".

Prints one JSON line on rank 0 (the driver contract), with
  value       = input GB/s of all ranks (10^9 B of input / s)
  roofline    = the dominant kernel's algorithmic bytes / its mean duration,
                over the MI355X HBM3E peak (8.0 TB/s, MI355X_MICROARCH.md)
  cpu_baseline= the reference's own CPU zfp 0.5.0 (oracle/_ref), timed here
                on this GPU's share of the host cores, for the headline array
                and for BASELINE configs[0] (1D f32 1M sine field, rate 8)
  config5     = BASELINE configs[4] at this N: one 1024^3 f32 array at rate 8
                strong-scaled over the N ranks as z-slabs of 1024/N planes,
                its step time (max over ranks), per-rank kernel times, the RCCL
                all-gather of the compressed stream and the gathered stream's
                SHA-256 against the reference's (tests/golden/golden.json)
  hbm_copy    = achievable bandwidth: cuzfp_hip_copy (16-byte non-temporal
                copy kernel) and torch's copy_, at 1 GiB and at the input size
  host_path   = the pinned host pipeline's rates and the bare pinned H2D/D2H
                link rates measured in the same run.
  configs     = BASELINE configs[2] (3D f64 256^3 rate 16) and configs[3] (2D
                f32 8192^2 rate 2) at N=1: graph-timed step GB/s, encode_ms /
                decode_ms, the dominant kernel's roofline and the stream and
                decoded-array SHA-256 against the reference's; timed right
                after the headline's timed region (never part of `value`).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GB/s input encoded+decoded (device-resident), 3D f32 fixed-rate; % HBM peak"
METRIC_OTHER = "GB/s input encoded+decoded (device-resident), {dims}D {dt} fixed-rate; % HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--size", type=int, default=256, help="per-GPU array edge (cube edge in 3D)")
    p.add_argument("--dims", type=int, default=3, choices=[1, 2, 3],
                   help="1D / 2D arrays of edge --size (BASELINE configs 2D 8192^2 r2, 1D 1M r8); "
                        "the headline workload is 3D")
    p.add_argument("--global-edge", type=int, default=0,
                   help="3D only: shard one E^3 global array over the ranks as z-slabs of E/N planes "
                        "(strong scaling; BASELINE configs[4] is E=1024 over 8 GPUs) instead of a "
                        "--size^3 slab per rank")
    p.add_argument("--rate", type=float, default=8.0)
    p.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    p.add_argument("--field", default="polynomial", choices=["polynomial", "splitmix"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-path", action="store_true")
    p.add_argument("--no-copy-probe", action="store_true", help="skip the device-to-device copy bandwidth probe")
    p.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    p.add_argument("--per-graph", type=int, default=0,
                   help="steps captured per hipGraph (default: the largest divisor of --steps up to 200)")
    p.add_argument("--kernel-ms", type=float, default=50.0,
                   help="GPU time each per-kernel measurement (encode_ms, decode_ms) runs for, back to back just "
                        "before the warmup steps")
    p.add_argument("--no-config5", action="store_true", help="skip BASELINE configs[4] (1024^3 sharded)")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the records of BASELINE configs[2] (3D f64 256^3 r16) and configs[3] (2D f32 8192^2 r2) "
                        "that the N=1 headline run times after its timed region")
    p.add_argument("--config5-edge", type=int, default=1024, help="edge of configs[4]'s global array")
    p.add_argument("--config5-steps", type=int, default=10)
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend for N > 1 (nccl = RCCL, the measured path; gloo runs the "
                        "collectives on host copies: tests of the multi-rank bookkeeping)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0 (tests of the N > 1 path on a one-GPU box; not a measurement)")
    p.add_argument("--dry-run-cpu", action="store_true",
                   help="test mode, no GPU: every rank runs the gloo backend and the CPU oracle stands in for "
                        "the codec, so the launcher and the rank bookkeeping can be checked on a CPU-only host; "
                        "the line it prints is not a measurement")
    p.add_argument("--dist-init", action="store_true",
                   help="N = 1: initialise the process group anyway (RCCL with --backend nccl, world size 1) and "
                        "run the stream all-gathers through it, so RCCL's library load, device binding and "
                        "all_gather_into_tensor run on a one-GPU box; the gathered stream is checked against "
                        "the local one")
    a = p.parse_args()
    if a.same_device and a.backend != "gloo":
        # two RCCL ranks on one device are refused or hang inside RCCL: say so at once
        p.error("--same-device needs --backend gloo (RCCL does not run two ranks on one GPU)")
    return a


def launch_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks of this script with
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and
    return their exit code.  Runs before anything touches the GPU, and starts
    the ranks as children (no exec), so `python bench.py --gpus 8` measures 8
    ranks or fails -- it can never report one."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, CUZFP_BENCH_LAUNCHED="1")
    return subprocess.call(cmd, env=env)


# Collectives of the bench's bookkeeping.  With RCCL they run on the device
# tensors; with gloo (--backend gloo, tests of the N > 1 path) on host copies,
# since gloo has no device collectives on this build.
HOST_COLL = False


def all_reduce_max(dist, t):
    if HOST_COLL:
        c = t.cpu()
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        t.copy_(c)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)


def all_gather_into(dist, out, t):
    if HOST_COLL:
        parts = list(torch_empty_like_cpu(out).chunk(dist.get_world_size()))
        dist.all_gather(parts, t.cpu())
        out.copy_(torch_cat(parts))
    else:
        dist.all_gather_into_tensor(out, t)


def torch_empty_like_cpu(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype, device="cpu")


def torch_cat(parts):
    import torch
    return torch.cat(parts)


def rank_info(dist, world: int, dev, backend: str) -> dict:
    """What the ranks saw: the process group's size and backend, the devices
    this process can see, and every rank's device id (gathered)."""
    import torch
    seen = dist.get_world_size() if dist.is_initialized() else 1
    did = dev.index if dev.type == "cuda" else -1
    if dist.is_initialized() and seen > 1:
        t = torch.tensor([did], dtype=torch.int64, device=dev)
        out = torch.empty(seen, dtype=torch.int64, device=dev)
        all_gather_into(dist, out, t)
        devs = [int(v) for v in out.cpu()]
    else:
        devs = [did]
    return {"world_size_seen": seen, "backend": backend, "device_count": torch.cuda.device_count(),
            "rank_devices": devs}


def dry_run(args):
    """The launcher and rank bookkeeping of main() on CPUs (gloo), with the
    CPU oracle standing in for the codec on a small array: tests/test_bench_launch.py
    checks that `bench.py --gpus 2 --dry-run-cpu` reports two ranks."""
    import torch
    import torch.distributed as dist
    import oracle
    from cuzfp_amd.datagen import polynomial_slab
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if oracle.restatement is None:
        oracle.build(with_reference=False)
        oracle.reload()
    n = 16
    a = polynomial_slab((n * world, n, n), rank * n, (rank + 1) * n, np.float32)
    mb = int(oracle.restatement.rate_to_maxbits(args.rate, np.float32, 3))
    dev = torch.device("cpu")

    def step():
        w = oracle.restatement.compress(a, mb)
        return oracle.restatement.decompress(w, a.shape, np.float32, mb)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    info = rank_info(dist, world, dev, "gloo" if world > 1 else "none")
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(a.nbytes * world * args.steps / float(t) / 1e9, 6),
                          "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "data": "dry run: CPU oracle on a 16^3 slab per rank, not a measurement",
                          **info}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_share() -> tuple[int, int]:
    """(threads used, CPUs in this process's affinity).  On the GPU box one
    GPU's share of the host is OMP_NUM_THREADS (16): the harness sizes every
    CPU pool to it, and so does the baseline."""
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return max(1, min(aff, share)), aff


def cpu_baseline(a: np.ndarray, maxbits: int):
    """Reference CPU zfp 0.5.0 (zfp_compress + zfp_decompress, oracle/_ref) on
    this process's host cores: the whole headline array, slab-parallel over
    this GPU's share of the cores, median of 30 round trips (10-15 core-s);
    one core on a quarter of it; and BASELINE configs[0], the reference's own
    CPU test (src/tests/t_encode_decode_1.cpp:15-30: 1M float32 sine values,
    rate 8), median of 30 single-core round trips."""
    try:
        import oracle
        from cuzfp_amd.datagen import sine_field
    except Exception:  # pragma: no cover
        return None
    ref = oracle.reference
    kind = "reference"
    if ref is None:
        return None
    sample = np.ascontiguousarray(a)
    quarter = np.ascontiguousarray(a[: max(4, (a.shape[0] // 16) * 4)])
    cores, aff = cpu_share()
    reps = 30
    t0 = time.perf_counter()
    rt, enc, dec, _ = ref.time_roundtrip(sample, maxbits, threads=cores, reps=reps)
    rt1, enc1, dec1, _ = ref.time_roundtrip(quarter, maxbits, threads=1, reps=3)
    s1 = sine_field(1 << 20, np.float32)
    mb1 = int(oracle.restatement.rate_to_maxbits(8, np.float32, 1)) if oracle.restatement else 32
    rtc0, encc0, decc0, _ = ref.time_roundtrip(s1, mb1, threads=1, reps=reps)
    wall = time.perf_counter() - t0
    nbytes = sample.nbytes
    model = None
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:  # pragma: no cover
        pass
    return {"value": round(nbytes / rt / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": kind,
            "cpu_model": model, "host_cpus_visible": os.cpu_count(), "cpu_affinity": aff,
            "cores_note": "threads = this GPU's share of the host (OMP_NUM_THREADS on the GPU box, which "
                          "sizes every CPU pool to it); the whole machine's CPUs serve 8 GPUs",
            "sample": f"the whole {'x'.join(map(str, sample.shape))} {sample.dtype} workload array, maxbits "
                      f"{maxbits}, median of {reps} round trips, slab threads (slowest axis)",
            "encode_GBps": round(nbytes / enc / 1e9, 4), "decode_GBps": round(nbytes / dec / 1e9, 4),
            "single_core_GBps": round(quarter.nbytes / rt1 / 1e9, 4),
            "config0": {"workload": "1d_float32_1M_rate8 (t_encode_decode_1.cpp sine field)", "cores": 1,
                        "roundtrip_GBps": round(s1.nbytes / rtc0 / 1e9, 4),
                        "encode_GBps": round(s1.nbytes / encc0 / 1e9, 4),
                        "decode_GBps": round(s1.nbytes / decc0 / 1e9, 4),
                        "roundtrip_ms": round(rtc0 * 1e3, 3), "maxbits": mb1,
                        "sample": f"median of {reps} single-core round trips"},
            # the whole host (north star: "the box's own host cores"), not run: the GPU
            # box caps a job's CPU pools at its GPU's share (OMP_NUM_THREADS), so the
            # whole-host figure is this share's measured rate scaled by CPUs / threads
            # (z-slabs are independent; the share's own parallel efficiency is given)
            "whole_host": {"cpus": aff, "measured": False,
                           "projected_GBps": round(nbytes / rt / 1e9 * aff / cores, 3),
                           "share_parallel_efficiency": round((nbytes / rt) / (cores * quarter.nbytes / rt1), 3),
                           "note": f"linear projection of the {cores}-thread measurement to all {aff} CPUs of the "
                                   "host; not timed (the box's rules keep a job's CPU pool to its GPU's share)"},
            "wall_s": round(wall, 2)}


def allgather_words(zd, words):
    """The stream all-gather: RCCL on the device words, or gloo on a host copy."""
    if HOST_COLL:
        return zd.allgather_stream(words.cpu()).to(words.device)
    return zd.allgather_stream(words)


def run_config5(E: int, steps: int, world: int, rank: int, dev, graphed, dist, use_dist: bool = False):
    """BASELINE configs[4] at this N, GPU phase: one E^3 f32 polynomial
    array at rate 8 strong-scaled over the N ranks as z-slabs of E/N planes.  Each
    rank encodes and decodes its slab (no communication); the step time is the
    max over ranks of K steps between barriers.  Then, outside that timed region,
    the RCCL all-gather that assembles the global stream on every rank, timed with
    HIP events on the launch stream.  Returns the record and what finish_config5
    needs for the parity check (host-side hashing, done after the headline's timed
    region so that the GPU does not idle for seconds just before it)."""
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd import dist as zd
    stream = torch.cuda.current_stream()
    maxbits = cz.rate_to_maxbits(8, np.float32, 3)
    sh = zd.StrongShard(E, world, rank, maxbits)
    from cuzfp_amd.datagen import polynomial_slab_device
    x = polynomial_slab_device(sh.global_shape, sh.z0, sh.z1, dev)
    words = torch.empty(sh.words, dtype=torch.int64, device=dev)
    y = torch.empty_like(x)

    def step():
        cz.encode(x, maxbits, out=words)
        cz.decode(words, sh.shape, x.dtype, maxbits, out=y)

    step()
    err = (y - x).abs().max()  # stays on the device until finish_config5

    def allmax(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        if world > 1:
            all_reduce_max(dist, t)
        return float(t.item())

    def allgather_floats(v: float) -> list:
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        if world == 1:
            return [v]
        out = torch.empty(world, dtype=torch.float64, device=dev)
        all_gather_into(dist, out, t)
        return [float(u) for u in out.cpu()]

    per_graph = next(c for c in (5, 2, 1) if steps % c == 0)
    run = graphed(step, per_graph)
    run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // per_graph):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    step_s = allmax((time.perf_counter() - t0) / steps)

    def time_kernel(fn, reps=10):
        r = graphed(fn, reps)
        r()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    enc_s = allgather_floats(time_kernel(lambda: cz.encode(x, maxbits, out=words)))
    dec_s = allgather_floats(time_kernel(lambda: cz.decode(words, sh.shape, x.dtype, maxbits, out=y)))
    cz.encode(x, maxbits, out=words)
    torch.cuda.synchronize()

    ag_s, full = None, None
    if use_dist:  # (world 1 with --dist-init: RCCL's one-rank all-gather, a copy)
        full = allgather_words(zd, words)
        torch.cuda.synchronize()
        dist.barrier()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            full = allgather_words(zd, words)
        e1.record(stream)
        torch.cuda.synchronize()
        dist.barrier()
        ag_s = allmax(e0.elapsed_time(e1) / 5 * 1e-3)
        if world == 1:
            full = None  # the local stream is the gathered one (checked in main's all-gather)
        if rank != 0:
            full = None
    out = zd.sharded_summary(sh, 4, step_s, enc_s, dec_s, HBM_PEAK_GBS, ag_s,
                             "gloo (host-copy collectives)" if HOST_COLL else "nccl (RCCL)")
    out["steps"] = steps
    del x, y
    return {"record": out, "E": E, "words": words, "full": full, "err": err}


def finish_config5(st: dict, world: int, rank: int, dev, dist) -> dict:
    """configs[4]'s parity, on the host: every rank's segment against the
    reference's SHA-256 of its word range, the gathered stream (rank 0) against
    the reference's whole-stream hash, the round-trip error against the
    reference's (tests/golden/golden.json)."""
    import torch
    out, E = st["record"], st["E"]

    def allmax(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        if world > 1:
            all_reduce_max(dist, t)
        return float(t.item())

    gold = None
    gpath = os.path.join(ROOT, "tests", "golden", "golden.json")
    if os.path.exists(gpath):
        gold = json.load(open(gpath))["cases"].get(f"baseline/3d_f32_{E}_r8/polynomial")
    local = st["words"].cpu().numpy()
    slab_ok = None
    if gold and world > 1 and f"slab_sha256_n{world}" in gold:
        slab_ok = hashlib.sha256(local.tobytes()).hexdigest() == gold[f"slab_sha256_n{world}"][rank]
        slab_ok = allmax(0.0 if slab_ok else 1.0) == 0.0
    full_host = (st["full"].cpu().numpy() if st["full"] is not None else None) if world > 1 else local
    out["max_abs_err"] = allmax(float(st["err"].item()))
    if rank == 0:
        got = hashlib.sha256(full_host.tobytes()).hexdigest()
        out["parity"] = {"reference_sha256": gold["stream_sha256"] if gold else None,
                         "gathered_stream_sha256": got,
                         "stream_matches_reference": (got == gold["stream_sha256"]) if gold else None,
                         "slabs_match_reference_word_ranges": slab_ok,
                         "max_abs_err_matches_reference": (out["max_abs_err"] == gold["max_abs_err"]) if gold else None}
    st.clear()
    torch.cuda.empty_cache()
    return out


OTHER_CONFIGS = (  # BASELINE configs[2], configs[3]: (workload, golden key, dims, edge, dtype, rate)
    ("3d_float64_256^3_rate16", "baseline/3d_f64_256_r16/polynomial", 3, 256, "float64", 16.0),
    ("2d_float32_8192^2_rate2", "baseline/2d_f32_8192_r2/polynomial", 2, 8192, "float32", 2.0),
)


def run_other_configs(dev, graphed, stream, steps: int = 20):
    """BASELINE configs[2] (3D f64 256^3 rate 16) and configs[3] (2D f32 8192^2
    rate 2), N=1, GPU phase, right after the headline's timed region: each one's
    encode+decode step timed over `steps` steps replayed from one hipGraph (HIP
    events on the launch stream, after ~50 ms of replays), each kernel's mean
    duration (hipGraphs of 20 launches), the dominant kernel's roofline.  Parity
    (stream and decoded SHA-256 against the reference's, tests/golden/golden.json)
    is finished on the host by finish_other_configs, after the GPU work."""
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    out = []
    for workload, key, dims, edge, dt, rate in OTHER_CONFIGS:
        try:
            dtype = np.dtype(dt)
            shape = (edge,) * dims
            a = polynomial_field(shape, dtype)
            x = torch.from_numpy(a).to(dev)
            del a
            mb = cz.rate_to_maxbits(rate, dtype, dims)
            nbs = cz.stream_bytes(shape, dtype, mb)
            w = torch.empty(nbs // 8, dtype=torch.int64, device=dev)
            y = torch.empty_like(x)

            def step():
                cz.encode(x, mb, out=w)
                cz.decode(w, shape, x.dtype, mb, out=y)

            run = graphed(step, steps)
            eg = graphed(lambda: cz.encode(x, mb, out=w), 20)
            dg = graphed(lambda: cz.decode(w, shape, x.dtype, mb, out=y), 20)
            run()
            torch.cuda.synchronize()

            def timed(fn, count, reps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(reps):
                    fn()
                e1.record(stream)
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / (reps * count)

            t_w = time.perf_counter()
            while time.perf_counter() - t_w < 0.05:  # the clocks under load first
                run()
                torch.cuda.synchronize()
            step_ms = timed(run, steps, 3)
            enc_ms = timed(eg, 20, 3)
            dec_ms = timed(dg, 20, 3)
            run()  # leave the last step's stream and array in w, y
            nin = x.numel() * x.element_size()
            dom = "encode" if enc_ms >= dec_ms else "decode"
            dom_ms = max(enc_ms, dec_ms)
            ach = (nin + nbs) / (dom_ms * 1e-3) / 1e9
            rec = {"workload": workload, "baseline_config": "configs[2]" if dims == 3 else "configs[3]",
                   "shape": list(shape), "maxbits": mb, "dtype": "f64" if dt == "float64" else "f32",
                   "GBps_input": round(nin / (step_ms * 1e-3) / 1e9, 1), "ms_per_step": round(step_ms, 4),
                   "pct_hbm_peak": round(100.0 * 2 * (nin + nbs) / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 2),
                   "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                   "roofline": {"bound": "hbm", "kernel": f"zfp_{dom}", "achieved": round(ach, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                "algorithmic_bytes_per_launch": nin + nbs},
                   "timing": f"{steps} steps replayed from one hipGraph x 3 (HIP events, after ~50 ms of "
                             "replays); kernels: hipGraphs of 20 launches x 3"}
            out.append({"record": rec, "key": key, "w": w, "y": y, "x": x})
        except Exception as e:  # a side record never fails the bench
            out.append({"record": {"workload": workload, "error": repr(e)[:300]}})
    return out


def finish_other_configs(st: list) -> list:
    """Host-side parity of run_other_configs' last steps: the stream's and the
    decoded array's SHA-256 against the reference zfp 0.5.0's, and the max
    round-trip error against the reference's."""
    import torch
    gpath = os.path.join(ROOT, "tests", "golden", "golden.json")
    gold = json.load(open(gpath))["cases"] if os.path.exists(gpath) else {}
    recs = []
    for s in st:
        rec = s["record"]
        if "w" in s:
            g = gold.get(s["key"])
            got = hashlib.sha256(s["w"].cpu().numpy().tobytes()).hexdigest()
            dec = hashlib.sha256(s["y"].cpu().numpy().tobytes()).hexdigest()
            err = float((s["y"].double() - s["x"].double()).abs().max().item())
            rec["parity"] = {"stream_matches_reference": (got == g["stream_sha256"]) if g else None,
                             "decoded_matches_reference": (dec == g["decoded_sha256"]) if g else None,
                             "max_abs_err": err,
                             "max_abs_err_matches_reference": (err == g["max_abs_err"]) if g else None,
                             "golden_case": s["key"]}
            rec["parity_ok"] = bool(g) and got == g["stream_sha256"] and dec == g["decoded_sha256"]
        # roofline.traffic: the dominant kernel's HBM bytes a launch from the
        # builder's PMC session for this workload (profiles/traffic_configs.json)
        tpath = os.path.join(ROOT, "profiles", "traffic_configs.json")
        roof = rec.get("roofline")
        if roof is not None and os.path.exists(tpath):
            try:
                tj = json.load(open(tpath)).get(rec.get("workload"))
            except (OSError, ValueError):
                tj = None
            kind = "decode" if roof.get("kernel") == "zfp_decode" else "encode"
            if tj and tj.get(kind + "_hbm_bytes_per_launch"):
                roof["traffic"] = tj[kind + "_hbm_bytes_per_launch"]
                roof["traffic_source"] = {"file": "profiles/traffic_configs.json", "session": tj.get("source"),
                                          "method": tj.get("method"),
                                          "note": "PMC counters of an earlier profiled session of this workload, "
                                                  "not of this run"}
        recs.append(rec)
        s.clear()
    torch.cuda.empty_cache()
    return recs


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import cuzfp_amd as cz
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_slab, splitmix_uniform

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # a measurement of fewer ranks than asked for is never printed
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch N ranks (python bench.py --gpus N "
                         f"starts them itself) or pass --gpus {world}")
    global HOST_COLL
    gpu = 0 if args.same_device else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    backend = "nccl (RCCL)" if args.backend == "nccl" else "gloo (host-copy collectives)"
    use_dist = world > 1 or args.dist_init
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            import socket
            with socket.socket() as s_:
                s_.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s_.getsockname()[1])
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            HOST_COLL = True

    dtype = np.dtype(args.dtype)
    n = args.size
    dims = args.dims
    shape = (n,) * dims                                # this rank's slab
    gshape = (n * world,) + (n,) * (dims - 1)          # the global array
    strong = args.global_edge > 0
    if strong:
        E = args.global_edge
        if dims != 3 or E % (4 * world):
            raise SystemExit(f"--global-edge needs 3D and an edge divisible by 4*N (got {E}, N={world})")
        n = E
        shape = (E // world, E, E)
        gshape = (E, E, E)
    maxbits = cz.rate_to_maxbits(args.rate, dtype, dims)
    # each rank's slab: planes [rank*n, (rank+1)*n) of the global field
    if args.field == "polynomial":
        if dims == 3:
            a = polynomial_slab(gshape, rank * shape[0], (rank + 1) * shape[0], dtype)
        else:
            from cuzfp_amd.datagen import polynomial_field
            a = polynomial_field(shape, dtype)
    else:
        a = splitmix_uniform(shape, dtype, seed=42 + rank)
    x = torch.from_numpy(a).to(dev)
    nbytes_stream = cz.stream_bytes(shape, dtype, maxbits)
    words = torch.empty(nbytes_stream // 8, dtype=torch.int64, device=dev)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream()

    def step():  # launches on torch's current stream (the capture stream under a graph)
        cz.encode(x, maxbits, out=words)
        cz.decode(words, shape, x.dtype, maxbits, out=y)

    def graphed(fn, count):
        """`count` calls of fn captured into one hipGraph (launch overhead off the
        host's critical path); falls back to eager calls if capture fails."""
        if args.no_graph:
            return lambda: [fn() for _ in range(count)]
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(count):
                    fn()
            return g.replay
        except Exception as e:  # pragma: no cover
            print(f"graph capture failed ({e}); timing eager launches", file=sys.stderr)
            return lambda: [fn() for _ in range(count)]

    # correctness of the benchmarked configuration: round-trip error within
    # testzfp's bound for this field, and (N=1, polynomial) the stream hash of
    # the reference's own zfp 0.5.0 output (tests/golden/golden.json)
    step()
    torch.cuda.synchronize()
    max_err = float((y.double() - x.double()).abs().max().item())
    # Order of the GPU work.  The other GPU measurements of the line (BASELINE
    # configs[4], the copy calibrator, the RCCL all-gather, per-kernel times) run
    # before the timed region, with every graph captured up front and every
    # host-side check (stream hashes, the CPU baseline) after it, so that the
    # timed steps start on a GPU that has been busy up to that point: after the
    # GPU idles (a host-side hash of the 1 GiB configs[4] stream takes seconds)
    # its clocks ramp again over the first ~10 ms of work, and a 20-step run
    # measured 8-11 % below the same steps on a busy GPU (1,150-1,203 vs
    # 1,294 GB/s on one box).  The timed region itself is unchanged: W warmup
    # steps, then exactly K steps.
    per_graph = args.per_graph or next(c for c in range(min(200, args.steps), 0, -1) if args.steps % c == 0)
    if args.steps % per_graph:
        raise SystemExit(f"--per-graph {per_graph} does not divide --steps {args.steps}")
    run = graphed(step, per_graph)
    run()  # the graph's first replay uploads it: never inside the timed region
    enc_graph = graphed(lambda: cz.encode(x, maxbits, out=words), 50)
    dec_graph = graphed(lambda: cz.decode(words, shape, x.dtype, maxbits, out=y), 50)
    enc_graph()
    dec_graph()

    c5 = None
    if not args.no_config5 and dims == 3 and args.dtype == "float32" and not strong:
        try:
            c5 = run_config5(args.config5_edge, args.config5_steps, world, rank, dev, graphed, dist, use_dist)
        except torch.cuda.OutOfMemoryError as e:  # pragma: no cover
            c5 = {"error": f"out of memory: {e}"}

    # per-kernel durations with HIP events on the launch stream: replays of a
    # hipGraph of 50 launches, back to back for at least `min_ms` of GPU time
    # (sized from one replay), so each mean is over thousands of launches on a
    # GPU under sustained load -- the state the timed steps then start in
    def time_kernel(r, min_ms, then=None):
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r()
        e1.record(stream)
        torch.cuda.synchronize()
        n = max(2, int(min_ms / max(e0.elapsed_time(e1), 1e-3)) + 1)
        e0.record(stream)
        for _ in range(n):
            r()
        e1.record(stream)
        if then is not None:
            then()  # queued behind the measured launches, before the synchronize
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / (n * 50), n * 50


    # achievable HBM bandwidth on this box: the library's 16-byte
    # non-temporal copy kernel (cuzfp_hip_copy, the codec's access width and
    # cache policy) and torch's copy_, read + write bytes over time
    def copy_GBps(nbytes, fn_name):
        src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        dst = torch.empty_like(src)
        fn = (lambda: cz.copy(src, dst)) if fn_name == "cuzfp" else (lambda: dst.copy_(src))
        r = graphed(fn, 10)
        r()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(3):
            r()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 30
        del src, dst
        return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)

    hbm_copy = None
    if rank == 0 and not args.no_copy_probe:
        hbm_copy = {"kernel": "cuzfp_hip_copy (16-B non-temporal loads/stores, one per lane, one grid)",
                    "GBps_1GiB": copy_GBps(1 << 30, "cuzfp"), "GBps_at_input_size": copy_GBps(a.nbytes, "cuzfp"),
                    "torch_copy_GBps_1GiB": copy_GBps(1 << 30, "torch"), "input_bytes": a.nbytes,
                    "note": "read + write bytes / time, hipGraph of 10 copies; at the input size source and "
                            "destination sit in the 256 MiB Infinity Cache between copies"}

    # optional RCCL all-gather of the compressed stream (the exchange step)
    allgather = None
    if use_dist and zd.uniform_shard_ok(gshape, world, maxbits):
        full = allgather_words(zd, words)
        torch.cuda.synchronize()
        dist.barrier()
        ag0 = time.perf_counter()
        agr = 5
        for _ in range(agr):
            full = allgather_words(zd, words)
        torch.cuda.synchronize()
        ag_s = (time.perf_counter() - ag0) / agr
        t = torch.tensor([ag_s], dtype=torch.float64, device=dev)
        all_reduce_max(dist, t)
        ag_s = float(t.item())
        allgather = {"bytes_per_rank_in": int(full.numel() * 8 - nbytes_stream), "ms": round(ag_s * 1e3, 3),
                     "GBps_per_rank_in": round((full.numel() * 8 - nbytes_stream) / ag_s / 1e9, 2),
                     "backend": backend, "world_size": world}
        # this rank's segment of the gathered stream is its own stream, word for word
        seg = full[rank * words.numel():(rank + 1) * words.numel()]
        allgather["own_segment_matches"] = bool(torch.equal(seg, words))
        del full, seg

    # (last before the warmup steps: the ~100 ms of back-to-back kernels bring
    # the GPU to the clocks it holds under load, see "Order of the GPU work")
    # The W warmup steps are queued right behind the decode timing's last launch
    # (as replays of the timed graph and of a graph of the W % per_graph rest),
    # so the GPU does not idle between the two.
    warm_rest = graphed(step, args.warmup % per_graph) if args.warmup % per_graph else None
    if warm_rest is not None:
        warm_rest()  # upload

    def warmup():
        for _ in range(args.warmup // per_graph):
            run()
        if warm_rest is not None:
            warm_rest()

    t_pre = time.perf_counter()
    enc_ms, enc_n = time_kernel(enc_graph, args.kernel_ms)
    dec_ms, dec_n = time_kernel(dec_graph, args.kernel_ms, then=warmup)
    pre_timed = {"what": "per-kernel timing (encode_ms, decode_ms): back-to-back hipGraph replays, then the W "
                         "warmup steps", "encode_launches": enc_n, "decode_launches": dec_n,
                 "wall_ms": round((time.perf_counter() - t_pre) * 1e3, 1)}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps // per_graph):
        run()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    t_local = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        all_reduce_max(dist, t_local)
    elapsed = float(t_local.item())
    gpu_ms_per_step = ev0.elapsed_time(ev1) / args.steps

    # BASELINE configs[2] and configs[3] (N=1, headline run only), on the GPU
    # right after the timed region; their hashes with the other host checks
    others = None
    if (world == 1 and not strong and not args.no_configs and dims == 3 and args.dtype == "float32"
            and n == 256 and args.rate == 8.0 and args.field == "polynomial"):
        others = run_other_configs(dev, graphed, stream)

    # host-side checks, after the timed region: the stream's SHA-256 against the
    # reference's (N=1; the timed steps rewrote the same words), configs[4]'s parity
    parity = None
    gpath = os.path.join(ROOT, "tests", "golden", "golden.json")
    key = {(3, 256, "float32", 8.0): "baseline/3d_f32_256_r8", (3, 256, "float64", 16.0): "baseline/3d_f64_256_r16",
           (2, 8192, "float32", 2.0): "baseline/2d_f32_8192_r2",
           (1, 1048576, "float32", 8.0): "baseline/1d_f32_1M_r8"}.get((dims, n, args.dtype, float(args.rate)))
    if key and world == 1 and not strong and os.path.exists(gpath):
        rec = json.load(open(gpath))["cases"].get(f"{key}/{args.field}")
        if rec:
            got = hashlib.sha256(words.cpu().numpy().tobytes()).hexdigest()
            dec = hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()
            if got != rec["stream_sha256"]:
                parity = "MISMATCH (stream)"
            elif dec != rec.get("decoded_sha256", dec):
                parity = "MISMATCH (decoded array)"
            else:
                parity = "stream and decoded sha256 == reference zfp 0.5.0"
    config5 = None
    if c5 is not None:
        config5 = c5 if "error" in c5 else finish_config5(c5, world, rank, dev, dist)
    configs = finish_other_configs(others) if others is not None else None

    n_in = a.nbytes
    value = n_in * world * args.steps / elapsed / 1e9
    s_bytes = nbytes_stream
    enc_bytes = n_in + s_bytes     # read array, write stream
    dec_bytes = s_bytes + n_in     # read stream, write array
    dominant = "encode" if enc_ms >= dec_ms else "decode"
    dom_ms = max(enc_ms, dec_ms)
    dom_bytes = enc_bytes if dominant == "encode" else dec_bytes
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    workload = f"{dims}d_{args.dtype}_{n}^{dims}_rate{args.rate:g}" + (f"_zslab{world}" if strong and world > 1 else "")
    # roofline.traffic: HBM bytes a launch from rocprofv3 PMC counters, which a
    # run cannot collect on itself (a --pmc pass is its own profiled run): read
    # from the builder's PMC session record for this workload, and say which
    traffic, traffic_source = None, None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            wk = workload
            if tj.get("workload") == wk:
                traffic = tj.get(dominant + "_hbm_bytes_per_launch")
                traffic_source = {"file": os.path.relpath(args.traffic_json, ROOT), "session": tj.get("source"),
                                  "method": tj.get("method"),
                                  "note": "PMC counters of an earlier profiled session of this workload, "
                                          "not of this run"}
        except Exception:
            traffic = None

    ranks = rank_info(dist, world, dev, backend if use_dist else "none")
    result = None
    if rank == 0:
        host_path = None
        if world == 1 and not args.no_host_path and not strong:
            hp_in = torch.from_numpy(a).pin_memory().numpy()
            hp_out = torch.empty(s_bytes // 8, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
            hp_back = torch.empty(a.shape, dtype=x.dtype).pin_memory().numpy()
            cz.compress_host(hp_in, maxbits, out=hp_out)
            cz.decompress_host(hp_out, shape, dtype, maxbits, out=hp_back)
            def med7(fn):  # median of 7 synchronous calls
                ts = []
                for _ in range(7):
                    t0 = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - t0)
                return sorted(ts)[3]
            tc = med7(lambda: cz.compress_host(hp_in, maxbits, out=hp_out))
            td = med7(lambda: cz.decompress_host(hp_out, shape, dtype, maxbits, out=hp_back))
            # the bare pinned link in the same run: one copy of the array each
            # way (the larger of each call's two transfers), mean of 5 each
            h_in = torch.from_numpy(hp_in)
            h_back = torch.from_numpy(hp_back)
            d_tmp = torch.empty(a.shape, dtype=x.dtype, device=dev)
            torch.cuda.synchronize()
            t_h2d = time.perf_counter()
            for _ in range(5):
                d_tmp.copy_(h_in, non_blocking=True)
            torch.cuda.synchronize()
            t_h2d = (time.perf_counter() - t_h2d) / 5
            t_d2h = time.perf_counter()
            for _ in range(5):
                h_back.copy_(d_tmp, non_blocking=True)
            torch.cuda.synchronize()
            t_d2h = (time.perf_counter() - t_d2h) / 5
            del d_tmp
            h2d = n_in / t_h2d / 1e9
            d2h = n_in / t_d2h / 1e9
            # link-bound time of a call: its two transfers overlap (separate copy
            # queues), so the bound is the larger one alone at its direction's
            # one-way rate -- compression the array's H2D, decompression the
            # array's D2H; the rate over it is the pipeline's link efficiency
            c_link = n_in / max(n_in / (h2d * 1e9), s_bytes / (d2h * 1e9)) / 1e9
            d_link = n_in / max(n_in / (d2h * 1e9), s_bytes / (h2d * 1e9)) / 1e9
            host_path = {"compress_GBps": round(n_in / tc / 1e9, 2), "decompress_GBps": round(n_in / td / 1e9, 2),
                         "roundtrip_GBps": round(n_in / (tc + td) / 1e9, 2),
                         "link_GBps": {"h2d": round(h2d, 2), "d2h": round(d2h, 2)},
                         "frac_of_link": {"compress": round(n_in / tc / 1e9 / c_link, 3),
                                          "decompress": round(n_in / td / 1e9 / d_link, 3)},
                         "chunk_bytes": int(os.environ.get("CUZFP_HOST_CHUNK_BYTES", 64 << 20)), "nstreams": 4,
                         "schedule": "per-stream" if os.environ.get("CUZFP_HOST_ORDERED", "1") == "0" else "ordered",
                         "zero_copy": int(os.environ.get("CUZFP_HOST_ZEROCOPY", "1") or 0),
                         "note": "pinned host buffers, PCIe-inclusive (cuzfp_hip_compress_host/decompress_host), median of 7 calls; "
                                 "frac_of_link = rate over the larger transfer's one-way link rate: compress "
                                 "array bytes / max(array/h2d, stream/d2h), decompress array bytes / "
                                 "max(array/d2h, stream/h2d); H2D beside D2H run at ~48 GB/s each "
                                 "(profiles/r05_copy_chunks.txt), so ~0.95 is the practical ceiling"}
        cpu = None if (args.no_cpu_baseline or world > 1 or strong) else cpu_baseline(a, maxbits)
        result = {
            "metric": METRIC if (dims == 3 and args.dtype == "float32") else
                      METRIC_OTHER.format(dims=dims, dt="f32" if args.dtype == "float32" else "f64"),
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.dtype == "float32" else "f64",
            "data": f"synthetic ({'testzfp polynomial field' if args.field == 'polynomial' else 'splitmix64 uniform [-1,1)'})",
            "config": {"workload": workload, "shape_per_gpu": list(shape),
                       "global_shape": list(gshape), "maxbits": maxbits, "rate": args.rate,
                       "parallelism": f"z-slab x{world}", "stream_bytes_per_gpu": s_bytes},
            "pct_hbm_peak": round(100.0 * value / world * (enc_bytes + dec_bytes) / n_in / HBM_PEAK_GBS, 2),
            "gpu_ms_per_step": round(gpu_ms_per_step, 4),
            "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_GBps_input": round(n_in / (enc_ms * 1e-3) / 1e9, 1),
            "decode_GBps_input": round(n_in / (dec_ms * 1e-3) / 1e9, 1),
            "roofline": {"bound": "hbm", "kernel": f"zfp_{dominant}", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_source,
                         "algorithmic_bytes_per_launch": dom_bytes,
                         "frac_of_copy": round(achieved / hbm_copy["GBps_1GiB"], 4) if hbm_copy else None},
            "hbm_copy": hbm_copy,
            "cpu_baseline": cpu,
            "host_path": host_path,
            "allgather": allgather,
            "config5": config5,
            "configs": configs,
            "max_abs_err": max_err,
            "parity": parity,
            "pre_timed_gpu_work": pre_timed,
            **ranks,
        }
        print(json.dumps(result), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    _args = parse()
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(_args))
    if _args.dry_run_cpu:
        dry_run(_args)
    else:
        main()
