"""bench.py's multi-rank launcher on CPU: `python bench.py --gpus 2` with no
torchrun around it starts its two ranks itself (torch.distributed.run, gloo in
the dry-run mode, the CPU oracle standing in for the codec) and the line it
prints reports both ranks -- the scaling run cannot under-report its ranks."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True,
                          text=True, timeout=300, env=env, cwd=ROOT)


def test_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--dry-run-cpu", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["world_size_seen"] == 2
    assert d["backend"] == "gloo"
    assert len(d["rank_devices"]) == 2
    assert d["value"] > 0


def test_world_size_mismatch_is_an_error():
    # a launcher that started fewer ranks than --gpus asks for: refused, no line
    r = _run(["--gpus", "2", "--dry-run-cpu", "--steps", "1", "--warmup", "0"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "WORLD_SIZE" in r.stderr


def test_single_rank_dry_run():
    r = _run(["--dry-run-cpu", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["world_size_seen"] == 1


@pytest.mark.gpu
@pytest.mark.timeout(290)
def test_gpus2_gloo_same_device_bench():
    """bench.main()'s N > 1 path on a one-GPU box (verdict r03): two ranks on
    cuda:0, gloo with host-copy collectives in place of RCCL.  Exercises the
    multi-rank bookkeeping the driver's scaling run depends on -- the rank
    gather, max-over-ranks timing, configs[4] strong-scaled over 2 z-slabs with
    its all-gather and the per-slab reference hashes -- before such a run does.
    Not a measurement (two ranks share one GPU)."""
    r = _run(["--gpus", "2", "--backend", "gloo", "--same-device", "--steps", "10", "--warmup", "2",
              "--no-cpu-baseline", "--no-host-path", "--no-copy-probe", "--config5-steps", "2",
              "--kernel-ms", "5"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2
    assert d["rank_devices"] == [0, 0]
    assert d["backend"].startswith("gloo")
    c5 = d["config5"]
    assert c5["n_ranks"] == 2 and len(c5["encode_ms_per_rank"]) == 2
    assert c5["parity"]["slabs_match_reference_word_ranges"] is True
    assert c5["parity"]["stream_matches_reference"] is True
    assert c5["allgather"]["backend"].startswith("gloo")
    assert d["allgather"] is not None and d["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(290)
def test_rccl_one_rank_bench():
    """bench.main() through its RCCL branch on a one-GPU box (--dist-init):
    init_process_group("nccl", world_size=1, device_id=cuda:0), the headline's
    and configs[4]'s stream all-gathers on RCCL, the gathered segment equal to
    the local stream.  Not a scaling measurement (one rank)."""
    r = _run(["--gpus", "1", "--dist-init", "--steps", "10", "--warmup", "2", "--no-cpu-baseline",
              "--no-host-path", "--no-copy-probe", "--config5-steps", "2", "--kernel-ms", "5"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["world_size_seen"] == 1
    assert d["backend"].startswith("nccl")
    ag = d["allgather"]
    assert ag is not None and ag["backend"].startswith("nccl") and ag["own_segment_matches"] is True
    c5 = d["config5"]
    assert c5["allgather"]["backend"].startswith("nccl")
    assert c5["parity"]["stream_matches_reference"] is True
    assert d["parity"].startswith("stream and decoded sha256 == reference")


def test_same_device_needs_gloo():
    # two RCCL ranks on one GPU are refused at argument parsing
    r = _run(["--gpus", "2", "--same-device", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "--same-device needs --backend gloo" in r.stderr
