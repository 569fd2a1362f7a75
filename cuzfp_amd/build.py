"""Build the MI355X codec libraries in-tree (hipcc for gfx950, no JIT cache).

Outputs (git-ignored, shipped to the GPU box with the repo snapshot):
  cuzfp_amd/lib/libcuzfp_hip.so  -- kernels + the C-ABI of include/cuzfp_hip.h
  cuzfp_amd/lib/libcuZFP.so      -- the reference's C++ surface (include/cuZFP.h)
  cuzfp_amd/bin/cuda_zfp         -- the reference's CLI (src/utils/cuda_zfp.cpp) on libcuZFP.so
  cuzfp_amd/bin/data_gen         -- the reference's test-data generator (src/utils/data_gen.cpp)
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
BIN = os.path.join(HERE, "bin")
CLI = os.path.join(HERE, "cli")
OBJ = os.path.join(ROOT, "build", "obj")
INC = os.path.join(ROOT, "include")

ARCH = os.environ.get("CUZFP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INC}",
            "-Wall", "-Wno-unused-function", "-Wno-pass-failed"]

KERNEL_UNITS = ["inst_f32", "inst_f64", "inst_i32", "inst_i64", "capi"]
HEADERS = ["zfp_block.hpp", "kernels.hpp", "launch.hpp"]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))


def build(verbose: bool = False, jobs: int | None = None) -> dict:
    """Compile (incrementally) and link both libraries; returns their paths."""
    os.makedirs(LIB, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INC, "cuzfp_hip.h")]
    jobs_list = []
    objs = []
    for u in KERNEL_UNITS:
        src = os.path.join(CSRC, u + ".hip")
        obj = os.path.join(OBJ, u + ".o")
        objs.append(obj)
        if _newer(obj, [src] + hdrs):
            jobs_list.append([HIPCC, *CXXFLAGS, "-c", src, "-o", obj])
    with ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
        for cmd in jobs_list:
            if verbose:
                print(" ".join(cmd))
        list(ex.map(_run, jobs_list))
    hip_so = os.path.join(LIB, "libcuzfp_hip.so")
    if jobs_list or _newer(hip_so, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", hip_so, *objs])
    cpp_src = os.path.join(CSRC, "cuZFP.cpp")
    cpp_so = os.path.join(LIB, "libcuZFP.so")
    if _newer(cpp_so, [cpp_src, hip_so, os.path.join(INC, "cuZFP.h"),
                       os.path.join(INC, "zfp_structs.h")]):
        _run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{INC}", "-o", cpp_so, cpp_src,
              f"-L{LIB}", "-lcuzfp_hip", "-Wl,-rpath,$ORIGIN"])
    os.makedirs(BIN, exist_ok=True)
    cli = os.path.join(BIN, "cuda_zfp")
    if _newer(cli, [os.path.join(CLI, "cuda_zfp.cpp"), cpp_so, os.path.join(INC, "cuZFP.h"),
                    os.path.join(INC, "zfp_structs.h")]):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-Wno-unused-function", f"-I{INC}", "-o", cli,
              os.path.join(CLI, "cuda_zfp.cpp"), f"-L{LIB}", "-lcuZFP", "-Wl,-rpath,$ORIGIN/../lib"])
    gen = os.path.join(BIN, "data_gen")
    if _newer(gen, [os.path.join(CLI, "data_gen.cpp")]):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-o", gen, os.path.join(CLI, "data_gen.cpp")])
    return {"hip": hip_so, "cpp": cpp_so, "cli": cli, "data_gen": gen}


if __name__ == "__main__":
    print(build(verbose=True))
