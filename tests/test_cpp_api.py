"""The reference's C++ surface (include/cuZFP.h) through libcuZFP.so.

tests/cpp/t_cuzfp_api.cpp restates the reference's gtest programs
(src/tests/t_sanity_check_{1,2,3}.cpp, t_encode_decode_{1,2,3}.cpp,
t_cuda_mem.cu) against the unchanged API.  Compiling it is a CPU check (the
drop-in headers build caller code unchanged); running it needs the GPU, and
every stream it writes is then compared bit-for-bit with the CPU oracle.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "t_cuzfp_api.cpp")
EXE = os.path.join(ROOT, "build", "t_cuzfp_api")
LIBDIR = os.path.join(ROOT, "cuzfp_amd", "lib")


@pytest.fixture(scope="module")
def exe():
    from cuzfp_amd.build import build
    build()
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(SRC):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", f"-I{ROOT}/include", "-o", EXE, SRC,
                               f"-L{LIBDIR}", "-lcuZFP", "-lcuzfp_hip", f"-Wl,-rpath,{LIBDIR}"])
    return EXE


def test_cpp_tests_compile(exe):
    assert os.access(exe, os.X_OK)


CASES = {  # name: (dtype, shape (slowest first), maxbits)
    "sanity_1": (np.float32, (128,), 32),
    "sanity_2": (np.float32, (4, 4), 128),
    "sanity_3": (np.float32, (4, 8, 16), 512),
    "encode_decode_1": (np.float32, (256,), 32),
    "encode_decode_2": (np.float32, (1024, 4096), 128),
    "encode_decode_3": (np.float32, (256, 256, 256), 512),
    "encode_decode_3_f64": (np.float64, (256, 256, 256), 512),
}


@pytest.mark.gpu
def test_cpp_reference_tests(exe, tmp_path, restatement):
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    for name, (dt, shape, mb) in CASES.items():
        a = np.fromfile(tmp_path / f"{name}.in", dtype=dt).reshape(shape)
        s = np.fromfile(tmp_path / f"{name}.bin", dtype=np.uint64)
        out = np.fromfile(tmp_path / f"{name}.out", dtype=dt).reshape(shape)
        ref = restatement.compress(a, mb)
        assert np.array_equal(s, ref), name
        assert np.array_equal(out.view(np.uint8), restatement.decompress(ref, shape, dt, mb).view(np.uint8)), name
    dev = np.fromfile(tmp_path / "device_stream.bin", dtype=np.uint64)
    assert np.array_equal(dev, np.fromfile(tmp_path / "sanity_3.bin", dtype=np.uint64))
