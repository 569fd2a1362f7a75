"""The cuda_zfp CLI and data_gen.

CPU tests: data_gen reproduces the reference generator's fields (src/utils/data_gen.cpp:29-80,
restated here in numpy), and cuda_zfp's argument checks (cuda_zfp.cpp:230-268) fail before
any GPU call.  GPU tests: the differential fuzz of tests/fuzz_cli.py (test.py's cases against
the reference's CPU zfp tool), partial blocks, and the zfp header in both its forms.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "cuzfp_amd", "bin")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tools():
    from cuzfp_amd import build
    out = build.build()
    return out["cli"], out["data_gen"]


def _gen(tools, tmp_path, t, dims):
    p = tmp_path / "d.bin"
    subprocess.check_call([tools[1], "-o", str(p), "-t", t, f"-{len(dims)}"] + [str(d) for d in dims])
    return p


def _braid(nx, ny, nz):
    x = np.arange(nx, dtype=np.float64)
    y = np.arange(ny, dtype=np.float64)[:, None]
    dx, dy = 4.0 * 3.14 / (nx - 1), 2.0 * 3.14 / (ny - 1)
    cx, cy = x * dx + 2.0 * 3.14, y * dy - 3.14
    v = np.sin(cx) + np.sin(cy) + 2.0 * np.cos(np.sqrt(cx * cx / 2.0 + cy * cy) / .75) + 4.0 * np.cos(cx * cy / 4.0)
    out = np.repeat(v[None], nz, axis=0)
    if nz > 2:
        dz = 3.0 * 3.14 / (nz - 1)
        for z in range(2, nz):
            cz = z * dz - 1.5 * 3.14
            out[z] = v + np.sin(cz) + 1.5 * np.cos(np.sqrt(cx * cx + cy * cy + cz * cz) / 0.75)
    return out


@pytest.mark.parametrize("t,np_t", [("f32", np.float32), ("f64", np.float64), ("i32", np.int32), ("i64", np.int64)])
def test_data_gen_fields(tools, tmp_path, t, np_t):
    a = np.fromfile(_gen(tools, tmp_path, t, [37]), dtype=np_t)
    want = np.sin(np.arange(37) * (3.14 / 180.)) * 10.0
    np.testing.assert_allclose(a, want.astype(np_t), rtol=1e-6, atol=1 if t[0] == "i" else 1e-6)
    a = np.fromfile(_gen(tools, tmp_path, t, [12, 8, 5]), dtype=np_t).reshape(5, 8, 12)
    want = _braid(12, 8, 5)
    if t[0] == "i":  # C++ static_cast truncates toward zero
        assert np.array_equal(a, np.trunc(want).astype(np_t))
    else:
        np.testing.assert_allclose(a, want.astype(np_t), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("args,msg", [
    ([], "Usage"),
    (["-x"], "Usage"),
    (["-t", "f32", "-1", "16", "-r", "8"], "must specify uncompressed or compressed input file"),
    (["-i", "nofile", "-1", "16", "-r", "8"], "must specify scalar type"),
    (["-i", "nofile", "-t", "f32", "-r", "8"], "must specify array dimensions"),
    (["-i", "nofile", "-t", "f32", "-1", "16"], "must specify compression parameters"),
    (["-z", "nofile", "-t", "f32", "-1", "16", "-r", "8", "-s"], "must specify input file via -i to compute stats"),
    (["-z", "nofile", "-h", "-t", "f32"], "cannot specify both field type/size and header"),
    (["-i", "nofile", "-t", "f32", "-1", "16", "-p", "16"], "only the fixed rate"),
    (["-i", "/nonexistent/x", "-t", "f32", "-1", "16", "-r", "8"], "cannot open input file"),
])
def test_cli_argument_errors(tools, args, msg):
    r = subprocess.run([tools[0]] + args, capture_output=True, text=True)
    assert r.returncode != 0
    assert msg in r.stderr


@pytest.mark.gpu
def test_cli_fuzz_against_cpu_zfp(tools):
    """test.py's generator (dims 4*[1,100], rate [1,31], every scalar type), smaller count."""
    import fuzz_cli
    assert fuzz_cli.main(["--tests", "4", "--seed", "1", "--max-dim", "160", "--quiet"]) == 0


@pytest.mark.gpu
def test_cli_fuzz_partial_and_header(tools):
    import fuzz_cli
    assert fuzz_cli.main(["--tests", "3", "--seed", "2", "--max-dim", "90", "--partial", "--header",
                          "--types", "f32,f64,i32", "--quiet"]) == 0


@pytest.mark.gpu
def test_cli_long_header_and_stats(tools, tmp_path):
    """maxbits > 2048 takes the 64-bit mode word of the header (zfp.c:305-345)."""
    import fuzz_cli
    cli, _ = tools
    raw = _gen(tools, tmp_path, "f64", [20, 16, 12])
    ours, ref = tmp_path / "ours.z", tmp_path / "ref.z"
    subprocess.check_call([cli, "-q", "-h", "-t", "f64", "-3", "20", "16", "12", "-r", "40", "-i", str(raw), "-z", str(ours)])
    subprocess.check_call([fuzz_cli.CPU_ZFP, "-q", "-h", "-d", "-3", "20", "16", "12", "-r", "40", "-i", str(raw), "-z", str(ref)])
    assert ours.read_bytes() == ref.read_bytes()
    r = subprocess.run([cli, "-s", "-t", "f64", "-3", "20", "16", "12", "-r", "40", "-i", str(raw)],
                       capture_output=True, text=True, check=True)
    assert "type=double nx=20 ny=16 nz=12" in r.stderr and "psnr=" in r.stderr


@pytest.mark.gpu
def test_cli_decode_failure_exits_nonzero(tools, tmp_path):
    """A header whose maxbits the codec rejects (rate 300 in 3D f64: 19,200 bits
    per block, past CUZFP_MAX_BITS = 16,384) makes the CLI exit non-zero instead of
    writing a zero-filled output."""
    import fuzz_cli
    cli, _ = tools
    raw = _gen(tools, tmp_path, "f64", [8, 8, 8])
    z = tmp_path / "big.z"
    subprocess.check_call([fuzz_cli.CPU_ZFP, "-q", "-h", "-d", "-3", "8", "8", "8", "-r", "300", "-i", str(raw), "-z", str(z)])
    out = tmp_path / "out.raw"
    r = subprocess.run([cli, "-q", "-h", "-z", str(z), "-o", str(out)], capture_output=True, text=True)
    assert r.returncode != 0
    assert "failed" in r.stderr
