"""GPU check of the lane-pair 3D f32 encoder against the one-block-per-lane
encoder (CUZFP_SPLIT3=0) and the reference's golden hashes; timing of both
(design tool: python tools/split_check.py on the GPU box)."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import os, sys, json, hashlib, torch, numpy as np
sys.path.insert(0, @ROOT@)
import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
out = {}
rng = np.random.default_rng(5)
# parity on random shapes / rates (multiple-of-4 extents and maxbits % 64 == 0 take the split kernel)
streams = {}
for t in range(40):
    shape = tuple(int(4 * rng.integers(1, 20)) for _ in range(3))
    kind = t % 4
    if kind == 0: a = np.cumsum(rng.standard_normal(shape), axis=-1)
    elif kind == 1: a = rng.standard_normal(shape)
    elif kind == 2: a = rng.standard_normal(shape) * 10.0 ** rng.integers(-30, 30, size=shape)
    else: a = np.where(rng.random(shape) < 0.6, 0.0, rng.standard_normal(shape))
    a = a.astype(np.float32)
    mb = 64 * int(rng.integers(1, 40))
    w = cz.encode(torch.from_numpy(a).cuda(), mb)
    streams[t] = hashlib.sha256(w.cpu().numpy().tobytes()).hexdigest()
out['fuzz'] = streams
gold = json.load(open(os.path.join(@ROOT@, 'tests', 'golden', 'golden.json')))['cases']
for field in ('polynomial', 'splitmix'):
    shape = (256,) * 3
    arr = polynomial_field(shape) if field == 'polynomial' else splitmix_uniform(shape)
    x = torch.from_numpy(arr).cuda()
    mb = 512
    w = cz.encode(x, mb); y = cz.decode(w, shape, x.dtype, mb)
    torch.cuda.synchronize()
    g = gold['baseline/3d_f32_256_r8/' + field]
    ok = hashlib.sha256(w.cpu().numpy().tobytes()).hexdigest() == g['stream_sha256']
    def t(fn):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20): fn()
        gr.replay(); torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        r = []
        for _ in range(11):
            torch.cuda.synchronize(); e0.record(); gr.replay(); gr.replay(); e1.record(); torch.cuda.synchronize()
            r.append(e0.elapsed_time(e1) / 40 * 1000)
        return round(sorted(r)[5], 2)
    def step():
        cz.encode(x, mb, out=w); cz.decode(w, shape, x.dtype, mb, out=y)
    out[field] = dict(stream_ok=ok, enc_us=t(lambda: cz.encode(x, mb, out=w)), step_us=t(step))
print(json.dumps(out))
"""


def run(split):
    env = dict(os.environ, CUZFP_SPLIT3=str(split))
    r = subprocess.run([sys.executable, "-c", CODE.replace("@ROOT@", repr(ROOT))], capture_output=True, text=True, env=env,
                       timeout=300)
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)
    return json.loads(r.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    a = run(1)
    b = run(0)
    same = [k for k in a["fuzz"] if a["fuzz"][k] == b["fuzz"][k]]
    print("fuzz streams equal (split vs per-lane):", len(same), "of", len(a["fuzz"]))
    for f in ("polynomial", "splitmix"):
        print(f, "split", a[f], "per-lane", b[f])
