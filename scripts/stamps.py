"""Phase timestamps of the scoring kernel (diagnostic build libmr_engine_stamps.so).
Usage: python scripts/stamps.py [config] [model] [block_songs] [stage1]"""
import os
import sys

os.environ.setdefault("MR_ENGINE_LIB", "stamps")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
model = sys.argv[2] if len(sys.argv) > 2 else "ibm"
bs = int(sys.argv[3]) if len(sys.argv) > 3 else 0
stage1 = sys.argv[4] if len(sys.argv) > 4 else "auto"
ds = synth.config(cfg).dataset()
e = Engine(ds, block_songs=bs, stage1=stage1)
for _ in range(20):
    e.run(model)
e.sync()
n = e.n_tiles * ds.n_test
buf = np.zeros(n * 32, dtype=np.int64)
rc = e._L.mr_debug_stamps(e._h, buf.ctypes.data, buf.size)
assert rc == 0, e._L.mr_last_error()
full = buf.reshape(n, 32)
rt = full[:, :16].astype(np.float64) * 10.0 / 1e3  # us (100 MHz)
cy = full[:, 16:].astype(np.float64)
last = (full[:, 15] & 1) == 1
t0 = rt[:, 0].min()
print(f"{cfg} {model} fused={e.fused} bs={e.block_songs} tiles={e.n_tiles} WGs={n}")
mhz = (cy[:, 5] - cy[:, 0]) / (rt[:, 5] - rt[:, 0])
print(f"clock MHz med {np.median(mhz):.0f}; WG start offsets us min/med/max",
      *np.round(np.percentile(rt[:, 0] - t0, [0, 50, 100]), 2))


def phase(name, a, b, rows=None):
    rows = np.ones(n, bool) if rows is None else rows
    d = rt[rows, b] - rt[rows, a]
    c = cy[rows, b] - cy[rows, a]
    print(f"  {name:22s} us med {np.median(d):7.3f} p90 {np.percentile(d, 90):7.3f} max {d.max():7.3f}"
          f"   kcyc med {np.median(c) / 1e3:6.2f}")


phase("stage1", 0, 1)
if e.fused and (full[:, 10] != 0).all() and (full[:, 11] != 0).all():  # fused stage-1 sub-phases
    phase("  songs+scan", 0, 10)
    phase("  search+loads+adds", 10, 11)
    phase("  barrier wait+weights", 11, 1)
phase("stage2", 1, 2)
phase("epilogue", 2, 3)
phase("tile-topk", 3, 4)
if (full[:, 12] != 0).all():  # diagnostic sub-phases of the fused tile top-k
    phase("  topk best+rows", 3, 12)
    phase("  topk row rank/tau", 12, 13)
    phase("  topk collect", 13, 14)
    phase("  topk rank+write", 14, 4)
phase("handoff", 4, 5)
phase("merge stage", 5, 6, last)
phase("merge tournament", 6, 8, last)
phase("merge write", 8, 9, last)
end = np.where(last, rt[:, 9], rt[:, 5])
print("WG end offsets (us) min/med/max", *np.round(np.percentile(end - t0, [0, 50, 100]), 2))
lu = np.where(last)[0]
print("last-WG merge start (us) per user:", np.round(rt[lu, 5] - t0, 2).tolist())
if e.fused and e.shape == "fused":
    nt = e.n_tiles
    sub = (("s1 songs", 0, 10), ("s1 gather", 10, 11), ("s1 tail", 11, 1)) if (full[:, 10] != 0).all() else ()
    for name, a, b in (("stage1", 0, 1), *sub, ("stage2", 1, 2), ("start", None, 0)):
        d = (rt[:, b] - (rt[:, a] if a is not None else t0)).reshape(-1, nt)
        print(f"per-user {name:9s} med/max us:", [(round(float(np.median(r)), 2), round(float(r.max()), 2)) for r in d])
