"""Per-workgroup phase stamps of the co-listening index build (k_cooc_build,
heavy rows, one workgroup per (row, tile)) in the diagnostic build
libmr_engine_stamps.so. Usage: python scripts/cooc_stamps.py [N_TRAIN N_TEST]
Phases (s_memrealtime, 100 MHz): zero the counters | walk the listeners |
count + reserve | write the segment."""
import os
import sys

os.environ.setdefault("MR_ENGINE_LIB", "stamps")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

n_tr = int(sys.argv[1]) if len(sys.argv) > 1 else 1_009_318
n_te = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
ds = synth.generate_bulk(n_tr, n_te, 4).dataset()
with Engine(ds, topk=10, dense=False, ibm_route="cooc") as e:
    e.run("ibm")
    e.sync()
    e.run("ibm")
    e.sync()
    off = e.n_tiles * (max(e.batch, min(n_te, 65528)) + 8) * 32
    total = off + 8 * e.n_tiles * e.cooc_rows
    buf = np.zeros(total, dtype=np.int64)
    assert e._L.mr_debug_stamps(e._h, buf.ctypes.data, buf.size) == 0
b = buf[off:].reshape(-1, 8)
b = b[b[:, 0] != 0]
us = (b[:, :5] - b[:, :1]).astype(np.float64) * 10.0 / 1e3  # from WG start, us
n = b[:, 6]
dense = b[:, 5] == 1
span = (b[:, 4].max() - b[:, 0].min()) * 10.0 / 1e3
dur = us[:, 4]
print(f"{n_tr}/{n_te}: build WGs {len(b)} (dense segments {dense.mean():.2f}), kernel span {span / 1e3:.2f} ms, "
      f"sum(WG time)/512 = {dur.sum() / 512 / 1e3:.2f} ms")
for name, a, c in (("zero", 0, 1), ("walk", 1, 2), ("count", 2, 3), ("write", 3, 4), ("total", 0, 4)):
    d = us[:, c] - us[:, a]
    print(f"  {name:6s} us med {np.median(d):8.1f} p90 {np.percentile(d, 90):8.1f} max {d.max():9.1f} "
          f"share {d.sum() / dur.sum():.3f}")
edges = [0, 256, 1024, 4096, 16384, 65536, 1 << 30]
for lo, hi in zip(edges[:-1], edges[1:]):
    m = (n >= lo) & (n < hi)
    if not m.any():
        continue
    w = us[m, 2] - us[m, 1]
    print(f"  listeners [{lo},{hi}): WGs {m.sum():7d} walk med {np.median(w):8.1f} us, total med "
          f"{np.median(dur[m]):8.1f} us, share of WG time {dur[m].sum() / dur.sum():.3f}")
