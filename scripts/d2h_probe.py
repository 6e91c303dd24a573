"""Dense D2H probe (C3 by default): GB/s of mr_copy_dense into a fresh numpy
array (Engine.dense), a huge-page mapping, a reused (already touched) array
and a pinned torch buffer, on one engine and on a fresh engine
per copy (as bench.py's end_to_end does).
Usage: python scripts/d2h_probe.py [config] [reps]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ds = synth.config(cfg).dataset()
res = {"config": cfg}


def copy_into(e, out):
    t = time.perf_counter()
    rc = e._L.mr_copy_dense(e._h, ctypes.c_void_p(out))
    assert rc == 0, e._L.mr_last_error()
    return time.perf_counter() - t


e = Engine(ds, device=0, out_dtype="f32", topk=10)
e.run("ibm")
e.sync()
nbytes = e.n_test * e.width * 4
res["bytes"] = nbytes
gbs = lambda ts: [round(nbytes / t / 1e9, 2) for t in ts]  # noqa: E731
ts = []
for _ in range(reps):
    t = time.perf_counter()
    d = e.dense()
    ts.append(time.perf_counter() - t)
    del d  # the munmap of 632 MB stays outside the timing
res["engine_dense_GBps"] = gbs(ts)
ts = []
for _ in range(reps):
    a = np.empty((e.n_test, e.width), np.float32)  # held: the copy writes into it
    ts.append(copy_into(e, a.ctypes.data))
    del a
res["fresh_numpy_empty_GBps"] = gbs(ts)
a = np.empty((e.n_test, e.width), np.float32)
a.fill(0)
res["touched_array_GBps"] = gbs([copy_into(e, a.ctypes.data) for _ in range(reps)])
t = time.perf_counter()
p = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
res["pinned_alloc_ms"] = round((time.perf_counter() - t) * 1e3, 2)
res["pinned_GBps"] = gbs([copy_into(e, p.data_ptr()) for _ in range(reps)])
ts = []
import mmap  # noqa: E402
for _ in range(reps):  # fresh anonymous mapping with MADV_HUGEPAGE (THP-backed first touch)
    m = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if hasattr(mmap, "MADV_HUGEPAGE"):
        m.madvise(mmap.MADV_HUGEPAGE)
    arr = np.frombuffer(m, dtype=np.float32)
    ts.append(copy_into(e, arr.ctypes.data))
    del arr
    m.close()
res["fresh_thp_mapping_GBps"] = gbs(ts)
for f in ("enabled", "defrag"):
    try:
        with open("/sys/kernel/mm/transparent_hugepage/" + f) as fh:
            res["thp_" + f] = fh.read().strip()
    except OSError as ex:
        res["thp_" + f] = str(ex)
e.close()
ts = []
for _ in range(reps):
    e = Engine(ds, device=0, out_dtype="f32", topk=10)
    e.run("ibm")
    e.sync()
    t = time.perf_counter()
    d = e.dense()
    ts.append(time.perf_counter() - t)
    del d
    e.close()
res["engine_dense_fresh_engine_GBps"] = gbs(ts)
print(json.dumps(res))
