"""Host/device breakdown of one C5 step (bench.py --config c5): wall time of
each call with a device sync after it, plus the engine's own device time."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from musicrecommendation_amd import evaluation, synth
from musicrecommendation_amd.engine import Engine
from musicrecommendation_amd.ensemble import DeviceEnsemble

t0 = time.perf_counter()
ds = synth.config("c5").dataset()
print(f"dataset {time.perf_counter()-t0:.1f} s", flush=True)
eng = Engine(ds, device=0, out_dtype="f32", topk=10)
ens = DeviceEnsemble(eng, pos=evaluation.label_pos(ds), n_label_songs=ds.n_label_songs)
print("launch", eng.shape, eng.block_songs, eng.n_tiles, flush=True)

def timed(name, f, *a, **kw):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = f(*a, **kw)
    torch.cuda.synchronize()
    print(f"  {name:12s} {1e3*(time.perf_counter()-t):8.2f} ms", flush=True)
    return r

for it in range(3):
    print(f"step {it}", flush=True)
    ts = time.perf_counter()
    ubm = timed("ubm", ens.model, "ubm")
    ibm = timed("ibm", ens.model, "ibm")
    m = {"ubm": ubm, "ibm": ibm,
         "lcm": timed("lcm", ens.linear, ubm, ibm, 0.5),
         "am": timed("am", ens.aggregation, ubm, ibm, 0.5),
         "scm": timed("scm", ens.stochastic, ubm, ibm, 0.5, seed=1)}
    for k, t in m.items():
        mn, mx = timed("minmax " + k, eng.eval_minmax, t.data_ptr())
        timed("counts " + k, eng.eval_counts, t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs)
        timed("map " + k, ens.threshold_map, t)
    print(f" step total {1e3*(time.perf_counter()-ts):.1f} ms", flush=True)
