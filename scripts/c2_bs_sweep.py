"""C2 device time per step (engine-stream event window, as bench.py) across
fused tile widths. Usage: python scripts/c2_bs_sweep.py [model] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "ibm"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 400
ds = synth.config("c2").dataset()
shapes = (("fused", (256, 512, 768, 1024, 2048)),)
if os.environ.get("BS"):
    shapes = (("fused", tuple(int(x) for x in os.environ["BS"].split())),)
for stage1, bss in shapes:
    for bs in bss:
        e = Engine(ds, stage1=stage1, block_songs=bs, topk=10, out_dtype="f32")
        res = []
        for rep in range(3):
            for _ in range(30):
                e.run(model)
            e.sync()
            e.timing_begin()
            for _ in range(steps):
                e.run(model)
            n, ms = e.timing_end()
            res.append(ms / steps * 1e3)
        print(f"merge_rows={os.environ.get('MR_MERGE_ROWS', '-')} {stage1:6s} bs={e.block_songs:5d} tiles={e.n_tiles:3d} us/step " + " ".join(f"{r:6.2f}" for r in res),
              flush=True)
        e.close()
