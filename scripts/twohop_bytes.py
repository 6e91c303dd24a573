"""SURVEY.md §8(d)'s two-hop byte model of a full-scale config, computed once
on the host (bench.algorithmic_bytes walks every test user's neighbour set:
minutes at C4) and cached in profiles/<config>_twohop_bytes.json, which
bench.py reads beside the co-listening route's own byte model (the north-star
block): the route does less work than the survey's algorithm, bit-exactly, so
its time against the survey's bytes can exceed the roofline.
  python scripts/twohop_bytes.py [c4|c5]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import algorithmic_bytes, dataset_signature  # noqa: E402
from musicrecommendation_amd import synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    t0 = time.time()
    ds = synth.config(cfg).dataset()
    t1 = time.time()
    ab = algorithmic_bytes(ds, 0, 10)  # top-10 only (no dense output), as the north-star block
    out = {"config": cfg, "signature": dataset_signature(ds), "out_bytes": 0, "k": 10,
           "bytes": ab, "total_bytes": int(sum(ab.values())),
           "note": "SURVEY.md §8(d) two-hop byte model (bench.algorithmic_bytes, top-k only): stage 1 "
                   "12|T(u)| + 4 Σ c_tr(s2); stage 2 Σ_{v∈N(u)} (8 + 4|S(v)|) + 4 n_s; merge 12 k",
           "generate_s": t1 - t0, "model_s": time.time() - t1}
    path = os.path.join(ROOT, "profiles", f"{cfg}_twohop_bytes.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
