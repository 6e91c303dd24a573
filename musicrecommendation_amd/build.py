"""In-tree build of the HIP engine: csrc/*.hip + csrc/*.cpp -> libmr_engine.so (gfx950).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container; the resulting .so travels to the GPU box with the repository.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "libmr_engine.so")
ARCH = os.environ.get("MR_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    # The fixed-point oracle (oracle/fixedpoint.c) performs the same IEEE ops:
    # no FMA contraction, no fast-math.
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function",
    "-Wl,-rpath,/opt/rocm/lib",
]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _stale(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(p) > t for p in deps)


OUT_STAMPS = os.path.join(HERE, "libmr_engine_stamps.so")


def _compile_all(jobs, verbose: bool) -> None:
    """Compile the (out, extra flags) variants in parallel (one hipcc each)."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    procs = []
    for out, extra in jobs:
        cmd = [hipcc, *FLAGS, *extra, f"-I{INCLUDE}", *sources(), "-o", out + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((out, cmd, subprocess.Popen(cmd)))
    failed = [cmd for out, cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    for out, _cmd, _p in procs:
        os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False, stamps: bool = True) -> str:
    """Production library; plus the diagnostic variant with per-workgroup
    phase timestamps (libmr_engine_stamps.so)."""
    jobs = [(OUT, [])]
    if stamps:
        jobs += [(OUT_STAMPS, ["-DMR_STAMPS"])]
    jobs = [(o, x) for o, x in jobs if force or _stale(o)]
    if jobs:
        _compile_all(jobs, verbose)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
