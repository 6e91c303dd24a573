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


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(p) > t for p in deps)


OUT_STAMPS = os.path.join(HERE, "libmr_engine_stamps.so")
OUT_CHECKS = os.path.join(HERE, "libmr_engine_checks.so")


def _compile(out: str, extra, verbose: bool) -> None:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, *extra, f"-I{INCLUDE}", *sources(), "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False, stamps: bool = True) -> str:
    """Production library; plus the diagnostic variants (phase timestamps,
    bounds-checked pull kernels)."""
    if force or _stale():
        _compile(OUT, [], verbose)
        if stamps:
            _compile(OUT_STAMPS, ["-DMR_STAMPS"], verbose)
            _compile(OUT_CHECKS, ["-DMR_CHECKS"], verbose)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
