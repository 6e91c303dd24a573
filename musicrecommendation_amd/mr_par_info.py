"""Usable host cores, the rule of csrc/mr_par.h (affinity mask capped by the
cgroup v2 CPU quota, divided among torchrun's LOCAL_WORLD_SIZE ranks of this
node unless each rank is pinned to its own CPU set; MR_THREADS overrides)."""
from __future__ import annotations

import os


def usable_cores() -> int:
    if os.environ.get("MR_THREADS", "").isdigit() and int(os.environ["MR_THREADS"]) > 0:
        return min(int(os.environ["MR_THREADS"]), 256)
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = 0
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    # split among the node's ranks only when this rank's mask covers the whole
    # share (a launcher that pinned each rank to its own CPU set already split it)
    shared_mask = n >= (quota if quota > 0 else (os.cpu_count() or 1))
    if quota > 0:
        n = min(n, max(1, quota))
    local = os.environ.get("LOCAL_WORLD_SIZE", "")
    if shared_mask and local.isdigit() and int(local) > 1:
        n //= int(local)
    return max(1, min(n, 256))
