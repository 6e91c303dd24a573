"""Usable host cores, the rule of csrc/mr_par.h (affinity mask capped by the
cgroup v2 CPU quota, divided among torchrun's LOCAL_WORLD_SIZE ranks of this
node; MR_THREADS overrides)."""
from __future__ import annotations

import os


def usable_cores() -> int:
    if os.environ.get("MR_THREADS", "").isdigit() and int(os.environ["MR_THREADS"]) > 0:
        return min(int(os.environ["MR_THREADS"]), 256)
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    local = os.environ.get("LOCAL_WORLD_SIZE", "")
    if local.isdigit() and int(local) > 1:
        n //= int(local)
    return max(1, min(n, 256))
