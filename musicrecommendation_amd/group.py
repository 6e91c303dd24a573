"""Python handle on a multi-GPU group (include/mr_engine.h ``mr_group_*``).

One call fans out over G = song shards x test-user blocks engine contexts and
exchanges the per-user top-k lists inside the library (RCCL all-gather when the
contexts span several GPUs, device copies when they share one) — the C-ABI
counterpart of the reference's ``getItemBasedModel2`` / ``getUserBasedModel2``
(distributed.scala:459-479: ``parallelize(songs, n).map(getRanks2).collect``).
A single-threaded caller (the JNI shim of INTEGRATION.md) reaches every GPU
through it; ``sharding.py`` is the one-process-per-GPU (torchrun) equivalent.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .dataset import Dataset
from .engine import model_id

TRANSPORTS = {"auto": _lib.MR_TRANSPORT_AUTO, "copy": _lib.MR_TRANSPORT_COPY, "rccl": _lib.MR_TRANSPORT_RCCL}


def song_shards_native(ds: Dataset, n_shards: int, tile: int = 0) -> List[Tuple[int, int]]:
    """The group's shard boundaries (mr_song_shards / mr_song_shards_tiled; host only)."""
    L = _lib.lib()
    cd = ds.c_struct()
    b = np.empty(n_shards + 1, dtype=np.int32)
    if tile > 0:
        _lib.check(L.mr_song_shards_tiled(ctypes.byref(cd), n_shards, int(tile), b.ctypes.data_as(ctypes.c_void_p)),
                   "mr_song_shards_tiled")
    else:
        _lib.check(L.mr_song_shards(ctypes.byref(cd), n_shards, b.ctypes.data_as(ctypes.c_void_p)),
                   "mr_song_shards")
    return [(int(b[g]), int(b[g + 1])) for g in range(n_shards)]


class Group:
    def __init__(self, dataset: Dataset, *, song_shards: int = 1, user_blocks: int = 1,
                 devices: Optional[Sequence[int]] = None, transport: str = "auto", frac_bits: int = 32,
                 out_dtype: str = "f32", topk: int = 10, dense: bool = True, stage1: str = "auto",
                 ibm_route: str = "auto"):
        self._L = _lib.lib()
        opt = _lib.MrOptions()
        _lib.check(self._L.mr_options_default(ctypes.byref(opt)), "mr_options_default")
        opt.frac_bits = frac_bits
        opt.out_dtype = {"f32": _lib.MR_OUT_F32, "f64": _lib.MR_OUT_F64}[out_dtype]
        opt.topk = topk
        opt.dense = 1 if dense else 0
        opt.stage1 = _lib.STAGE1[stage1]
        opt.ibm_route = {"auto": 0, "two_hop": 1, "cooc": 2}[ibm_route]  # mr_options.ibm_route
        go = _lib.MrGroupOptions()
        _lib.check(self._L.mr_group_options_default(ctypes.byref(go)), "mr_group_options_default")
        go.n_song_shards, go.n_user_blocks = song_shards, user_blocks
        go.transport = TRANSPORTS[transport]
        devs = np.ascontiguousarray(list(devices) if devices else [0], dtype=np.int32)
        go.n_devices = devs.size
        go.devices = devs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        self.dtype = np.float32 if out_dtype == "f32" else np.float64
        self.topk_k = topk
        self.n_contexts = song_shards * user_blocks
        self._h = ctypes.c_void_p()
        _lib.check(self._L.mr_group_create(ctypes.byref(opt), ctypes.byref(go), ctypes.byref(self._h)),
                   "mr_group_create")
        self.dataset = dataset
        try:
            cd = dataset.c_struct()
            _lib.check(self._L.mr_group_load(self._h, ctypes.byref(cd)), "mr_group_load")
        except Exception:
            self.close()
            raise
        t = ctypes.c_int32()
        _lib.check(self._L.mr_group_transport(self._h, ctypes.byref(t)), "mr_group_transport")
        self.transport = {v: k for k, v in TRANSPORTS.items()}[t.value]
        self.layout = []  # per context: (song_lo, song_hi, user_lo, user_hi, device)
        for i in range(self.n_contexts):
            v = [ctypes.c_int32() for _ in range(5)]
            _lib.check(self._L.mr_group_info(self._h, i, *[ctypes.byref(x) for x in v]), "mr_group_info")
            self.layout.append(tuple(x.value for x in v))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.mr_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def run(self, model) -> None:
        _lib.check(self._L.mr_group_run(self._h, model_id(model)), "mr_group_run")

    def sync(self) -> None:
        _lib.check(self._L.mr_group_sync(self._h), "mr_group_sync")

    def topk(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        n, k = self.dataset.n_test, self.topk_k
        songs = np.empty((n, k), np.int32)
        scores = np.empty((n, k), np.float64)
        keys = np.empty((n, k), np.int64)
        _lib.check(self._L.mr_group_copy_topk(self._h, songs.ctypes.data_as(ctypes.c_void_p),
                                              scores.ctypes.data_as(ctypes.c_void_p),
                                              keys.ctypes.data_as(ctypes.c_void_p)), "mr_group_copy_topk")
        return songs, scores, keys

    def dense(self) -> np.ndarray:
        out = np.empty((self.dataset.n_test, self.dataset.n_songs), self.dtype)
        _lib.check(self._L.mr_group_copy_dense(self._h, out.ctypes.data_as(ctypes.c_void_p)), "mr_group_copy_dense")
        return out

    def allgather_dense(self, dst_ptrs: Sequence[int]) -> None:
        """dst_ptrs[i]: device buffer on context i's GPU, (user_hi - user_lo) x n_songs."""
        arr = (ctypes.c_void_p * len(dst_ptrs))(*dst_ptrs)
        _lib.check(self._L.mr_group_allgather_dense(self._h, arr), "mr_group_allgather_dense")

    def device_topk(self, i: int) -> Tuple[int, int, int]:
        p = [ctypes.c_void_p() for _ in range(3)]
        _lib.check(self._L.mr_group_device_topk(self._h, i, *[ctypes.byref(x) for x in p]), "mr_group_device_topk")
        return tuple(x.value or 0 for x in p)
