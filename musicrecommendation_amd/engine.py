"""Python handle on one engine context (one GPU, one song-range shard).

Thin wrapper over the C ABI (include/mr_engine.h); all compute runs in the HIP
kernels of csrc/mr_engine.hip. There is no CPU fallback: without a GPU or
without the built library every call raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple, Union

import numpy as np

from . import _lib
from .dataset import Dataset

MODELS = {"ubm": _lib.MR_UBM, "ibm": _lib.MR_IBM, _lib.MR_UBM: _lib.MR_UBM, _lib.MR_IBM: _lib.MR_IBM}
KERNELS = {"neighbours": 0, "score": 1}
# mr_options.ibm_route: the wide shape's ItemBasedModel route
IBM_ROUTES = {"auto": 0, "two_hop": 1, "cooc": 2}


def model_id(model: Union[str, int]) -> int:
    try:
        return MODELS[model]
    except KeyError:
        raise ValueError(f"unknown model {model!r}: use 'ubm' or 'ibm'") from None


class Engine:
    def __init__(self, dataset: Dataset, *, device: int = 0, frac_bits: int = 32, song_lo: int = 0,
                 song_hi: int = 0, block_songs: int = 0, out_dtype: str = "f32", topk: int = 10,
                 dense: bool = True, time_kernels: bool = False, stage1: str = "auto",
                 stage1_chunk: int = 0, train_order: str = "auto", topk_lists: bool = False,
                 ibm_route: str = "auto"):
        self._L = _lib.lib()
        opt = _lib.MrOptions()
        _lib.check(self._L.mr_options_default(ctypes.byref(opt)), "mr_options_default")
        opt.device = device
        opt.frac_bits = frac_bits
        opt.song_lo = song_lo
        opt.song_hi = song_hi
        opt.block_songs = block_songs
        opt.out_dtype = {"f32": _lib.MR_OUT_F32, "f64": _lib.MR_OUT_F64}[out_dtype]
        opt.topk = topk
        opt.dense = 1 if dense else 0
        opt.time_kernels = 1 if time_kernels else 0
        opt.stage1 = _lib.STAGE1[stage1]
        opt.stage1_chunk = stage1_chunk
        opt.train_order = {"auto": 0, "given": 1}[train_order]
        opt.topk_lists = 1 if topk_lists else 0
        opt.ibm_route = IBM_ROUTES[ibm_route]
        self.opt = opt
        self.dtype = np.float32 if out_dtype == "f32" else np.float64
        self._h = ctypes.c_void_p()
        _lib.check(self._L.mr_create(ctypes.byref(opt), ctypes.byref(self._h)), "mr_create")
        self.dataset = dataset
        try:
            cd = dataset.c_struct()
            _lib.check(self._L.mr_load(self._h, ctypes.byref(cd)), "mr_load")
        except Exception:
            self.close()
            raise
        lo, hi, nte = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self._L.mr_shard_info(self._h, ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(nte)),
                   "mr_shard_info")
        self.song_lo, self.song_hi, self.n_test = lo.value, hi.value, nte.value
        self.width = self.song_hi - self.song_lo
        self.topk_k = topk
        fz, bsz, nt = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self._L.mr_launch_info(self._h, ctypes.byref(fz), ctypes.byref(bsz), ctypes.byref(nt)),
                   "mr_launch_info")
        self.shape = _lib.SHAPES[fz.value]
        self.fused, self.block_songs, self.n_tiles = self.shape == "fused", bsz.value, nt.value
        b, ch, nch = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self._L.mr_batch_info(self._h, ctypes.byref(b), ctypes.byref(ch), ctypes.byref(nch)),
                   "mr_batch_info")
        self.batch, self.stage1_chunk, self.n_chunks = b.value, ch.value, nch.value
        rt, nr, pe = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        _lib.check(self._L.mr_route_info(self._h, ctypes.byref(rt), ctypes.byref(nr), ctypes.byref(pe)),
                   "mr_route_info")
        # "two_hop" or "cooc" (co-listening index), and the index's size
        self.ibm_route = {1: "two_hop", 2: "cooc"}[rt.value]
        self.cooc_rows, self.cooc_pool_entries = nr.value, pe.value
        co = ctypes.c_int32()
        _lib.check(self._L.mr_topk_mode(self._h, ctypes.byref(co)), "mr_topk_mode")
        # wide shape, top-k only: the tile top-k over fp32 approximations + exact candidates
        self.candidate_topk = bool(co.value)

    # ---- lifecycle ----------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.mr_destroy(self._h)
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

    # ---- compute --------------------------------------------------------------
    def run(self, model: Union[str, int]) -> None:
        """Asynchronous: score every pair of the shard into device buffers."""
        _lib.check(self._L.mr_run(self._h, model_id(model)), "mr_run")

    def cooc_stats(self) -> Tuple[int, int, int]:
        """(index non-zeros, entries consumed by the scoring, entries the build
        reads) of the latest ibm run on the co-listening route (mr_cooc_stats)."""
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self._L.mr_cooc_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "mr_cooc_stats")
        return a.value, b.value, c.value

    def cooc_bytes(self) -> dict:
        """Encoding-independent byte counts of the latest ibm run on the
        co-listening route, split heavy / light rows (mr_cooc_bytes)."""
        b = _lib.MrCoocBytes()
        _lib.check(self._L.mr_cooc_bytes(self._h, ctypes.byref(b)), "mr_cooc_bytes")
        return {name: int(getattr(b, name)) for name, _t in _lib.MrCoocBytes._fields_}

    def sync(self) -> None:
        _lib.check(self._L.mr_sync(self._h), "mr_sync")

    def graph_capture(self, model: Union[str, int], n_steps: int) -> None:
        """Capture n_steps back-to-back runs of `model` into a HIP graph."""
        _lib.check(self._L.mr_graph_capture(self._h, model_id(model), int(n_steps)), "mr_graph_capture")

    def graph_launch(self) -> None:
        """Replay the captured graph (asynchronous on the engine stream)."""
        _lib.check(self._L.mr_graph_launch(self._h), "mr_graph_launch")

    @property
    def stream(self) -> int:
        return self._L.mr_stream(self._h) or 0

    def dense(self) -> np.ndarray:
        """n_test x width scores of the last run (NaN = heard song, no pair)."""
        out = np.empty((self.n_test, self.width), dtype=self.dtype)
        _lib.check(self._L.mr_copy_dense(self._h, out.ctypes.data_as(ctypes.c_void_p)), "mr_copy_dense")
        return out

    def topk(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(songs int32, scores f64, keys int64), each n_test x k, of the last run."""
        k = self.topk_k
        songs = np.empty((self.n_test, k), dtype=np.int32)
        scores = np.empty((self.n_test, k), dtype=np.float64)
        keys = np.empty((self.n_test, k), dtype=np.int64)
        _lib.check(self._L.mr_copy_topk(self._h, songs.ctypes.data_as(ctypes.c_void_p),
                                        scores.ctypes.data_as(ctypes.c_void_p),
                                        keys.ctypes.data_as(ctypes.c_void_p)), "mr_copy_topk")
        return songs, scores, keys

    def copy_topk_device(self, songs_ptr: int, keys_ptr: int, wait: bool = True) -> None:
        """Copy the last run's top-k lists into device buffers (D2D); wait=False
        only enqueues the copies on the engine stream."""
        fn = self._L.mr_copy_topk_device if wait else self._L.mr_copy_topk_device_async
        _lib.check(fn(self._h, songs_ptr, keys_ptr), "mr_copy_topk_device")

    def score_dense(self, model: Union[str, int]) -> np.ndarray:
        self.run(model)
        return self.dense()

    def device_outputs(self) -> Tuple[int, int, int, int]:
        ptrs = [ctypes.c_void_p() for _ in range(4)]
        _lib.check(self._L.mr_device_outputs(self._h, *[ctypes.byref(p) for p in ptrs]), "mr_device_outputs")
        return tuple(p.value or 0 for p in ptrs)

    def merge_topk_device(self, n_shards: int, songs_ptr: int, keys_ptr: int, out_songs_ptr: int,
                          out_keys_ptr: int, out_scores_ptr: int = 0, wait: bool = True) -> None:
        """Merge n_shards gathered [shard][n_test][k] device lists on this GPU
        (wait=False: enqueued on the engine stream only)."""
        if wait:
            rc = self._L.mr_topk_merge_device(self._h, n_shards, self.n_test, self.topk_k, songs_ptr, keys_ptr,
                                              None, out_songs_ptr, out_keys_ptr, out_scores_ptr or None)
        else:
            rc = self._L.mr_topk_merge_device_async(self._h, n_shards, self.n_test, self.topk_k, songs_ptr,
                                                    keys_ptr, out_songs_ptr, out_keys_ptr, out_scores_ptr or None)
        _lib.check(rc, "mr_topk_merge_device")

    def record_bytes(self) -> int:
        """Bytes of this engine's top-k record block (keys then songs, padded):
        the unit of the single all-gather of a song-sharded exchange."""
        b = ctypes.c_int64()
        _lib.check(self._L.mr_topk_record_bytes(self.n_test, self.topk_k, ctypes.byref(b)), "mr_topk_record_bytes")
        return b.value

    def copy_topk_record(self, record_ptr: int, wait: bool = False) -> None:
        """Copy the last run's lists into a device record block (keys at byte 0,
        songs at byte 8 * n_test * k)."""
        n = self.n_test * self.topk_k
        self.copy_topk_device(record_ptr + 8 * n, record_ptr, wait=wait)

    def merge_topk_records(self, n_shards: int, records_ptr: int, rec_bytes: int, out_songs_ptr: int,
                           out_keys_ptr: int, out_scores_ptr: int = 0) -> None:
        """Merge n_shards gathered record blocks (stride rec_bytes) on this GPU,
        enqueued on the engine stream."""
        _lib.check(self._L.mr_topk_merge_records_async(self._h, n_shards, self.n_test, self.topk_k, records_ptr,
                                                       rec_bytes, out_songs_ptr, out_keys_ptr, out_scores_ptr or None),
                   "mr_topk_merge_records_async")

    # ---- device-resident models (combination models, evaluation) -------------
    def run_into(self, model: Union[str, int], dense_ptr: int) -> None:
        """Asynchronous: like run(), the dense model written to a caller-owned
        device buffer (n_test x width of this engine's dtype)."""
        _lib.check(self._L.mr_run_into(self._h, model_id(model), ctypes.c_void_p(dense_ptr)), "mr_run_into")

    def topk_dense(self, dense_ptr: int) -> None:
        """Top-k of a dense device model into this engine's top-k outputs (read
        them with topk()); synchronous."""
        _lib.check(self._L.mr_topk_dense_device(self._h, ctypes.c_void_p(dense_ptr), self.topk_k),
                   "mr_topk_dense_device")

    def combine(self, kind: int, param: float, ubm_ptr: int, ibm_ptr: int, out_ptr: int, *, seed: int = 0,
                pair_base: int = 0, n_pairs: int = 0) -> None:
        """Combination model (MR:317-481) of two dense device models; synchronous."""
        _lib.check(self._L.mr_combine_device(self._h, kind, float(param), int(seed) & (2 ** 64 - 1), int(pair_base),
                                             int(n_pairs), ctypes.c_void_p(ubm_ptr), ctypes.c_void_p(ibm_ptr),
                                             ctypes.c_void_p(out_ptr)), "mr_combine_device")

    def combine_all(self, alpha: float, ibm_percentage: float, ibm_probability: float, ubm_ptr: int, ibm_ptr: int,
                    out_ptrs: Tuple[int, int, int], *, seed: int = 0, pair_base: int = 0,
                    n_pairs: int = 0) -> Tuple[Tuple[float, float], Tuple[float, float], Tuple[float, float]]:
        """The linear, aggregation and stochastic combinations in one pass
        (mr_combine_all_device), each bit-equal to combine(); returns each
        output's (min, max) over its pairs; synchronous."""
        mm = (ctypes.c_double * 6)()
        _lib.check(self._L.mr_combine_all_device(self._h, float(alpha), float(ibm_percentage), float(ibm_probability),
                                                 int(seed) & (2 ** 64 - 1), int(pair_base), int(n_pairs),
                                                 ctypes.c_void_p(ubm_ptr), ctypes.c_void_p(ibm_ptr),
                                                 *(ctypes.c_void_p(x) for x in out_ptrs), mm),
                   "mr_combine_all_device")
        return (mm[0], mm[1]), (mm[2], mm[3]), (mm[4], mm[5])

    def dense_minmax(self) -> Optional[Tuple[float, float]]:
        """(min, max) of the last run's dense model from the scoring kernels
        (mr_dense_minmax), or None when the last run did not compute it."""
        mn, mx = ctypes.c_double(), ctypes.c_double()
        if self._L.mr_dense_minmax(self._h, ctypes.byref(mn), ctypes.byref(mx)) != 0:
            return None
        return mn.value, mx.value

    def eval_minmax(self, dense_ptr: int) -> Tuple[float, float]:
        mn, mx = ctypes.c_double(), ctypes.c_double()
        _lib.check(self._L.mr_eval_minmax_device(self._h, ctypes.c_void_p(dense_ptr), ctypes.byref(mn),
                                                 ctypes.byref(mx)), "mr_eval_minmax_device")
        return mn.value, mx.value

    def eval_counts(self, dense_ptr: int, mn: float, mx: float, lab_off: np.ndarray,
                    lab_songs: np.ndarray, pred: Optional[np.ndarray] = None,
                    tp: Optional[np.ndarray] = None, n_thresholds: int = 10) -> Tuple[np.ndarray, np.ndarray]:
        """(pred, tp) counts, each width x n_thresholds int32 (MR:529, MR:541-553;
        10 thresholds = MR:590, 11 = distributed.scala:395); pred / tp may be
        caller-owned (e.g. pinned) C-contiguous int32 arrays of that shape."""
        lab_off = np.ascontiguousarray(lab_off, dtype=np.int64)
        lab_songs = np.ascontiguousarray(lab_songs, dtype=np.int32)
        shape = (self.width, n_thresholds)
        for a in (pred, tp):
            if a is not None and (a.dtype != np.int32 or a.shape != shape or not a.flags.c_contiguous):
                raise ValueError(f"pred / tp must be C-contiguous int32 arrays of shape {shape}")
        pred = np.empty(shape, dtype=np.int32) if pred is None else pred
        tp = np.empty(shape, dtype=np.int32) if tp is None else tp
        _lib.check(self._L.mr_eval_counts_device(
            self._h, ctypes.c_void_p(dense_ptr), float(mn), float(mx), lab_off.ctypes.data_as(ctypes.c_void_p),
            lab_songs.ctypes.data_as(ctypes.c_void_p), pred.ctypes.data_as(ctypes.c_void_p),
            tp.ctypes.data_as(ctypes.c_void_p), int(n_thresholds)), "mr_eval_counts_device")
        return pred, tp

    def eval_map(self, dense_ptr: int, mn: float, mx: float, lab_off: np.ndarray, lab_songs: np.ndarray,
                 pos: np.ndarray, n_label_songs: int, n_thresholds: int = 10) -> float:
        """Threshold mAP with counts and per-class AP on the device
        (mr_eval_map_device; the context must hold every test user)."""
        lab_off = np.ascontiguousarray(lab_off, dtype=np.int64)
        lab_songs = np.ascontiguousarray(lab_songs, dtype=np.int32)
        pos = np.ascontiguousarray(pos, dtype=np.int32)
        if pos.shape[0] < self.song_hi:
            raise ValueError("pos must cover the shard's songs")
        out = ctypes.c_double()
        _lib.check(self._L.mr_eval_map_device(
            self._h, ctypes.c_void_p(dense_ptr), float(mn), float(mx), lab_off.ctypes.data_as(ctypes.c_void_p),
            lab_songs.ctypes.data_as(ctypes.c_void_p), pos.ctypes.data_as(ctypes.c_void_p), int(n_label_songs),
            ctypes.byref(out), int(n_thresholds)), "mr_eval_map_device")
        return out.value

    def eval_class_counts(self, dense_ptrs, mins, maxs, lab_off: np.ndarray, lab_songs: np.ndarray,
                          classes: np.ndarray, counts_ptr: int, n_thresholds: int = 10) -> None:
        """The label classes' (pred, tp) counts of several dense device models
        into one device buffer of len(dense_ptrs) x 2 x len(classes) x
        n_thresholds int32 (mr_eval_class_counts_device; classes: ascending
        global song ids, shared by every rank; 0 for classes outside this
        context's songs; mins / maxs: each model's global extremes), ready for
        ONE SUM all-reduce."""
        n = len(dense_ptrs)
        ptrs = (ctypes.c_void_p * n)(*[ctypes.c_void_p(p) for p in dense_ptrs])
        mn = np.ascontiguousarray(mins, dtype=np.float64)
        mx = np.ascontiguousarray(maxs, dtype=np.float64)
        lab_off = np.ascontiguousarray(lab_off, dtype=np.int64)
        lab_songs = np.ascontiguousarray(lab_songs, dtype=np.int32)
        classes = np.ascontiguousarray(classes, dtype=np.int32)
        _lib.check(self._L.mr_eval_class_counts_device(
            self._h, n, ptrs, mn.ctypes.data_as(ctypes.c_void_p), mx.ctypes.data_as(ctypes.c_void_p),
            lab_off.ctypes.data_as(ctypes.c_void_p), lab_songs.ctypes.data_as(ctypes.c_void_p), int(classes.shape[0]),
            classes.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(counts_ptr), int(n_thresholds)),
            "mr_eval_class_counts_device")

    def eval_map_counts(self, n_models: int, counts_ptr: int, class_pos: np.ndarray, n_label_songs: int,
                        n_thresholds: int = 10) -> list:
        """Each model's mAP from a (reduced) class-count device buffer
        (mr_eval_map_counts_device)."""
        class_pos = np.ascontiguousarray(class_pos, dtype=np.int32)
        out = np.empty(int(n_models), dtype=np.float64)
        _lib.check(self._L.mr_eval_map_counts_device(
            self._h, int(n_models), int(class_pos.shape[0]), class_pos.ctypes.data_as(ctypes.c_void_p),
            ctypes.c_void_p(counts_ptr), int(n_label_songs), out.ctypes.data_as(ctypes.c_void_p), int(n_thresholds)),
            "mr_eval_map_counts_device")
        return out.tolist()

    def timing_begin(self) -> None:
        """Open a timing window (one event on the engine stream)."""
        _lib.check(self._L.mr_timing_begin(self._h), "mr_timing_begin")

    def timing_stop(self) -> None:
        """Record the window's closing event without waiting (read it with timing_end)."""
        _lib.check(self._L.mr_timing_stop(self._h), "mr_timing_stop")

    def timing_end(self) -> Tuple[int, float]:
        """Close the window: (scoring-kernel launches, device ms) since timing_begin."""
        n = ctypes.c_int64()
        ms = ctypes.c_double()
        _lib.check(self._L.mr_timing_end(self._h, ctypes.byref(n), ctypes.byref(ms)), "mr_timing_end")
        return n.value, ms.value

    def kernel_times(self, kernel: Union[str, int], reset: bool = False) -> Tuple[int, float]:
        n = ctypes.c_int64()
        ms = ctypes.c_double()
        which = KERNELS[kernel] if isinstance(kernel, str) else kernel
        _lib.check(self._L.mr_kernel_times(self._h, which, ctypes.byref(n), ctypes.byref(ms), 1 if reset else 0),
                   "mr_kernel_times")
        return n.value, ms.value


def merge_topk_host(songs: np.ndarray, keys: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Merge [n_shards][n_test][k] per-shard lists (song ids global) -> n_test x k
    by (key desc, song asc): the exchange step of a song-sharded run, host side."""
    L = _lib.lib()
    songs = np.ascontiguousarray(songs, dtype=np.int32)
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    g, n_te, k = songs.shape
    os_ = np.empty((n_te, k), dtype=np.int32)
    ok = np.empty((n_te, k), dtype=np.int64)
    osc = np.empty((n_te, k), dtype=np.float64)
    _lib.check(L.mr_topk_merge_host(g, n_te, k, songs.ctypes.data_as(ctypes.c_void_p),
                                    keys.ctypes.data_as(ctypes.c_void_p), None,
                                    os_.ctypes.data_as(ctypes.c_void_p), ok.ctypes.data_as(ctypes.c_void_p),
                                    osc.ctypes.data_as(ctypes.c_void_p)), "mr_topk_merge_host")
    return os_, osc, ok
