"""Combination models and the reference's threshold mAP on the device.

The reference builds three ensembles from the sorted ubm / ibm arrays
(main.scala:57-59, MusicRecommender.scala MR:317-481) and scores every model
with the threshold mAP of MR:521-639. Here both models stay on the GPU as
dense [n_test x width] buffers (NaN = no pair); the combination, the min/max,
the per-class confusion counts and the top-k run as HIP kernels
(csrc/mr_ensemble.hip, csrc/mr_engine.hip k_topk_dense); the AP/mAP fold runs
on the host over the integer counts (mr_eval_map).

Multi-GPU: every rank holds one engine context (a song shard or a block of
test users). threshold_map all-reduces min/max (MIN/MAX) and the counts
(SUM) into a full n_songs x 10 table per model; threshold_maps does several
models at once with one MAX all-reduce of their (-min, max) and one SUM
all-reduce of a class-indexed count block built and folded on the device
(mr_eval_class_counts_device / mr_eval_map_counts_device). Either way every
rank computes the same mAP, bit for bit, for any layout.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from .engine import Engine

LINEAR, AGGREGATION, STOCHASTIC = _lib.MR_COMB_LINEAR, _lib.MR_COMB_AGGREGATION, _lib.MR_COMB_STOCHASTIC
_MASK = 2 ** 64 - 1


def pair_uniform(seed: int, idx: int) -> float:
    """The stochastic model's draw for pair `idx` (as mr_combine_device):
    24 bits of splitmix64(seed + (idx+1)·0x9E3779B97F4A7C15) / 2^24 — the
    distribution of java.util.Random.nextFloat (MR:414), seeded and
    independent of launch geometry."""
    z = (seed + (idx + 1) * 0x9E3779B97F4A7C15) & _MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK
    z ^= z >> 31
    return float(np.float32(z >> 40) * np.float32(1.0 / 16777216.0))


def eval_map(pred: np.ndarray, tp: np.ndarray, pos: np.ndarray, n_label_songs: int) -> float:
    """mAP from the per-class counts (mr_eval_map, MR:588-627; the threshold
    count is pred.shape[1]: 10 = MR:590, 11 = distributed.scala:395)."""
    pred = np.ascontiguousarray(pred, dtype=np.int32)
    tp = np.ascontiguousarray(tp, dtype=np.int32)
    pos = np.ascontiguousarray(pos, dtype=np.int32)
    out = ctypes.c_double()
    _lib.check(_lib.lib().mr_eval_map(pred.shape[0], pred.ctypes.data_as(ctypes.c_void_p),
                                      tp.ctypes.data_as(ctypes.c_void_p), pos.ctypes.data_as(ctypes.c_void_p),
                                      int(n_label_songs), ctypes.byref(out), int(pred.shape[1])), "mr_eval_map")
    return out.value


class DeviceEnsemble:
    """Dense models of one engine context as torch device tensors.

    pair_base / n_pairs place this context's pairs in the full model's
    (user, song) order (aggregation threshold and stochastic draws); pos /
    n_label_songs are the GLOBAL per-class label counts (defaults: this
    context's dataset, i.e. a single-process run)."""

    def __init__(self, engine: Engine, *, pair_base: int = 0, n_pairs: Optional[int] = None,
                 pos: Optional[np.ndarray] = None, n_label_songs: Optional[int] = None, group=None,
                 collectives: Optional[bool] = None):
        import torch

        from . import evaluation

        self.e = engine
        self.ds = engine.dataset
        # (host stand-ins of the CPU tests: torch's CPU device)
        self.device = torch.device("cuda", engine.opt.device) if torch.cuda.is_available() else torch.device("cpu")
        self.torch_dtype = torch.float64 if engine.dtype == np.float64 else torch.float32
        self.shape = (engine.n_test, engine.width)
        self.pair_base = int(pair_base)
        self.n_pairs = int(n_pairs if n_pairs is not None else self.ds.n_pairs())
        self.pos = evaluation.label_pos(self.ds) if pos is None else np.asarray(pos, dtype=np.int32)
        self.n_label_songs = int(self.ds.n_label_songs if n_label_songs is None else n_label_songs)
        self.group = group
        # None: the MIN/MAX/SUM reductions run when the process group has more
        # than one rank; True: always (a one-rank RCCL rehearsal of that path)
        self.collectives = collectives
        self._host = None  # pinned (pred, tp) count buffers of threshold_map

    def empty(self):
        import torch

        return torch.empty(self.shape, dtype=self.torch_dtype, device=self.device)

    def _after_torch(self) -> None:
        """Order the engine's own HIP stream after everything queued so far on
        torch's current stream (an event + hipStreamWaitEvent, no host wait):
        inputs produced by pending torch kernels are complete and recycled
        output allocations are no longer in use when the engine touches them.
        Every engine call below returns after its stream has drained, so torch
        may use the outputs right away."""
        import torch

        if not torch.cuda.is_available():  # host stand-ins of the gloo tests: nothing queued
            return
        ext = torch.cuda.ExternalStream(self.e.stream, device=self.device)
        ext.wait_stream(torch.cuda.current_stream(self.device))

    # ---- models ----------------------------------------------------------------
    def model(self, name: str):
        """ubm / ibm dense model (MR:132-307) into a new device tensor."""
        t = self.empty()
        self._after_torch()
        self.e.run_into(name, t.data_ptr())
        self.e.sync()
        mm = self.e.dense_minmax()  # the scoring kernels' min / max (wide shape), for threshold_map
        if mm is not None:
            t._mr_minmax = (t._version, mm[0], mm[1])
        return t

    def _combine(self, kind: int, ubm, ibm, param: float, seed: int = 0):
        out = self.empty()
        self._after_torch()
        self.e.combine(kind, param, ubm.data_ptr(), ibm.data_ptr(), out.data_ptr(), seed=seed,
                       pair_base=self.pair_base, n_pairs=self.n_pairs)
        return out

    def linear(self, ubm, ibm, alpha: float):
        """getLinearCombinationModel (MR:317-351)."""
        return self._combine(LINEAR, ubm, ibm, alpha)

    def aggregation(self, ubm, ibm, item_based_percentage: float = 0.5):
        """getAggregationModel (MR:361-418)."""
        return self._combine(AGGREGATION, ubm, ibm, item_based_percentage)

    def stochastic(self, ubm, ibm, item_based_probability: float = 0.5, seed: int = 0):
        """getStochasticCombinationModel (MR:429-481), seeded."""
        return self._combine(STOCHASTIC, ubm, ibm, item_based_probability, seed)

    def combinations(self, ubm, ibm, alpha: float = 0.5, item_based_percentage: float = 0.5,
                     item_based_probability: float = 0.5, seed: int = 0):
        """The driver's three combinations (main.scala:57-89: linear, aggregation,
        stochastic) in one pass over ubm and ibm (mr_combine_all_device), each
        bit-equal to linear() / aggregation() / stochastic(). Each output keeps
        its min / max from the same pass for threshold_map, valid while the
        tensor is unmodified (torch's version counter)."""
        outs = (self.empty(), self.empty(), self.empty())
        self._after_torch()
        mms = self.e.combine_all(alpha, item_based_percentage, item_based_probability, ubm.data_ptr(),
                                 ibm.data_ptr(), tuple(t.data_ptr() for t in outs), seed=seed,
                                 pair_base=self.pair_base, n_pairs=self.n_pairs)
        for t, mm in zip(outs, mms):
            t._mr_minmax = (t._version, mm[0], mm[1])
        return outs

    def _minmax(self, t) -> Tuple[float, float]:
        """Global min / max of a dense model (MR:524-525). The value carried by
        the producing pass (model / combinations) is reused while torch's
        version counter of `t` is unchanged: the cache assumes only torch
        mutates the tensor — a write through its data_ptr from outside torch
        (an engine call, DLPack) must be followed by t.add_(0) or a fresh
        tensor, or the stale min / max is used. Otherwise the engine's min/max
        kernel reads `t`, ordered after torch's pending work on it."""
        cached = getattr(t, "_mr_minmax", None)
        if cached is not None and cached[0] == t._version:  # from the producing pass, tensor unchanged
            return cached[1], cached[2]
        self._after_torch()  # e.g. an in-place torch op on t still running on torch's stream
        return self.e.eval_minmax(t.data_ptr())

    # ---- evaluation --------------------------------------------------------------
    def _world(self) -> int:
        import torch.distributed as dist

        return dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1

    def _reduce(self) -> bool:
        """Whether threshold_map all-reduces (more than one rank, or forced)."""
        return self._world() > 1 or (bool(self.collectives) and self._pg())

    @staticmethod
    def _pg() -> bool:
        import torch.distributed as dist

        return dist.is_available() and dist.is_initialized()

    def threshold_map(self, t, n_thresholds: int = 10) -> float:
        """evaluateModel (MR:636) of a dense device model; n_thresholds = 11 is
        the distributed evaluation (distributed.scala:395)."""
        import torch
        import torch.distributed as dist

        self._after_torch()
        mn, mx = self._minmax(t)
        world = self._world()
        reduce = self._reduce()
        if reduce:
            be = dist.get_backend(self.group)
            dev = self.device if be == "nccl" else torch.device("cpu")
            a = torch.tensor([mn], dtype=torch.float64, device=dev)
            b = torch.tensor([mx], dtype=torch.float64, device=dev)
            dist.all_reduce(a, op=dist.ReduceOp.MIN, group=self.group)
            dist.all_reduce(b, op=dist.ReduceOp.MAX, group=self.group)
            mn, mx = float(a.item()), float(b.item())
        if not (mn <= mx):
            raise ValueError("model has no pairs: min/max undefined (the reference throws here, MR:524)")
        if not reduce and world == 1 and self.e.song_lo == 0 and self.e.song_hi == self.ds.n_songs and hasattr(self.e, "eval_map"):
            # one context holds the whole model: counts, AP per class on the device
            return self.e.eval_map(t.data_ptr(), mn, mx, self.ds.lab_off, self.ds.lab_songs, self.pos,
                                   self.n_label_songs, n_thresholds=n_thresholds)
        if (self._host is None or self._host[0].shape[1] != n_thresholds) and torch.cuda.is_available():
            # pinned, reused: no page faults per call
            self._host = [torch.empty((self.e.width, n_thresholds), dtype=torch.int32, pin_memory=True).numpy()
                          for _ in range(2)]
        bufs = {} if self._host is None else {"pred": self._host[0], "tp": self._host[1]}
        pred, tp = self.e.eval_counts(t.data_ptr(), mn, mx, self.ds.lab_off, self.ds.lab_songs,
                                      n_thresholds=n_thresholds, **bufs)
        if self.e.song_lo == 0 and self.e.song_hi == self.ds.n_songs:
            full_p, full_t = pred, tp
        else:
            full_p = np.zeros((self.ds.n_songs, n_thresholds), dtype=np.int32)
            full_t = np.zeros_like(full_p)
            full_p[self.e.song_lo:self.e.song_hi] = pred
            full_t[self.e.song_lo:self.e.song_hi] = tp
        if reduce:
            be = dist.get_backend(self.group)
            dev = self.device if be == "nccl" else torch.device("cpu")
            c = torch.from_numpy(np.stack([full_p, full_t])).to(dev)
            dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
            c = c.cpu().numpy()
            full_p, full_t = c[0], c[1]
        return eval_map(full_p, full_t, self.pos, self.n_label_songs)

    def _classes(self) -> Tuple[np.ndarray, np.ndarray]:
        """The label classes every rank shares: ascending song ids with a label
        (pos > 0; label-only songs are never predicted) and their label counts."""
        if getattr(self, "_cls", None) is None:
            cls = np.nonzero(self.pos > 0)[0].astype(np.int32)
            self._cls = (cls, self.pos[cls].astype(np.int32))
        return self._cls

    def threshold_maps(self, models: dict, n_thresholds: int = 10) -> dict:
        """evaluateModel (MR:636) of several dense device models, {name: mAP}.
        One rank: threshold_map each (counts and AP on the device). Several
        ranks (song shards, test-user blocks or both): ONE MAX all-reduce of
        every model's (-min, max); the label classes' counts of every model into
        one device block (mr_eval_class_counts_device, laid out by the global
        class list, so any layout sums alike); ONE SUM all-reduce of that block
        (RCCL; on a gloo group through the host); the AP per class on the device
        (mr_eval_map_counts_device). Only the per-class AP crosses PCIe —
        instead of every model's full [songs x thresholds] count tables down,
        reduced and back per model. Bit-equal to threshold_map per model."""
        import torch
        import torch.distributed as dist

        if not self._reduce():
            return {n: self.threshold_map(t, n_thresholds) for n, t in models.items()}
        names = list(models)
        be = dist.get_backend(self.group)
        host = be != "nccl"
        dev = torch.device("cpu") if host else self.device
        mm = []
        for n in names:
            mn, mx = self._minmax(models[n])
            mm += [-mn, mx]
        mmt = torch.tensor(mm, dtype=torch.float64, device=dev)
        dist.all_reduce(mmt, op=dist.ReduceOp.MAX, group=self.group)
        mmv = mmt.cpu().tolist()
        mins, maxs = [-x for x in mmv[0::2]], mmv[1::2]
        for mn, mx in zip(mins, maxs):
            if not (mn <= mx):
                raise ValueError("model has no pairs: min/max undefined (the reference throws here, MR:524)")
        cls, cpos = self._classes()
        cdev = self.device if torch.cuda.is_available() else torch.device("cpu")
        counts = torch.empty((len(names), 2, cls.shape[0], n_thresholds), dtype=torch.int32, device=cdev)
        self._after_torch()
        self.e.eval_class_counts([models[n].data_ptr() for n in names], mins, maxs, self.ds.lab_off,
                                 self.ds.lab_songs, cls, counts.data_ptr(), n_thresholds=n_thresholds)
        red = counts.cpu() if host and counts.is_cuda else counts
        dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group)
        if red is not counts:
            counts.copy_(red)
        self._after_torch()  # the reduced block, written on torch's stream
        maps = self.e.eval_map_counts(len(names), counts.data_ptr(), cpos, self.n_label_songs,
                                      n_thresholds=n_thresholds)
        return dict(zip(names, maps))

    def topk(self, t) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Top-k recommendation lists of a dense device model (k = engine topk)."""
        self._after_torch()
        self.e.topk_dense(t.data_ptr())
        return self.e.topk()
