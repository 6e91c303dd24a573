"""Host-side mirror of the reference class ``MusicRecommender``
(src/main/scala/music_recommandation/MusicRecommender.scala, MR:12).

Same constructor inputs (train, test and test-labels triplet sources, MR:12),
same public method names and result shape — ``Array[(user, (song, score))]``
for every (test user, unheard song) pair — so a caller of the reference can
switch over. The scoring runs on the MI355X engine (one batched call per
model instead of one closure call per pair, MR:105-125); the ingest runs in
the native C++ TSV reader (MR:26-91).

Emission order: the reference emits s-major, u-minor in JVM HashSet order
(MR:105-111), which no other runtime reproduces; we emit s-major, u-minor in
lexicographic id order. The driver sorts both by (user, song, -score)
anyway (main.scala:57-59); ``sorted_model`` gives that order directly.
The ``*P`` variants exist for API parity; on the GPU both are the parallel path.
"""
from __future__ import annotations

import os
import tempfile
from typing import Iterable, List, Optional, Tuple, Union

import numpy as np

from .dataset import Dataset
from .engine import Engine
from . import evaluation

Model = List[Tuple[str, Tuple[str, float]]]
Source = Union[str, os.PathLike, Iterable[str]]


def _as_path(src: Source, tmpdir: str, name: str) -> str:
    """A path is used as is (and must exist: the reference's Source.fromFile
    throws FileNotFoundException); any other iterable is a source of lines."""
    if isinstance(src, (str, bytes, os.PathLike)):
        if not os.path.exists(src):
            raise FileNotFoundError(f"{os.fsdecode(src)}: no such file")
        return os.fsdecode(src)
    path = os.path.join(tmpdir, name)
    with open(path, "w") as f:
        for line in src:  # a BufferedSource-like iterable of lines
            f.write(line if line.endswith("\n") else line + "\n")
    return path


class MusicRecommender:
    def __init__(self, trainFile: Source, testFile: Source, testLabelsFile: Source, *, device: int = 0,
                 out_dtype: str = "f64", topk: int = 10):
        with tempfile.TemporaryDirectory() as td:
            self.dataset = Dataset.from_tsv(_as_path(trainFile, td, "train.txt"),
                                            _as_path(testFile, td, "test.txt"),
                                            _as_path(testLabelsFile, td, "labels.txt"))
        self._device = device
        self._out_dtype = out_dtype
        self._topk = topk
        self._engine: Optional[Engine] = None

    # ---- engine ------------------------------------------------------------
    def engine(self) -> Engine:
        if self._engine is None:
            self._engine = Engine(self.dataset, device=self._device, out_dtype=self._out_dtype, topk=self._topk)
        return self._engine

    def scores(self, model: str) -> np.ndarray:
        """Dense n_test x n_songs scores (NaN for heard songs)."""
        return self.engine().score_dense(model)

    def recommendations(self, model: str) -> Tuple[np.ndarray, np.ndarray]:
        """Per test user, the top-k (song ids, scores) by (score desc, song asc)."""
        e = self.engine()
        e.run(model)
        songs, scores, _keys = e.topk()
        return songs, scores

    def _to_model(self, dense: np.ndarray) -> Model:
        """Pair list in getModel's emission order: s-major, u-minor
        (MR:106-108), heard songs (NaN) emit no pair (MR:109). Vectorised:
        one nonzero over the transposed mask, names gathered as object arrays."""
        ds = self.dataset
        s_idx, u_idx = np.nonzero(~np.isnan(dense.T))
        users = np.array([ds.test_names(u) for u in range(ds.n_test)], dtype=object)
        songs = np.array([ds.song_names(s) for s in range(ds.n_songs)], dtype=object)
        vals = dense[u_idx, s_idx].astype(np.float64).tolist()
        return list(zip(users[u_idx].tolist(), zip(songs[s_idx].tolist(), vals)))

    # ---- reference API (MR:132-307) -------------------------------------------
    def getUserBasedModel(self) -> Model:
        return self._to_model(self.scores("ubm"))

    def getUserBasedModelP(self) -> Model:
        return self.getUserBasedModel()

    def getItemBasedModel(self) -> Model:
        return self._to_model(self.scores("ibm"))

    def getItemBasedModelP(self) -> Model:
        return self.getItemBasedModel()

    @staticmethod
    def sorted_model(model: Model) -> Model:
        """main.scala:57-59 ordering: (user, song, -score)."""
        return sorted(model, key=lambda t: (t[0], t[1][0], -t[1][1]))

    # ---- combination models (MR:317-481) ------------------------------------------
    # Over the Model arrays, in the order given (the driver passes them sorted
    # by (user, song), main.scala:57-59). Mismatched pairs: the reference calls
    # System.exit(2) (MR:326); a bad percentage: System.exit(-1) (MR:366-369).
    # Both raise ValueError here. On-device versions over dense models:
    # ensemble.DeviceEnsemble (the C5 path).
    @staticmethod
    def _zip(ubm: Model, ibm: Model):
        if len(ubm) != len(ibm):
            raise ValueError("ubm and ibm differ in length (reference: System.exit(2), MR:326)")
        for (u1, (s1, r1)), (u2, (s2, r2)) in zip(ubm, ibm):
            if u1 != u2 or s1 != s2:
                raise ValueError(f"pair mismatch ({u1},{s1}) vs ({u2},{s2}) (reference: System.exit(2), MR:326)")
            yield u1, s1, r1, r2

    @staticmethod
    def _check_fraction(x: float, what: str) -> None:
        if x < 0 or x > 1:
            raise ValueError(f"{what} must be between 0 and 1 (reference: System.exit(-1), MR:366-369)")

    def getLinearCombinationModel(self, ubm: Model, ibm: Model, alpha: float) -> Model:
        return [(u, (s, r1 * alpha + r2 * (1 - alpha))) for u, s, r1, r2 in self._zip(ubm, ibm)]

    def getLinearCombinationModelP(self, ubm: Model, ibm: Model, alpha: float) -> Model:
        return self.getLinearCombinationModel(ubm, ibm, alpha)

    def getAggregationModel(self, ubm: Model, ibm: Model, itemBasedPercentage: float = 0.5) -> Model:
        self._check_fraction(itemBasedPercentage, "Percentage")
        threshold = int(itemBasedPercentage * len(ubm))
        return [(u, (s, r2 if i < threshold else r1)) for i, (u, s, r1, r2) in enumerate(self._zip(ubm, ibm))]

    def getAggregationModelP(self, ubm: Model, ibm: Model, itemBasedPercentage: float = 0.5) -> Model:
        return self.getAggregationModel(ubm, ibm, itemBasedPercentage)

    def getStochasticCombinationModel(self, ubm: Model, ibm: Model, itemBasedProbability: float = 0.5,
                                      seed: int = 0) -> Model:
        """The reference draws from an unseeded java.util.Random (MR:439); here
        the draw of the i-th pair is ensemble.pair_uniform(seed, i), the stream
        the device kernel uses, so list and device results agree."""
        from .ensemble import pair_uniform

        self._check_fraction(itemBasedProbability, "Probability")
        return [(u, (s, r2 if pair_uniform(seed, i) < itemBasedProbability else r1))
                for i, (u, s, r1, r2) in enumerate(self._zip(ubm, ibm))]

    def getStochasticCombinationModelP(self, ubm: Model, ibm: Model, itemBasedProbability: float = 0.5,
                                       seed: int = 0) -> Model:
        return self.getStochasticCombinationModel(ubm, ibm, itemBasedProbability, seed)

    # ---- model files (MR:489-512) --------------------------------------------------
    @staticmethod
    def writeModelOnFile(model: Model, outputFileName: str) -> None:
        """One "user\tsong\tscore" line per element, in the given order, the
        score as java.lang.Double.toString (MR:489-497)."""
        from .modelio import java_double_string

        with open(outputFileName, "w") as f:
            for u, (s, x) in model:
                f.write(f"{u}\t{s}\t{java_double_string(x)}\n")

    @staticmethod
    def importModelFromFile(pathToModel: str):
        """(user, song, score) triplets sorted by (user, song, -score) (MR:505-512)."""
        from .modelio import import_model

        return import_model(pathToModel)

    # ---- evaluation (MR:636-639) ------------------------------------------------
    def evaluateModel(self, model: Union[Model, np.ndarray], parallel: bool = False) -> float:
        """Threshold mAP (MR:636) on the device: the model goes to HBM as a
        dense buffer, min/max + confusion counts run as HIP kernels."""
        import torch

        from .ensemble import DeviceEnsemble

        dense = model if isinstance(model, np.ndarray) else self._from_model(model)
        eng = self.engine()
        ens = DeviceEnsemble(eng)
        t = torch.from_numpy(np.ascontiguousarray(dense, dtype=eng.dtype)).to(ens.device)
        torch.cuda.synchronize(ens.device)
        return ens.threshold_map(t)

    def _from_model(self, model: Model) -> np.ndarray:
        ds = self.dataset
        sidx = {ds.song_names(i): i for i in range(ds.n_songs)}
        uidx = {ds.test_names(i): i for i in range(ds.n_test)}
        dense = np.full((ds.n_test, ds.n_songs), np.nan)
        for u, (s, x) in model:
            dense[uidx[u], sidx[s]] = x
        return dense

    def close(self) -> None:
        if self._engine is not None:
            self._engine.close()
            self._engine = None
