"""mr_graph_capture / mr_graph_launch: n back-to-back steps of one context
replayed as one HIP graph give the same outputs as stream launches (the fused
hand-off counters self-reset between the captured launches; the wide shape's
three kernels per batch capture in order), and the API's error behaviour."""
import numpy as np
import pytest

from musicrecommendation_amd import _lib, synth
from musicrecommendation_amd.engine import Engine
from oracle import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n_test,stage1", [("c2", 10, "auto"), ("c2", 40, "auto"), ("c3", 64, "wide"),
                                               ("c2", 24, "separate")])
def test_graph_replay_equals_oracle(cfg, n_test, stage1):
    ds = synth.config(cfg, n_test=n_test).dataset()
    for model in ("ibm", "ubm"):
        _, ts, tk = native.fp_model(ds, model, k=10, dense=False)
        with Engine(ds, topk=10, dense=True, stage1=stage1) as e:
            e.run(model)
            d_ref = e.dense()
            e.graph_capture(model, 7)
            for _ in range(3):
                e.graph_launch()
            s, _sc, k = e.topk()
            assert np.array_equal(s, ts) and np.array_equal(k, tk), (cfg, stage1, model)
            assert np.array_equal(e.dense(), d_ref, equal_nan=True), (cfg, stage1, model)


def test_graph_errors():
    ds = synth.config("c2", n_test=10).dataset()
    with Engine(ds, topk=10) as e:
        with pytest.raises(_lib.EngineError):
            e.graph_launch()            # nothing captured
        with pytest.raises(_lib.EngineError):
            e.graph_capture("ibm", 0)
        e.graph_capture("ibm", 2)
        e.graph_capture("ubm", 3)       # replaces the first graph
        e.graph_launch()
        e.sync()
    with Engine(ds, topk=10, time_kernels=True) as e:
        with pytest.raises(_lib.EngineError):
            e.graph_capture("ibm", 2)
