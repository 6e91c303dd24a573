"""The fused kernel's in-launch hand-off (tile candidates -> the user's last
workgroup, sc1 stores + agent-scope counter; MI355X_MICROARCH.md asks to test
hand-offs under UNEVEN load): many back-to-back launches while a second
context streams a large wide-shape job on its own stream, every result
checked against the fixed-point oracle."""
import numpy as np
import pytest

from musicrecommendation_amd import synth
from musicrecommendation_amd.engine import Engine
from oracle import native

pytestmark = pytest.mark.gpu


def test_fused_handoff_under_uneven_load():
    ds = synth.config("c2", n_test=40).dataset()
    _, ts, tk = native.fp_model(ds, "ibm", k=10, dense=False)
    big = synth.config("c3", n_test=300).dataset()
    with Engine(ds, topk=10, dense=True) as e, Engine(big, topk=10, dense=False) as noisy:
        assert e.shape == "fused" and e.n_tiles > 1
        for rnd in range(30):
            noisy.run("ibm")          # a long wide-shape job on the other stream
            for _ in range(10):
                e.run("ibm")          # back-to-back fused launches: counters self-reset
            s, _sc, k = e.topk()      # synchronises this context only
            assert np.array_equal(s, ts), rnd
            assert np.array_equal(k, tk), rnd
        noisy.sync()
