"""The C-ABI library: loads, exports every symbol include/mr_engine.h declares,
host-only entry points behave, and without a GPU the compute entry points fail
with an error code (never a crash or a silent CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from musicrecommendation_amd import _lib
from musicrecommendation_amd.engine import Engine, merge_topk_host

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "mr_engine.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mr_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(names)


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_lib.MrDataset) == 4 * 4 + 7 * 8
    assert ctypes.sizeof(_lib.MrOptions) == 16 * 4


def test_options_default_and_version():
    L = _lib.lib()
    o = _lib.MrOptions()
    assert L.mr_options_default(ctypes.byref(o)) == 0
    assert (o.frac_bits, o.topk, o.dense, o.out_dtype) == (32, 10, 1, _lib.MR_OUT_F32)
    assert b"gfx950" in L.mr_version()
    assert L.mr_options_default(None) == _lib.MR_E_INVALID
    assert L.mr_last_error()


def test_host_merge_orders_by_key_then_song():
    # two shards, one user, k = 3; keys are double bit patterns
    def key(x):
        return np.array([x], dtype=np.float64).view(np.int64)[0]
    songs = np.array([[[5, 9, -1]], [[2, 7, 8]]], dtype=np.int32)
    keys = np.array([[[key(0.5), key(0.25), -1]], [[key(0.5), key(0.3), key(0.1)]]], dtype=np.int64)
    s, sc, k = merge_topk_host(songs, keys)
    assert s.tolist() == [[2, 5, 7]]                  # tie at 0.5 -> lower song id first
    assert sc.tolist() == [[0.5, 0.5, 0.3]]
    s, sc, k = merge_topk_host(songs[:1, :, :1].copy(), keys[:1, :, :1].copy())
    assert s.tolist() == [[5]]


def test_host_merge_pads_missing_entries():
    songs = np.full((2, 1, 4), -1, dtype=np.int32)
    keys = np.full((2, 1, 4), -1, dtype=np.int64)
    songs[1, 0, 0], keys[1, 0, 0] = 3, 0
    s, sc, k = merge_topk_host(songs, keys)
    assert s.tolist() == [[3, -1, -1, -1]] and k.tolist() == [[0, -1, -1, -1]]
    assert np.isnan(sc[0, 1:]).all()


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU error path")
def test_no_gpu_is_an_error_code_not_a_fallback():
    from helpers import kat, dataset_from_lines

    K = kat()
    ds = dataset_from_lines(K["train"], K["test"], K["labels"])
    with pytest.raises(_lib.EngineError) as ei:
        Engine(ds)
    assert ei.value.code in (_lib.MR_E_HIP, _lib.MR_E_INVALID)


def test_null_arguments_are_rejected():
    L = _lib.lib()
    assert L.mr_load(None, None) == _lib.MR_E_INVALID
    assert L.mr_run(None, 0) == _lib.MR_E_INVALID
    assert L.mr_destroy(None) == _lib.MR_OK
    assert L.mr_topk_merge_host(1, 1, 1, None, None, None, None, None, None) == _lib.MR_E_INVALID
