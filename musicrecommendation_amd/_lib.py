"""ctypes binding of the engine's C ABI (include/mr_engine.h).

The shared library ``libmr_engine.so`` is built in-tree by
``musicrecommendation_amd.build`` (``python -c "import __graft_entry__ as g; g.build()"``).
There is NO fallback: if the library is missing every entry point raises.

PyTorch bundles its own HIP runtime (same soname ``libamdhip64.so.7``). When
torch is importable we import it BEFORE loading the engine so that the
process holds exactly one HIP runtime (the engine then binds to torch's).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# MR_ENGINE_LIB=stamps selects the diagnostic build (per-workgroup phase timestamps).
_VARIANT = os.environ.get("MR_ENGINE_LIB", "")
LIB_PATH = os.path.join(_HERE, f"libmr_engine_{_VARIANT}.so" if _VARIANT else "libmr_engine.so")

MR_OK = 0
MR_E_INVALID = -1
MR_E_HIP = -2
MR_E_OOM = -3
MR_E_STATE = -4
MR_E_IO = -5
MR_E_PARSE = -6
MR_E_RCCL = -7
MR_TRANSPORT_AUTO, MR_TRANSPORT_COPY, MR_TRANSPORT_RCCL = 0, 1, 2
MR_UBM = 0
MR_IBM = 1
# mr_options.stage1 by name, and mr_launch_info's shape codes
STAGE1 = {"auto": 0, "fused": 1, "separate": 2, "wide": 4}
SHAPES = {0: "separate", 1: "fused", 3: "wide"}
MR_OUT_F32 = 0
MR_OUT_F64 = 1

_ERRNAMES = {
    MR_E_INVALID: "MR_E_INVALID",
    MR_E_HIP: "MR_E_HIP",
    MR_E_OOM: "MR_E_OOM",
    MR_E_STATE: "MR_E_STATE",
    MR_E_IO: "MR_E_IO",
    MR_E_PARSE: "MR_E_PARSE",
    MR_E_RCCL: "MR_E_RCCL",
}


class MrDataset(ctypes.Structure):
    _fields_ = [
        ("n_train_users", c_int32),
        ("n_test_users", c_int32),
        ("n_songs", c_int32),
        ("reserved0", c_int32),
        ("tr_off", POINTER(c_int64)),
        ("tr_songs", POINTER(c_int32)),
        ("te_off", POINTER(c_int64)),
        ("te_songs", POINTER(c_int32)),
        ("song_count", POINTER(c_int32)),
        ("tr_len", POINTER(c_int32)),
        ("te_len", POINTER(c_int32)),
    ]


class MrOptions(ctypes.Structure):
    _fields_ = [
        ("device", c_int32),
        ("frac_bits", c_int32),
        ("song_lo", c_int32),
        ("song_hi", c_int32),
        ("block_songs", c_int32),
        ("out_dtype", c_int32),
        ("topk", c_int32),
        ("dense", c_int32),
        ("time_kernels", c_int32),
        ("stage1", c_int32),
        ("stage1_chunk", c_int32),
        ("train_order", c_int32),
        ("topk_lists", c_int32),
        ("ibm_route", c_int32),
        ("reserved", c_int32 * 2),
    ]


class MrGroupOptions(ctypes.Structure):
    _fields_ = [
        ("n_song_shards", c_int32),
        ("n_user_blocks", c_int32),
        ("transport", c_int32),
        ("n_devices", c_int32),
        ("devices", POINTER(c_int32)),
    ]


class MrView(ctypes.Structure):
    _fields_ = [
        ("n_test_users", c_int32),
        ("n_songs", c_int32),
        ("song_lo", c_int32),
        ("song_hi", c_int32),
        ("out_dtype", c_int32),
        ("device", c_int32),
        ("te_off", c_void_p),
        ("te_songs", c_void_p),
        ("stream", c_void_p),
    ]


class MrCoocBytes(ctypes.Structure):
    """mr_cooc_bytes_t: encoding-independent byte counts of the co-listening route."""
    _fields_ = [(n, c_int64) for n in ("heavy_rows", "light_rows", "heavy_reads", "light_reads",
                                       "heavy_index_bytes", "light_index_bytes", "heavy_visits", "consumed_bytes",
                                       "group_tiles", "n_groups", "index_sparse_entries", "index_dense_songs",
                                       "consumed_sparse_entries", "consumed_dense_songs")]


MR_COMB_LINEAR = 0
MR_COMB_AGGREGATION = 1
MR_COMB_STOCHASTIC = 2


class EngineError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


# name -> (restype, argtypes); every symbol include/mr_engine.h declares.
SIGNATURES = {
    "mr_options_default": (c_int, [POINTER(MrOptions)]),
    "mr_create": (c_int, [POINTER(MrOptions), POINTER(c_void_p)]),
    "mr_destroy": (c_int, [c_void_p]),
    "mr_load": (c_int, [c_void_p, POINTER(MrDataset)]),
    "mr_shard_info": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "mr_launch_info": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "mr_batch_info": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "mr_route_info": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int64)]),
    "mr_topk_mode": (c_int, [c_void_p, POINTER(c_int32)]),
    "mr_cooc_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "mr_cooc_bytes": (c_int, [c_void_p, POINTER(MrCoocBytes)]),
    "mr_shard_tile_songs": (c_int, [POINTER(MrOptions), c_int32, c_int32, POINTER(c_int32)]),
    "mr_shard_tile_songs_n": (c_int, [POINTER(MrOptions), c_int32, c_int32, c_int32, c_int32, POINTER(c_int32)]),
    "mr_run": (c_int, [c_void_p, c_int]),
    "mr_sync": (c_int, [c_void_p]),
    "mr_graph_capture": (c_int, [c_void_p, c_int, c_int32]),
    "mr_graph_launch": (c_int, [c_void_p]),
    "mr_device_outputs": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p)]),
    "mr_score_dense": (c_int, [c_void_p, c_int, c_void_p]),
    "mr_topk": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "mr_copy_dense": (c_int, [c_void_p, c_void_p]),
    "mr_copy_topk": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "mr_copy_topk_device": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mr_copy_topk_device_async": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mr_topk_merge_device_async": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
    "mr_topk_record_bytes": (c_int, [c_int32, c_int32, POINTER(c_int64)]),
    "mr_topk_merge_records_async": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int64, c_void_p, c_void_p,
                                            c_void_p]),
    "mr_topk_merge_host": (c_int, [c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mr_topk_merge_device": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mr_kernel_times": (c_int, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_double), c_int32]),
    "mr_debug_stamps": (c_int, [c_void_p, c_void_p, c_int64]),
    "mr_timing_begin": (c_int, [c_void_p]),
    "mr_timing_stop": (c_int, [c_void_p]),
    "mr_timing_end": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_double)]),
    "mr_stream": (c_void_p, [c_void_p]),
    "mr_run_into": (c_int, [c_void_p, c_int, c_void_p]),
    "mr_view_get": (c_int, [c_void_p, POINTER(MrView)]),
    "mr_topk_dense_device": (c_int, [c_void_p, c_void_p, c_int32]),
    "mr_combine_device": (c_int, [c_void_p, c_int, c_double, ctypes.c_uint64, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "mr_combine_all_device": (c_int, [c_void_p, c_double, c_double, c_double, ctypes.c_uint64, c_int64, c_int64,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, POINTER(c_double)]),
    "mr_eval_minmax_device": (c_int, [c_void_p, c_void_p, POINTER(c_double), POINTER(c_double)]),
    "mr_dense_minmax": (c_int, [c_void_p, POINTER(c_double), POINTER(c_double)]),
    "mr_eval_counts_device": (c_int, [c_void_p, c_void_p, c_double, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_int32]),
    "mr_eval_map_device": (c_int, [c_void_p, c_void_p, c_double, c_double, c_void_p, c_void_p, c_void_p, c_int32,
                                   POINTER(c_double), c_int32]),
    "mr_eval_map": (c_int, [c_int32, c_void_p, c_void_p, c_void_p, c_int32, POINTER(c_double), c_int32]),
    "mr_eval_class_counts_device": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_int32, c_void_p, c_void_p, c_int32]),
    "mr_eval_map_counts_device": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                          c_int32]),
    "mr_last_error": (c_char_p, []),
    "mr_corpus_from_tsv": (c_int, [c_char_p, c_char_p, c_char_p, POINTER(c_void_p)]),
    "mr_corpus_dataset": (c_int, [c_void_p, POINTER(MrDataset)]),
    "mr_corpus_labels": (c_int, [c_void_p, POINTER(POINTER(c_int64)), POINTER(POINTER(c_int32)), POINTER(c_int32), POINTER(c_int32)]),
    "mr_corpus_name": (c_char_p, [c_void_p, c_int32, c_int32]),
    "mr_corpus_names": (c_int, [c_void_p, c_int32, c_char_p, c_int64, POINTER(c_int64)]),
    "mr_corpus_free": (c_int, [c_void_p]),
    "mr_version": (c_char_p, []),
    "mr_model_write_tsv": (c_int, [c_char_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32]),
    "mr_model_read_tsv": (c_int, [c_char_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "mr_java_double_string": (c_int, [c_double, c_char_p, c_int32]),
    "mr_song_shards": (c_int, [POINTER(MrDataset), c_int32, c_void_p]),
    "mr_song_shards_tiled": (c_int, [POINTER(MrDataset), c_int32, c_int32, c_void_p]),
    "mr_group_options_default": (c_int, [POINTER(MrGroupOptions)]),
    "mr_group_create": (c_int, [POINTER(MrOptions), POINTER(MrGroupOptions), POINTER(c_void_p)]),
    "mr_group_destroy": (c_int, [c_void_p]),
    "mr_group_load": (c_int, [c_void_p, POINTER(MrDataset)]),
    "mr_group_info": (c_int, [c_void_p, c_int32, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32),
                              POINTER(c_int32), POINTER(c_int32)]),
    "mr_group_transport": (c_int, [c_void_p, POINTER(c_int32)]),
    "mr_group_shape": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "mr_group_context": (c_void_p, [c_void_p, c_int32]),
    "mr_group_run": (c_int, [c_void_p, c_int]),
    "mr_group_sync": (c_int, [c_void_p]),
    "mr_group_copy_topk": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "mr_group_topk": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "mr_group_device_topk": (c_int, [c_void_p, c_int32, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p)]),
    "mr_group_copy_dense": (c_int, [c_void_p, c_void_p]),
    "mr_group_score_dense": (c_int, [c_void_p, c_int, c_void_p]),
    "mr_group_allgather_dense": (c_int, [c_void_p, c_void_p]),
}

_lib = None


def _preload_torch_runtime() -> None:
    try:  # one HIP runtime per process: let torch's copy be the one
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is part of the image
        pass


def lib() -> ctypes.CDLL:
    """Load (once) and return the engine library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()'); there is no CPU fallback"
        )
    _preload_torch_runtime()
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, where: str) -> None:
    if rc != MR_OK:
        msg = lib().mr_last_error()
        raise EngineError(rc, where, msg.decode() if msg else "")
