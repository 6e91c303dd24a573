"""GPU, two ranks on one card (gloo process group; RCCL needs one GPU per
rank): C5's per-model layouts with real engine contexts (sharding.EnsembleScorer)
— ubm on test-user blocks, ibm on song shards, the ibm rows moved by the
all-to-all, the combinations on the blocks and the five threshold mAPs through
the class-count reduction (mr_eval_class_counts_device +
mr_eval_map_counts_device). Every model's rows and every mAP equal one
context's, bitwise, on both ibm routes."""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import pg_init_method

pytestmark = pytest.mark.gpu


def _dataset():
    from musicrecommendation_amd import synth
    return synth.config("c3", n_test=48).dataset()


def _run(rank, world, init, route, out):
    from musicrecommendation_amd.sharding import EnsembleScorer

    if world > 1:
        dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        sc = EnsembleScorer(_dataset(), rank, world, 0, ibm_route=route)
        try:
            blocks, maps = sc.step(0.5, 0.5, 0.5, seed=1)
            out[rank] = ({k: v.cpu().numpy() for k, v in blocks.items()}, maps, sc.ibm_route)
        finally:
            sc.close()
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("route", ["cooc", "auto"])
def test_two_ranks_per_model_layouts_on_one_gpu(route):
    one = {}
    _run(0, 1, 0, route, one)
    one_blocks, one_maps, _ = one[0]
    world = 2
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        mp.start_processes(_run, args=(world, pg_init_method(), route, out), nprocs=world, join=True,
                           start_method="spawn")
        res = dict(out)
    for name, rows in one_blocks.items():
        got = np.concatenate([res[r][0][name] for r in range(world)])
        assert np.array_equal(got, rows, equal_nan=True), name
    for r in range(world):
        assert res[r][1] == one_maps
    if route == "cooc":
        assert all(res[r][2] == "cooc" for r in range(world))


def test_class_count_reduction_equals_device_map():
    """mr_eval_class_counts_device + mr_eval_map_counts_device over both
    models at once on one context = mr_eval_map_device per model (counts over
    every test user, no reduction), and the class blocks = the full tables'
    label-class rows."""
    from musicrecommendation_amd import evaluation
    from musicrecommendation_amd.engine import Engine
    from musicrecommendation_amd.ensemble import DeviceEnsemble

    ds = _dataset()
    with Engine(ds, out_dtype="f32", topk=10) as e:
        ens = DeviceEnsemble(e)
        pos = evaluation.label_pos(ds)
        cls = np.nonzero(pos > 0)[0].astype(np.int32)
        ts = [ens.model(name) for name in ("ubm", "ibm")]
        mms = [e.eval_minmax(t.data_ptr()) for t in ts]
        for n_thr in (10, 11):
            want = [e.eval_map(t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs, pos, ds.n_label_songs,
                               n_thresholds=n_thr) for t, (mn, mx) in zip(ts, mms)]
            blk = torch.empty((2, 2, cls.shape[0], n_thr), dtype=torch.int32, device="cuda")
            e.eval_class_counts([t.data_ptr() for t in ts], [m[0] for m in mms], [m[1] for m in mms], ds.lab_off,
                                ds.lab_songs, cls, blk.data_ptr(), n_thresholds=n_thr)
            got = e.eval_map_counts(2, blk.data_ptr(), pos[cls], ds.n_label_songs, n_thresholds=n_thr)
            assert got == want, n_thr
            b = blk.cpu().numpy()
            for i, (t, (mn, mx)) in enumerate(zip(ts, mms)):
                p, tp = e.eval_counts(t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs, n_thresholds=n_thr)
                assert np.array_equal(b[i, 0], p[cls]) and np.array_equal(b[i, 1], tp[cls])
