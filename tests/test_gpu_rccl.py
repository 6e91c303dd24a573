"""GPU: the collective path the driver's N > 1 command runs, executed with
REAL RCCL on one GPU (a one-rank `nccl` process group, initialised the way
bench.py does it: `init_process_group("nccl", device_id=...)`).

Every multi-rank rehearsal so far used gloo, which takes the host branch of
the exchange (sharding.py ShardScorer.exchange / exchange_topk); these tests
run the `nccl` branches — `all_gather_into_tensor` of the packed top-k record
blocks with the engine-stream / torch-stream event ordering, the MIN/MAX/SUM
all-reduces of the threshold mAP, and bench.py's broadcast_object_list,
barriers and stats all-reduces (MR_BENCH_PG=1) — and compare the results
bitwise with the single-context engine (≙ distributed.scala:477-479's
`collect.flatten` of the song partition)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

from musicrecommendation_amd import evaluation, synth
from musicrecommendation_amd.engine import Engine
from musicrecommendation_amd.ensemble import DeviceEnsemble
from musicrecommendation_amd.sharding import ShardScorer, exchange_topk, merge_gathered_host

from oracle import native
from helpers import pg_init_method

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(args, env, tries=3):
    """bench.py under torchrun at one rank on a port found free just before.
    Another process can take that port before torchrun's store binds it
    (EADDRINUSE at the rendezvous, before any GPU work): then a fresh port."""
    for _ in range(tries):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
               *args]
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        if p.returncode == 0 or "EADDRINUSE" not in p.stderr:
            return p
    return p


@pytest.fixture
def rccl_group():
    """A one-rank RCCL group on cuda:0, as bench.py main() creates it
    (`device_id`), with a FileStore rendezvous (no TCP port to race for)."""
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=pg_init_method(), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg,route", [("c2", "auto"), ("c3", "cooc"), ("c3", "two_hop")])
def test_shard_scorer_exchange_over_rccl(rccl_group, cfg, route):
    """ShardScorer.step() + exchange(): the record block copied out on the
    engine stream, all_gather_into_tensor on torch's stream (the nccl branch),
    the merge back on the engine stream — no host sync in between. The merged
    lists equal the engine's own lists and the fixed-point oracle, bitwise."""
    ds = synth.config(cfg, n_test=16 if cfg == "c2" else 64).dataset()
    sc = ShardScorer(ds, 0, 1, 0, topk=10, dense=False, out_dtype="f32", ibm_route=route)
    try:
        sc.exchange_always = True
        for _ in range(3):  # repeated steps reuse the record / gather buffers
            sc.step("ibm")
        got_s, got_k = sc.topk()
        own_s, _sc, own_k = sc.engine.topk()
        assert np.array_equal(got_s, own_s) and np.array_equal(got_k, own_k)
        _, ts, tk = native.fp_model(ds, "ibm", k=10, dense=False)
        assert np.array_equal(got_s, ts) and np.array_equal(got_k, tk)
        # the exchange alone, twice more (bench.py times it in its own loop)
        sc.exchange()
        sc.exchange()
        s2, k2 = sc.topk()
        assert np.array_equal(s2, own_s) and np.array_equal(k2, own_k)
        if route != "auto":
            assert sc.engine.ibm_route == route
    finally:
        sc.engine.close()


def test_exchange_topk_cuda_tensors_over_rccl(rccl_group):
    """sharding.exchange_topk with CUDA tensors under an nccl group: the
    packed record block goes through all_gather_into_tensor on the device
    (not the host branch); unpacked and merged = the inputs."""
    ds = synth.config("c2", n_test=12).dataset()
    with Engine(ds, topk=10, dense=False) as e:
        e.run("ibm")
        s, _sc, k = e.topk()
    ts, tk = torch.from_numpy(s).cuda(), torch.from_numpy(k).cuda()
    gs, gk = exchange_topk(ts, tk)
    assert gs.is_cuda and gs.shape == (1, ds.n_test, 10)
    ms, mk = merge_gathered_host(gs, gk)
    assert np.array_equal(ms, s) and np.array_equal(mk, k)


def test_threshold_map_reductions_over_rccl(rccl_group):
    """DeviceEnsemble with collectives forced on one rank: min/max all-reduced
    (MIN / MAX) and the per-class counts all-reduced (SUM) over RCCL, then
    the host fold — equal to the single-context device mAP, for all five
    models of C5's step (ubm, ibm, the three combinations)."""
    ds = synth.config("c2", n_test=24).dataset()
    with Engine(ds, out_dtype="f32", topk=10) as e:
        red = DeviceEnsemble(e, collectives=True)
        loc = DeviceEnsemble(e)
        u, i = red.model("ubm"), red.model("ibm")
        lcm, am, scm = red.combinations(u, i, 0.5, 0.5, 0.5, seed=1)
        for t in (u, i, lcm, am, scm):
            assert red._reduce() and not loc._reduce()
            for nt in (10, 11):
                assert red.threshold_map(t, nt) == loc.threshold_map(t, nt)
        exp = evaluation.threshold_map(lcm.cpu().numpy().astype(np.float64), ds)
        assert abs(red.threshold_map(lcm) - exp) <= 1e-12
        # the batched path of the multi-rank C5 step: one MAX all-reduce of
        # the five (-min, max), the class-indexed count block of all five
        # models SUM-all-reduced over RCCL on the device, the AP on the device
        models = {"ubm": u, "ibm": i, "lcm": lcm, "am": am, "scm": scm}
        for nt in (10, 11):
            got = red.threshold_maps(models, nt)
            assert got == {n: loc.threshold_map(t, nt) for n, t in models.items()}


def test_bench_one_rank_rccl_rehearsal(tmp_path):
    """The driver's N > 1 command shape at N = 1 (torchrun, one rank) with
    MR_BENCH_PG=1: init_process_group("nccl", device_id=...), the C2 line's
    barriers and stats all-reduces, and the north_star block's
    shared_bulk_dataset (broadcast_object_list + a file hand-off), timed
    barriers, MAX/SUM all-reduces and the forced all-gather exchange, all over
    RCCL (the north star on the 10k/1k C3 shape to keep the test short)."""
    env = dict(os.environ, MR_BENCH_PG="1", TMPDIR=str(tmp_path), PYTHONUNBUFFERED="1")
    p = _torchrun(["--gpus", "1", "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--no-e2e",
                   "--ns-config", "c3", "--ns-steps", "3", "--ns-warmup", "1"], env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["value"] > 0
    ns = line["north_star"]
    assert ns["process_group"]["backend"] == "nccl" and ns["process_group"]["world_size"] == 1
    assert ns["process_group"]["rehearsal"]
    assert ns["exchange_ms_per_step"] > 0 and ns["allgather_bytes_per_rank"] == ns["record_bytes"] > 0
    assert ns["ms_per_step"] > 0 and ns["layout"] == "songs1xusers1"
    # the temporary hand-off directory of shared_bulk_dataset was removed
    assert not [d for d in os.listdir(tmp_path) if d.startswith("mr_")]


def test_bench_c5_one_rank_rccl_rehearsal(tmp_path):
    """The C5 line under torchrun at N = 1 with MR_BENCH_PG=1: the process
    group up over RCCL, shared_bulk_dataset's hand-off, EnsembleScorer and
    DeviceEnsemble.threshold_maps' MAX and SUM all-reduces of the five
    models' extremes and class-count block over RCCL — the same five mAPs
    as the single-process line computes without collectives."""
    env = dict(os.environ, MR_BENCH_PG="1", TMPDIR=str(tmp_path), PYTHONUNBUFFERED="1")
    p = _torchrun(["--gpus", "1", "--config", "c5", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                   "--no-e2e"], env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    maps = line["threshold_mAP"]
    assert set(maps) == {"ubm", "ibm", "lcm", "am", "scm"} and all(0 < v < 1 for v in maps.values())
    # the single-process line's values on the same seeded data (every C5 bench
    # of rounds 5-6, e.g. profiles/r06/bench_c5.json): a regression anchor of
    # this engine's own output, not a reference fixture
    ref = {"ubm": 0.0009340961307245022, "ibm": 0.0020751807777950114, "lcm": 0.0009403874247581429,
           "am": 0.0009064927680186897, "scm": 0.0008915149560019554}
    assert maps == ref
