"""Multi-GPU exchange logic on CPU: world_size-2 `gloo` process group.

Each rank keeps a replica of the cluster state (the C oracle stands in for the
device scan of its shard), evaluates only its own node shard from
ksg_shard_range, packs the shard record, all-gathers the records over gloo and
applies the product's winner rule (ksg_merge_records, the same code the device
decide kernel runs after the RCCL all-gather). Every rank then commits the
winner to its replica. The pod -> node sequence and the RNG position must equal
the single-process schedule (generic_scheduler.go:54-96 run pod by pod).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kubernetes_amd import abi
from kubernetes_amd.engine import make_shard_record, merge_records, shard_range
from oracle.pyoracle import OracleScheduler
from tests.helpers import Case

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, nn, npods, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = Case(name, nn, npods)
        n = case.view.arrays.n_nodes
        lo, hi = shard_range(n, rank, world)
        spans = [shard_range(n, g, world) for g in range(world)]
        nwords_max = max((b + 63) // 64 - a // 64 for a, b in spans)
        orc = OracleScheduler(case.cfg)
        orc.set_cluster(case.view.arrays)
        rng = seed
        out = []
        for i in range(len(case.batch)):
            rc, fails, scores = orc.evaluate(case.batch, i)
            rec = make_shard_record(fails[lo:hi], scores[lo:hi], lo, lo // 64, nwords_max, error=rc < 0)
            gathered = [torch.zeros(len(rec), dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(gathered, torch.from_numpy(rec))
            recs = np.stack([g.numpy() for g in gathered])
            mrc, node, _, _, rng = merge_records(recs, n, rng_state=rng)
            if mrc == abi.KSG_OK:
                orc.add_pod(node, case.batch, i)  # every rank commits the same pod
                out.append(node)
            else:
                out.append(abi.KSG_OUT_NOFIT if mrc == abi.KSG_NOFIT else abi.KSG_OUT_ERROR)
        q.put((rank, out, rng, lo, hi))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,nn,npods", [("config2", 700, 160), ("config4", 450, 120), ("config1", 130, 300)])
def test_two_rank_sharded_schedule_matches_single(name, nn, npods):
    seed = 1234
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, name, nn, npods, seed, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    case = Case(name, nn, npods)
    orc = OracleScheduler(case.cfg)
    orc.set_cluster(case.view.arrays)
    want, st = orc.batch(case.batch, seed)
    for rank, out, rng, lo, hi in res:
        assert hi > lo
        assert np.array_equal(np.asarray(out), want), rank
        assert rng == st
    assert res[0][4] == res[1][3]  # shards are contiguous
    # both shards must have produced winners (the exchange is actually exercised)
    lo1 = res[1][3]
    assert (want >= lo1).any() and ((want >= 0) & (want < lo1)).any()


def test_shard_ranges_cover_nodes():
    for n in (0, 1, 63, 64, 65, 1000, 15000):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_range(n, g, world) for g in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a % 64 == 0
            assert all(a <= b for a, b in spans)


def test_merge_rule_tie_order_and_errors():
    """Global ix counts ties from the highest rank (types.go:42-47): shard 1's ties first."""
    n = 256
    recs = np.stack([
        make_shard_record(np.array([0, 0, 1]), np.array([5, 7, 7]), 0, 0, 2),       # node 1 ties at 7
        make_shard_record(np.array([0, 0]), np.array([7, 7]), 128, 2, 2),          # nodes 128,129 at 7
    ])
    got = [merge_records(recs, n, tie_index=i)[1] for i in range(4)]
    assert got == [129, 128, 1, 129]
    rc, node, m, k, _ = merge_records(recs, n, tie_index=0)
    assert (rc, m, k) == (abi.KSG_OK, 7, 3)
    rc, *_ = merge_records(recs, n, empty_priorities=True)
    assert rc == abi.KSG_NOFIT
    recs[0] = make_shard_record(np.array([1]), np.array([0]), 0, 0, 2, error=True)
    assert merge_records(recs, n)[0] == abi.KSG_ERR_NOPEER
    none = np.stack([make_shard_record(np.array([1]), np.array([0]), 0, 0, 2)] * 2)
    rc, node, _, _, st = merge_records(none, n, rng_state=9)
    assert rc == abi.KSG_NOFIT and st == 9  # no draw on FitError (generic_scheduler.go:72-77)


def _anti_worker(rank, world, port, nn, npods, seed, q):
    """ServiceAntiAffinity's sharded step (ksg_runtime.cpp scan_exchange): each
    rank sums the pod's service counts over the filtered nodes of its own shard
    per label domain, the partials are all-reduced (SUM, int32), every rank
    scores its shard with the global counts, and the shard records go through
    the product's winner rule."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = Case("config4", nn, npods)
        n = case.view.arrays.n_nodes
        n_pairs = len(case.view.arrays.pair_keys)
        n_anti = int(case.cfg.n_anti)
        lo, hi = shard_range(n, rank, world)
        spans = [shard_range(n, g, world) for g in range(world)]
        nwords_max = max((b + 63) // 64 - a // 64 for a, b in spans)
        orc = OracleScheduler(case.cfg)
        orc.set_cluster(case.view.arrays)
        rng = seed
        out, reduced_equal, split = [], True, 0
        for i in range(len(case.batch)):
            rc, part = orc.domain_counts(case.batch, i, lo, hi, n_anti, n_pairs)
            t = torch.from_numpy(part.copy())
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            glob = t.numpy()
            _, whole = orc.domain_counts(case.batch, i, 0, n, n_anti, n_pairs)
            reduced_equal &= bool(np.array_equal(glob, whole))
            split += int(0 < part.sum() < glob.sum())  # both shards hold counted pods
            rc2, fails, scores = orc.evaluate_counts(case.batch, i, glob)
            rec = make_shard_record(fails[lo:hi], scores[lo:hi], lo, lo // 64, nwords_max,
                                    error=rc < 0 or rc2 < 0)
            gathered = [torch.zeros(len(rec), dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(gathered, torch.from_numpy(rec))
            recs = np.stack([g.numpy() for g in gathered])
            mrc, node, _, _, rng = merge_records(recs, n, rng_state=rng)
            if mrc == abi.KSG_OK:
                orc.add_pod(node, case.batch, i)
                out.append(node)
            else:
                out.append(abi.KSG_OUT_NOFIT if mrc == abi.KSG_NOFIT else abi.KSG_OUT_ERROR)
        q.put((rank, out, rng, reduced_equal, split))
    finally:
        dist.destroy_process_group()


def test_two_rank_anti_affinity_domain_allreduce():
    """World-2 gloo rehearsal of the ServiceAntiAffinity all-reduce path: the
    summed shard partials equal the whole cluster's domain counts for every pod,
    and scoring each shard with them reproduces the single-process schedule."""
    nn, npods, seed = 450, 400, 4321
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_anti_worker, args=(r, WORLD, port, nn, npods, seed, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    case = Case("config4", nn, npods)
    assert int(case.cfg.n_anti) > 0
    orc = OracleScheduler(case.cfg)
    orc.set_cluster(case.view.arrays)
    want, st = orc.batch(case.batch, seed)
    for rank, out, rng, reduced_equal, split in res:
        assert reduced_equal, rank
        assert split >= 20, split  # the reduction actually combines two shards
        assert np.array_equal(np.asarray(out), want), rank
        assert rng == st


def _ext_worker(rank, world, port, nn, npods, seed, q):
    """The extensions' sharded step (ksg_runtime.cpp scan_exchange and the window path's
    count pass + all-reduce; parity unpinned): each rank takes the
    pod's max untolerated soft-taint count over the filtered nodes of its own shard
    (TaintTolerationPriority's NormalizeReduce max), the partials are all-reduced (MAX),
    every rank scores its shard with the global max, the shard records go through the
    product's winner rule, and every rank commits the winner with its extension record
    (extended resources)."""
    from tests.ext_cases import ExtCase

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = ExtCase("config2", nn, npods, w_taint=2, w_bal=1)
        n = c.case.view.arrays.n_nodes
        lo, hi = shard_range(n, rank, world)
        spans = [shard_range(n, g, world) for g in range(world)]
        nwords_max = max((b + 63) // 64 - a // 64 for a, b in spans)
        orc = c.load(OracleScheduler(c.cfg))
        rng = seed
        out, reduced_equal, split = [], True, 0
        for i in range(len(c.batch)):
            part = orc.taint_max(c.batch, i, lo, hi)
            t = torch.tensor([part], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            glob = int(t.item())
            reduced_equal &= glob == orc.taint_max(c.batch, i, 0, n)
            split += int(part < glob)  # the other shard holds the max
            rc, fails, scores = orc.evaluate_tmax(c.batch, i, glob)
            rec = make_shard_record(fails[lo:hi], scores[lo:hi], lo, lo // 64, nwords_max, error=rc < 0)
            gathered = [torch.zeros(len(rec), dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(gathered, torch.from_numpy(rec))
            recs = np.stack([g.numpy() for g in gathered])
            mrc, node, _, _, rng = merge_records(recs, n, rng_state=rng)
            if mrc == abi.KSG_OK:
                orc.add_pod(node, c.batch, i)
                out.append(node)
            else:
                out.append(abi.KSG_OUT_NOFIT if mrc == abi.KSG_NOFIT else abi.KSG_OUT_ERROR)
        q.put((rank, out, rng, reduced_equal, split, orc.read_ext_used().tolist()))
    finally:
        dist.destroy_process_group()


def test_two_rank_extension_taint_max_allreduce():
    """World-2 gloo rehearsal of the sharded extension path: the
    all-reduced shard maxima equal the whole cluster's TaintToleration max for every pod,
    and scoring each shard with it (plus BalancedAllocation and extended resources)
    reproduces the single-process schedule and extended-resource usage."""
    from tests.ext_cases import ExtCase

    nn, npods, seed = 700, 300, 77
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ext_worker, args=(r, WORLD, port, nn, npods, seed, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = ExtCase("config2", nn, npods, w_taint=2, w_bal=1)
    orc = c.load(OracleScheduler(c.cfg))
    want, st = orc.batch(c.batch, seed)
    used = orc.read_ext_used().tolist()
    for rank, out, rng, reduced_equal, split, ext_used in res:
        assert reduced_equal, rank
        assert np.array_equal(np.asarray(out), want), rank
        assert split >= 3, split  # the reduction actually combines two shards
        assert rng == st
        assert ext_used == used
