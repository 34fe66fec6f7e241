"""Node-sharded HIP path on one GPU: `world` ranks, each a separate process with
its own sharded ksg context on cuda:0, exchanging over gloo through
ksg_set_allgather (RCCL refuses two ranks on one device; with RCCL the same
kernels run and only the transport of the all-gather changes).

Each rank filters/scores only its node shard; the window path all-gathers the
shards' per-word results once per window and every rank resolves the window
over the replicated state; the per-pod path (window 0, ServiceAntiAffinity)
all-gathers shard records per pod (generic_scheduler.go:54-96 pod by pod).
Every rank's pod -> node sequence, RNG position and committed requested
totals must equal the C oracle's single-process schedule.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Fuzz:
    """A tests/test_gpu_fuzz.py case in the shape of tests.helpers.Case."""

    def __init__(self, fuzz_seed):
        from tests.test_gpu_fuzz import _case

        self.cfg, arrays, self.batch, _ = _case(fuzz_seed)
        self.view = type("View", (), {"arrays": arrays})()


# extension variants (parity unpinned: the C restatement is the checker):
# "ext:<config>:<variant>"
_EXT_KW = {"all": dict(w_taint=1, w_bal=1), "taint": dict(w_taint=2, w_bal=0), "filters": dict(w_taint=0, w_bal=0)}


def _make_case(name, nn, npods):
    from tests.families import FamilyCase
    from tests.helpers import Case

    if name.startswith("fam:"):
        return FamilyCase(name[4:], nn, npods)
    if name.startswith("ext:"):
        from tests.ext_cases import ExtCase
        _, cfg, var = name.split(":")
        return ExtCase(cfg, nn, npods, **_EXT_KW[var])
    return _Fuzz(nn) if name == "fuzz" else Case(name, nn, npods)


def _run_case(sched, case, seed, chunk=None):
    """run_batch, after the case's existing pods for a tests/families.py case."""
    from tests.helpers import run_batch

    if hasattr(case, "load"):
        case.load(sched)
        return sched.batch(case.batch, seed)
    return run_batch(sched, case, rng=seed, chunk=chunk)


def _worker(rank, world, port, name, nn, npods, window, chunk, seed, q):
    import torch.distributed as dist

    from kubernetes_amd.engine import DeviceScheduler, gloo_allgather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = _make_case(name, nn, npods)
        dev = DeviceScheduler(case.cfg, device=0, rank=rank, world=world, allgather=gloo_allgather())
        dev.set_window(window)
        out, rng = _run_case(dev, case, seed, chunk)
        used_c, used_m = dev.read_requested()
        lo, hi = dev.shard()
        stats = dev.last_batch_stats()
        if getattr(dev, "n_scalar", 0):  # (extensions: the extended resources taken, on every rank)
            stats = dict(stats, ext_used=dev.read_ext_used().tolist())
        dev.close()
        q.put((rank, out.tolist(), rng, used_c.tolist(), used_m.tolist(), lo, hi, stats, None))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, None, None, None, None, None, None, None, traceback.format_exc() + repr(e)))
    finally:
        dist.destroy_process_group()


def _run(name, nn, npods, window, world=2, chunk=None, seed=1234, timeout=110):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, nn, npods, window, chunk, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=timeout))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[8] is None, r[8]
    return res


def _oracle(name, nn, npods, seed=1234, ext_used=False):
    from oracle.pyoracle import OracleScheduler

    case = _make_case(name, nn, npods)
    orc = OracleScheduler(case.cfg)
    want, st = _run_case(orc, case, seed)
    wc, wm = orc.read_requested()
    if ext_used:
        return want, st, wc, wm, orc.read_ext_used().tolist()
    return want, st, wc, wm


@pytest.mark.parametrize("name,nn,npods,window,world,chunk", [
    ("config2", 700, 1500, 128, 2, None),    # window path, both shards non-empty
    ("config2", 5000, 2000, 1024, 2, None),  # config 2 node count, large windows
    ("config2", 1500, 900, 37, 3, 211),      # three ranks, ragged shards, windows cut by batches
    ("config2", 60, 300, 128, 2, None),      # one 64-node word: rank 0's shard is empty
    ("config2", 700, 400, 0, 2, None),       # per-pod exchange path
    ("config4", 900, 500, 128, 2, None),     # ServiceAntiAffinity: per-pod path + domain all-reduce
    ("config1", 500, 1000, 128, 2, None),    # BASELINE config 1
    ("config3", 15000, 50000, 128, 2, 1000), # BASELINE config 3 at full size, 1000-pod batches
    ("config4", 70000, 1000, 128, 2, 500),   # ServiceAntiAffinity, 35k-node shards: the LDS-slot resolver at P = 16
] + [(f"fam:{f}", 700, 400, 64, 2, None) for f in ("multi_service", "namespaces", "negative", "big_weights",
                                                   "existing_hosts", "invalid_selectors")])
def test_sharded_batch_matches_oracle(name, nn, npods, window, world, chunk):
    want, st, wc, wm = _oracle(name, nn, npods)
    res = _run(name, nn, npods, window, world=world, chunk=chunk)
    spans = [(r[5], r[6]) for r in res]
    assert spans[0][0] == 0 and (name == "fuzz" or spans[-1][1] == nn)
    for rank, out, rng, uc, um, lo, hi, stats, _ in res:
        got = np.asarray(out)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"rank {rank}: first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
        assert rng == st
        assert np.array_equal(np.asarray(uc), wc) and np.array_equal(np.asarray(um), wm)
    if world == 2 and all(b > a for a, b in spans):
        lo1 = spans[1][0]  # both shards must have produced winners
        assert (want >= lo1).any() and ((want >= 0) & (want < lo1)).any()


@pytest.mark.parametrize("name,nn,npods,window,world,chunk", [
    ("ext:config2:all", 700, 900, 128, 2, None),     # window path: TaintToleration max + histogram all-reduced
    ("ext:config2:all", 700, 400, 0, 2, None),       # per-pod path: scan phase 1 + the max all-reduce
    ("ext:config2:taint", 1500, 700, 37, 3, 211),    # three ranks, ragged shards, windows cut by batches
    ("ext:config2:filters", 5000, 1200, 128, 2, None),
    ("ext:config4:all", 900, 300, 128, 2, None),     # ServiceAntiAffinity + extensions: both all-reduces per pod
])
def test_sharded_extensions_match_oracle(name, nn, npods, window, world, chunk):
    """Extensions on a node-sharded context (parity unpinned): taints,
    extended resources (GPU counts), BalancedAllocation and TaintToleration, whose
    normalisation max is over every shard's filtered nodes. Every rank's placements, RNG
    position, requested totals and extended-resource usage equal the C restatement's
    single-process schedule."""
    want, st, wc, wm, xu = _oracle(name, nn, npods, ext_used=True)
    res = _run(name, nn, npods, window, world=world, chunk=chunk)
    for rank, out, rng, uc, um, lo, hi, stats, _ in res:
        got = np.asarray(out)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"rank {rank}: first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
        assert rng == st
        assert np.array_equal(np.asarray(uc), wc) and np.array_equal(np.asarray(um), wm)
        assert stats["ext_used"] == xu
        if window and "config4" not in name:
            assert stats["windows"] > 0  # (the window path took it)
    lo1 = res[1][5]  # both shards produced winners
    assert (want >= lo1).any() and ((want >= 0) & (want < lo1)).any()


@pytest.mark.parametrize("name,nn,npods,window,world,chunk", [
    ("config3", 15000, 50000, 128, 4, 1000),         # BASELINE config 3 at full size over 4 and 8 shards
    ("config3", 15000, 50000, 128, 8, 1000),
    ("config3", 15000, 1500, 0, 4, None),            # the per-pod exchange path
    ("config3", 15000, 1000, 0, 8, None),
    ("ext:config3:all", 15000, 6000, 128, 4, 1000),  # every extension: TaintToleration terms all-reduced
    ("ext:config3:all", 15000, 6000, 128, 8, 1000),
])
def test_sharded_four_and_eight_ranks_match_oracle(name, nn, npods, window, world, chunk):
    """the sharded merge and decide walk at 4 and 8 ranks (gloo on one GPU;
    the node loop that shards is generic_scheduler.go:107-126). 15,000 nodes = 235 words: 8 shards
    of 29-30 words. Every rank's placements, RNG position and committed totals equal the C
    restatement's single-process schedule."""
    ext = name.startswith("ext:")
    ref = _oracle(name, nn, npods, ext_used=ext)
    want, st, wc, wm = ref[:4]
    res = _run(name, nn, npods, window, world=world, chunk=chunk, timeout=600)
    spans = [(r[5], r[6]) for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == nn and all(b > a for a, b in spans)
    for rank, out, rng, uc, um, lo, hi, stats, _ in res:
        got = np.asarray(out)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"rank {rank}: first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
        assert rng == st
        assert np.array_equal(np.asarray(uc), wc) and np.array_equal(np.asarray(um), wm)
        if ext:
            assert stats["ext_used"] == ref[4]
        if window:
            assert stats["windows"] > 0
    for lo, hi in spans:  # every shard produced winners
        assert ((want >= lo) & (want < hi)).any(), (lo, hi)


@pytest.mark.parametrize("fuzz_seed", [2, 3, 6, 10, 11, 14])
def test_sharded_fuzz_matches_oracle(fuzz_seed):
    """Randomised clusters (tests/test_gpu_fuzz.py) over two ranks: anti-affinity
    domain counts all-reduced across shards, dense keys, tight capacities."""
    want, st, wc, wm = _oracle("fuzz", fuzz_seed, 0)
    res = _run("fuzz", fuzz_seed, 0, 64, world=2)
    for rank, out, rng, uc, um, lo, hi, stats, _ in res:
        got = np.asarray(out)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"rank {rank}: first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
        assert rng == st
        assert np.array_equal(np.asarray(uc), wc) and np.array_equal(np.asarray(um), wm)


# ---- RCCL itself on one GPU: the exchange path over a 1-rank communicator ------------
def _rccl_ctx(cfg):
    from kubernetes_amd.engine import DeviceScheduler

    return DeviceScheduler(cfg, device=0, rank=0, world=1, nccl_id=DeviceScheduler.nccl_unique_id())


@pytest.mark.parametrize("name,nn,npods,window", [
    ("config2", 1500, 1200, 128),  # window path: ncclAllGather of the per-word block per window
    ("config2", 700, 300, 0),      # per-pod path: ncclAllGather of the shard record per pod
    ("config4", 900, 400, 128),    # ServiceAntiAffinity: ncclAllReduce of the domain counts
])
def test_rccl_one_rank_batch_matches_oracle(name, nn, npods, window):
    """ncclCommInitRank / ncclAllGather / ncclAllReduce on the library's stream, through
    the same sharded code path world > 1 takes (RCCL refuses two ranks on one device)."""
    from tests.helpers import Case, run_batch

    want, st, wc, wm = _oracle(name, nn, npods)
    case = Case(name, nn, npods)
    dev = _rccl_ctx(case.cfg)
    try:
        dev.set_window(window)
        got, rng = run_batch(dev, case, rng=1234)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
        assert rng == st
        uc, um = dev.read_requested()
        assert np.array_equal(uc, wc) and np.array_equal(um, wm)
        if window:
            assert dev.last_batch_stats()["windows"] > 0
    finally:
        dev.close()


@pytest.mark.parametrize("window", [128, 0])
def test_rccl_one_rank_config2_every_extension_matches_oracle(window):
    """Config 2's shape (5,000 nodes) + taints, GPU counts, BalancedAllocation and
    TaintToleration over a 1-rank RCCL communicator: the sharded exchange path's
    ncclAllGather per window / per pod and the ncclAllReduce (max, sum) of the
    TaintToleration terms, against the C restatement (parity unpinned)."""
    from oracle.pyoracle import OracleScheduler
    from tests.ext_cases import ExtCase

    c = ExtCase("config2", 5000, 2400 if window else 600)
    orc = c.load(OracleScheduler(c.cfg))
    dev = c.load(_rccl_ctx(c.cfg))
    try:
        dev.set_window(window)
        for i in range(0, 60, 3):  # placed pods with extended resource requests
            dev.add_pod(i * 7, c.batch, i)
            orc.add_pod(i * 7, c.batch, i)
        from kubernetes_amd.engine import PodBatch
        rest = PodBatch(c.batch.pods[60:], c.batch.ids, c.batch.ext[60:])
        got, rg = dev.batch(rest, 99)
        want, rw = orc.batch(rest, 99)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
        assert rg == rw
        assert np.array_equal(dev.read_ext_used(), orc.read_ext_used())
        if window:
            assert dev.last_batch_stats()["windows"] > 0
    finally:
        dev.close()
        orc.close()


def test_rccl_one_rank_begin_commit_matches_oracle():
    from kubernetes_amd import abi
    from oracle.pyoracle import OracleScheduler
    from tests.helpers import Case

    case = Case("config4", 600, 150)
    dev, orc = _rccl_ctx(case.cfg), OracleScheduler(case.cfg)
    try:
        dev.set_cluster(case.view.arrays)
        orc.set_cluster(case.view.arrays)
        rng = np.random.default_rng(3)
        for i in range(len(case.batch)):
            rg, mg, kg, failg = dev.begin(case.batch, i, want_fail=True)
            ro, mo, ko, failo = orc.begin(case.batch, i, want_fail=True)
            assert (rg, kg) == (ro, ko), i
            assert np.array_equal(failg, failo)
            if rg == abi.KSG_OK:
                assert mg == mo
                ix = int(rng.integers(0, kg))
                assert dev.commit(ix) == orc.commit(ix)
    finally:
        dev.close()
        orc.close()


# ---- ranks with different histories before a shared batch -------------------------
def _history_worker(rank, world, port, q):
    """Both ranks run the same (collective) batches; between them rank 0 alone
    adds and removes extra pods (its host mirror, patch queue and deferred replay
    differ from rank 1's) and arrives late. Both ranks must enqueue the same
    launches and collectives in every batch (a rank that sized its window rounds
    from its own history would hang the all-gather) and end with the oracle's
    placements."""
    import time

    import torch.distributed as dist

    from kubernetes_amd.engine import DeviceScheduler, PodBatch, gloo_allgather
    from tests.helpers import Case

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = Case("config2", 1500, 1600)
        dev = DeviceScheduler(case.cfg, device=0, rank=rank, world=world, allgather=gloo_allgather())
        dev.set_window(128)
        dev.set_cluster(case.view.arrays)
        pods = case.batch.pods
        rng = 1234
        outs = []
        # (the batches themselves are collective: every rank makes the same calls)
        for a, b in ((0, 150), (150, 400), (400, 600)):
            o, rng = dev.batch(PodBatch(pods[a:b], case.batch.ids), rng)
            outs.append(o)
            if rank == 0:  # rank-local history between the batches
                ep = pods[1500 + a // 6:1500 + b // 6].copy()
                ep["service"], ep["n_svcs"] = -1, 0  # (a removed pod leaves no service peer behind)
                extra = PodBatch(ep, case.batch.ids)
                for i in range(len(extra)):
                    dev.add_pod((7 * i + a) % 1500, extra, i)
                for i in range(len(extra)):
                    dev.remove_pod(int(extra.pods[i]["uid"]))
                time.sleep(0.3)
        o, rng = dev.batch(PodBatch(pods[600:1500], case.batch.ids), rng)
        outs.append(o)
        used_c, used_m = dev.read_requested()
        dev.close()
        q.put((rank, np.concatenate(outs).tolist(), rng, used_c.tolist(), used_m.tolist(), None))
    except Exception as e:
        import traceback

        q.put((rank, None, None, None, None, traceback.format_exc() + repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_ranks_with_different_histories():
    """(Round-1 advisor: per-rank round sizing could hang the exchange.) Every
    collective of a window round is sized from this batch's progress only."""
    import torch.multiprocessing as mp

    from kubernetes_amd.engine import PodBatch
    from oracle.pyoracle import OracleScheduler
    from tests.helpers import Case

    case = Case("config2", 1500, 1600)
    orc = OracleScheduler(case.cfg)
    orc.set_cluster(case.view.arrays)
    want, st = orc.batch(PodBatch(case.batch.pods[:1500], case.batch.ids), 1234)
    wc, wm = orc.read_requested()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_history_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(2):
            res.append(q.get(timeout=110))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, out, rng, uc, um, err in sorted(res, key=lambda r: r[0]):
        assert err is None, err
        got = np.asarray(out)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"rank {rank}: first mismatches at {bad[:8]}"
        assert rng == st
        assert np.array_equal(np.asarray(uc), wc) and np.array_equal(np.asarray(um), wm)
