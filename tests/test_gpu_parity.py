"""GPU parity: the HIP path (through the C ABI) vs the C oracle, bit-exact.

Compared: pod -> node assignments (incl. FitError / error outcomes), the tie-break
RNG stream position, per-node fail codes and integer scores, and the committed
per-node requested totals. Sizes exercise every kernel variant (nodes per thread
R = 1..32) and every BASELINE config's predicate/priority set.
"""
import numpy as np
import pytest

from kubernetes_amd import abi
from kubernetes_amd.engine import DeviceScheduler, PodBatch
from oracle.pyoracle import OracleScheduler
from tests.helpers import Case, run_batch

pytestmark = pytest.mark.gpu


def _pair(case, window=None):
    dev = DeviceScheduler(case.cfg, device=0)
    if window is not None:
        dev.set_window(window)
    return dev, OracleScheduler(case.cfg)


@pytest.mark.parametrize("window", [0, 1024, 37])
@pytest.mark.parametrize("name,nn,npods", [
    ("config1", 500, 1000),      # BASELINE config 1 at full size
    ("config2", 700, 1500),
    ("config2", 2000, 3000),
    ("config4", 900, 1500),
    ("config2", 5000, 2000),     # config 2 node count
    ("config2", 9000, 800),      # R = 16 (memory-resident node state)
    ("config4", 20000, 300),     # R = 32, anti-affinity
    ("config2", 40000, 500),     # window path at P = 16 (8-entry ring)
])
def test_batch_matches_oracle(name, nn, npods, window):
    """window=0: exact one-pod-at-a-time kernel; >0: speculative window path."""
    case = Case(name, nn, npods)
    dev, orc = _pair(case, window)
    got, sg = run_batch(dev, case)
    want, sw = run_batch(orc, case)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    dev.close()


@pytest.mark.parametrize("resolver", [2048, 4096])
@pytest.mark.parametrize("name,nn,npods", [("config4", 900, 1500), ("config4", 5000, 3000)])
def test_anti_affinity_alternatives_match_oracle(name, nn, npods, resolver, monkeypatch):
    """ServiceAntiAffinity windows without the re-rank (KSG_DEBUG & 2048: a
    service's commit ends the window) and the re-rank in the LDS-slot resolver
    (& 4096) give the oracle's placements too (the default is the re-rank in
    the register-slot resolver)."""
    monkeypatch.setenv("KSG_DEBUG", str(resolver))
    case = Case(name, nn, npods)
    dev, orc = _pair(case, 1024)
    got, sg = run_batch(dev, case)
    want, sw = run_batch(orc, case)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    st = dev.last_batch_stats()
    assert st["windows"] > 0
    if resolver == 2048:  # windows end at pods whose service had a commit in them
        assert st["stops_service"] >= st["windows"] // 2
    dev.close()


@pytest.mark.parametrize("window", [0, 256])
def test_batch_chunks_equal_one_batch(window):
    """Batch boundaries must not change outcomes (state persists across launches)."""
    case = Case("config2", 1500, 1200)
    dev, orc = _pair(case, window)
    got, sg = run_batch(dev, case, chunk=97)
    want, sw = run_batch(orc, case)
    assert np.array_equal(got, want) and sg == sw
    dev.close()


def test_begin_commit_and_evaluate_match_oracle():
    case = Case("config4", 800, 300)
    dev, orc = _pair(case)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    rng = np.random.default_rng(7)
    for i in range(len(case.batch)):
        if i % 25 == 0:
            rcg, fg, sg = dev.evaluate(case.batch, i)
            rco, fo, so = orc.evaluate(case.batch, i)
            assert rcg == rco
            assert np.array_equal(fg, fo)
            fit = fg == 0
            assert np.array_equal(sg[fit], so[fit])
        rg, mg, kg, failg = dev.begin(case.batch, i, want_fail=True)
        ro, mo, ko, failo = orc.begin(case.batch, i, want_fail=True)
        assert (rg, kg) == (ro, ko), i
        assert np.array_equal(failg, failo)
        if rg == abi.KSG_OK:
            assert mg == mo
            ix = int(rng.integers(0, kg))
            assert dev.commit(ix) == orc.commit(ix)
    dev.close()


def test_existing_pods_add_remove():
    """ksg_add_pod / ksg_remove_pod incl. pods on hosts outside the node list."""
    case = Case("config2", 600, 900)
    dev, orc = _pair(case)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    n = case.view.arrays.n_nodes
    rng = np.random.default_rng(3)
    pre = 400
    for i in range(pre):
        host = int(rng.integers(0, n + 5))  # some hosts are not nodes
        for s in (dev, orc):
            s.add_pod(host, case.batch, i)
    for i in range(0, pre, 3):
        uid = int(case.batch.pods[i]["uid"])
        for s in (dev, orc):
            s.remove_pod(uid)
    rest = PodBatch(case.batch.pods[pre:], case.batch.ids)
    got, sg = dev.batch(rest, 99)
    want, sw = orc.batch(rest, 99)
    assert np.array_equal(got, want) and sg == sw
    dev.close()


def test_no_nodes_and_empty_priorities():
    case = Case("config2", 64, 10)
    # all-zero weights: prioritizeNodes returns an empty list -> FitError for every pod
    from kubernetes_amd import factory
    cfgz = factory.create_from_keys(["PodFitsResources"], ["EqualPriority"]).compile(case.it.key_id)
    dev = DeviceScheduler(cfgz)
    dev.set_cluster(case.view.arrays)
    out, st = dev.batch(case.batch, 5)
    assert (out == abi.KSG_OUT_NOFIT).all() and st == 5
    # no nodes
    empty = type(case.view.arrays)(case.view.arrays.nodes[:0], case.view.arrays.node_pairs[:0],
                                   case.view.arrays.pair_keys, case.view.arrays.n_services)
    dev.set_cluster(empty)
    out, _ = dev.batch(case.batch, 5)
    assert (out == abi.KSG_OUT_NONODES).all()
    dev.close()


def test_batch_rejects_duplicate_uids_and_keeps_mirror():
    """A pod uid already scheduled (replayed into the host mirror lazily) is refused
    before any device work; remove_pod after a batch sees that batch's commits."""
    from kubernetes_amd.engine import KsgError

    case = Case("config2", 300, 200)
    dev, orc = _pair(case, 128)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    half = PodBatch(case.batch.pods[:100], case.batch.ids)
    got, st = dev.batch(half, 7)
    want, sw = orc.batch(half, 7)
    assert np.array_equal(got, want) and st == sw
    with pytest.raises(KsgError):
        dev.batch(PodBatch(case.batch.pods[50:60], case.batch.ids), st)
    # removing a pod of the last batch undoes its commit exactly (mirror replay)
    uid = int(case.batch.pods[0]["uid"])
    dev.remove_pod(uid)
    orc.remove_pod(uid)
    rest = PodBatch(case.batch.pods[100:], case.batch.ids)
    g2, _ = dev.batch(rest, st)
    w2, _ = orc.batch(rest, sw)
    assert np.array_equal(g2, w2)
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    dev.close()


def test_batch_uid_reuse_after_no_fit_and_in_batch_duplicates():
    """The deferred-replay uid set: a pod that found no node leaves its uid free
    for a later batch (an unschedulable pod's retry); two placed pods of one batch
    with the same uid fail the call."""
    from kubernetes_amd.engine import KsgError

    case = Case("config2", 300, 200)
    for window in (0, 128):
        dev, orc = _pair(case, window)
        dev.set_cluster(case.view.arrays)
        orc.set_cluster(case.view.arrays)
        first = case.batch.pods[:40].copy()
        first[7]["milli_cpu"] = 10**13  # fits no node
        got, st = dev.batch(PodBatch(first, case.batch.ids), 11)
        want, sw = orc.batch(PodBatch(first, case.batch.ids), 11)
        assert np.array_equal(got, want) and st == sw
        assert got[7] == abi.KSG_OUT_NOFIT
        retry = case.batch.pods[40:80].copy()
        retry[0] = case.batch.pods[7]  # the same uid, now with a request that fits
        g2, st = dev.batch(PodBatch(retry, case.batch.ids), st)
        w2, sw = orc.batch(PodBatch(retry, case.batch.ids), sw)
        assert np.array_equal(g2, w2) and st == sw and g2[0] >= 0
        dup = case.batch.pods[80:90].copy()
        dup[5] = dup[2]
        with pytest.raises(KsgError):
            dev.batch(PodBatch(dup, case.batch.ids), st)
        dev.close()


@pytest.mark.parametrize("max_words", ["1024", "512"])
def test_fused_launch_at_p16_matches_oracle(max_words, monkeypatch):
    """40,000 nodes (625 words, P = 16): the fused window launch by default since round 6
    (KSG_FUSED_MAX_WORDS 1024), three launches with the gate at 512; both bit-exact against the
    oracle, and the launch form asserted from the kernel events (the fused launch has no phase-A
    events of its own)."""
    monkeypatch.setenv("KSG_KERNEL_EVENTS", "1")
    monkeypatch.setenv("KSG_FUSED_MAX_WORDS", max_words)
    case = Case("config2", 40000, 1500)
    dev, orc = _pair(case, 128)
    got, sg = run_batch(dev, case, chunk=500)
    want, sw = run_batch(orc, case, chunk=500)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    k = dev.last_batch_kernel_ms()
    assert k["launches"] > 0 and k["resolve_ms"] > 0
    assert (k["eval_ms"] == 0) == (max_words == "1024"), k
    dev.close()


@pytest.mark.parametrize("max_words", ["2048", "1024"])
def test_fused_launch_at_p32_matches_oracle(max_words, monkeypatch):
    """70,000 nodes (1,094 words, P = 32): three launches per window at the default gate (1,024
    words), the fused launch when the gate is lifted to 2,048 (measured slower there and not the
    default; the switch stays a supported setting, so it is held to the oracle)."""
    monkeypatch.setenv("KSG_KERNEL_EVENTS", "1")
    monkeypatch.setenv("KSG_FUSED_MAX_WORDS", max_words)
    case = Case("config5", 70000, 600)
    dev, orc = _pair(case, 128)
    got, sg = run_batch(dev, case, chunk=300)
    want, sw = run_batch(orc, case, chunk=300)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    k = dev.last_batch_kernel_ms()
    assert k["launches"] > 0 and k["resolve_ms"] > 0
    assert (k["eval_ms"] == 0) == (max_words == "2048"), k
    dev.close()


def test_kernel_time_sampling_strides(monkeypatch):
    """ksg_last_batch_kernel_ms: HIP events around every N-th window launch
    (KSG_KERNEL_EVENTS=N at context creation), scaled to all launches; 0 times
    nothing. The decisions never depend on it."""
    case = Case("config2", 600, 400)
    res = {}
    # (default: the fused window launch, phase A inside the resolver's launch, so eval_ms is 0;
    # KSG_FUSED=0: phase A launched and timed apart)
    for stride, fused in (("1", "1"), ("4", "1"), ("0", "1"), ("1", "0"), ("4", "0")):
        monkeypatch.setenv("KSG_KERNEL_EVENTS", stride)
        monkeypatch.setenv("KSG_FUSED", fused)
        dev, orc = _pair(case, 128)
        got, sg = run_batch(dev, case)
        res[stride + fused] = (got, sg, dev.last_batch_kernel_ms())
        dev.close()
    assert all(np.array_equal(res["11"][0], r[0]) and res["11"][1] == r[1] for r in res.values())
    for key in ("11", "41", "10", "40"):
        k = res[key][2]
        assert k["launches"] > 0 and k["resolve_ms"] > 0
        assert (k["eval_ms"] > 0) == (key[1] == "0"), (key, k)
    assert res["01"][2]["resolve_ms"] == 0 and res["01"][2]["launches"] > 0


@pytest.mark.parametrize("fused", ["1", "0"])
def test_batch_totals_sum_the_per_batch_diagnostics(fused, monkeypatch):
    """ksg_batch_totals = the per-batch diagnostics summed over batches."""
    monkeypatch.setenv("KSG_FUSED", fused)
    case = Case("config2", 500, 300)
    dev, _ = _pair(case, 128)
    dev.set_cluster(case.view.arrays)
    t0 = dev.batch_totals()
    assert t0["batches"] == 0 and t0["device_ms"] == 0.0
    rng, dms, res, win = 3, 0.0, 0.0, 0
    for s in (0, 150):
        _, rng = dev.batch(PodBatch(case.batch.pods[s:s + 150], case.batch.ids), rng)
        dms += dev.last_batch_ms()
        res += dev.last_batch_kernel_ms()["resolve_ms"]
        win += dev.last_batch_stats()["windows"]
    t1 = dev.batch_totals()
    assert t1["batches"] == 2 and win == t1["windows"] > 0
    assert abs(t1["device_ms"] - dms) < 1e-9 and abs(t1["resolve_ms"] - res) < 1e-9
    assert t1["host_us"]["validate"] > 0
    # phase A, the T0-image kernel and the resolver are timed apart (every 4th launch sampled);
    # the fused window launch (the default on one plain rank) is one kernel: all resolver time
    if fused == "0":
        assert t1["eval_ms"] > 0 and t1["t0_ms"] > 0 and t1["resolve_ms"] > 0
    else:
        assert t1["eval_ms"] == 0 and t1["t0_ms"] == 0 and t1["resolve_ms"] > 0
    dev.close()


_BIG = {}


def _big_case():
    # BASELINE config 5 shape: 100k nodes with 32 dense label keys (ingest ~10 s, built once)
    if "c5" not in _BIG:
        _BIG["c5"] = Case("config5", 100000, 400)
    return _BIG["c5"]


@pytest.mark.parametrize("window", [0, 128])
def test_config5_100k_nodes_matches_oracle(window):
    """One shard of 100k nodes: the exact kernel at R = 128 (per-node scores in HBM
    scratch) and the window path at P = 32 (4-entry ring)."""
    case = _big_case()
    dev, orc = _pair(case, window)
    got, sg = run_batch(dev, case)
    want, sw = run_batch(orc, case)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    dev.close()


@pytest.mark.parametrize("name,nn,npods", [
    ("config2", 5000, 10000),    # BASELINE config 2 at its stated size
    ("config3", 15000, 50000),   # BASELINE config 3 (one GPU)
    ("config4", 5000, 10000),    # BASELINE config 4 (ServiceAffinity + ServiceAntiAffinity)
])
def test_full_size_matches_oracle(name, nn, npods):
    """A BASELINE config at its stated size on one GPU, in 1,000-pod batches (as
    bench.py steps): every decision, the RNG position and the committed totals
    against the incremental oracle; plus the size-independent checksum requested
    totals == the sum of the placed pods' requests."""
    case = Case(name, nn, npods)
    dev, orc = _pair(case)
    got, sg = run_batch(dev, case, chunk=1000)
    want, sw = run_batch(orc, case, chunk=1000)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    ok = got >= 0
    sc = np.zeros_like(gc)
    np.add.at(sc, got[ok], case.batch.pods["milli_cpu"][ok].astype(np.int64))
    assert np.array_equal(sc, gc)
    assert dev.last_batch_stats()["windows"] > 0
    dev.close()


@pytest.mark.parametrize("rerank", [True, False])
@pytest.mark.parametrize("nn,npods", [
    (40000, 3000),   # P = 16: the domain rows' node bitmaps from HBM (win2_zg)
    (70000, 2000),   # P = 32: the fit and best-per-row bitmaps from phase A's rows too (win2_fg)
])
def test_anti_affinity_large_shard_window_matches_oracle(nn, npods, rerank, monkeypatch):
    """ServiceAntiAffinity (config 4's policy) past 32k nodes on one shard takes the window
    path, not the exact kernel: the re-rank resolver with its large bitmaps off LDS, and
    without the re-rank (KSG_DEBUG & 2048: the LDS-slot resolver, the one multi-priority and
    sharded anti-affinity contexts take) -- every decision, the RNG position and the committed
    totals against the incremental oracle."""
    if not rerank:
        monkeypatch.setenv("KSG_DEBUG", "2048")
    case = Case("config4", nn, npods)
    dev, orc = _pair(case)
    got, sg = run_batch(dev, case, chunk=1000)
    st = dev.last_batch_stats()
    want, sw = run_batch(orc, case, chunk=1000)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    assert st["windows"] > 0, st
    dev.close()


def test_many_anti_priorities_large_shard_window_matches_oracle():
    """Six ServiceAntiAffinity priorities (tests/families.py many_anti) at 40k nodes: the
    window path (phase A past its four register-held priorities, the LDS-slot resolver at
    P = 16) against the oracle."""
    from tests.families import FamilyCase

    case = FamilyCase("many_anti", 40000, 1500)
    orc = case.load(OracleScheduler(case.cfg))
    want, sw = orc.batch(case.batch, 4242)
    wc, wm = orc.read_requested()
    dev = case.load(DeviceScheduler(case.cfg, device=0))
    got, sg = dev.batch(case.batch, 4242)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches at {bad[:8]}: gpu {got[bad[:8]]} oracle {want[bad[:8]]}"
    assert sg == sw
    gc, gm = dev.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    assert dev.last_batch_stats()["windows"] > 0
    dev.close()


def test_config2_prefix_matches_faithful_restatement():
    """bench.py's cpu_baseline check as a test: the reference's own cost structure
    (faithful mode: per-pod MapPodsToMachines regroup, greedy CheckPodsExceedingCapacity,
    HostPriorityList sort) on the first 6,000 pods of BASELINE config 2 makes the same
    decisions as the GPU, from an empty cluster, with the same tie-break stream."""
    case = Case("config2", 5000, 6000)
    dev = DeviceScheduler(case.cfg, device=0)
    got, sg = run_batch(dev, case, chunk=1000)
    dev.close()
    orc = OracleScheduler(case.cfg, faithful=True)
    want, sw = run_batch(orc, case)
    orc.close()
    assert np.array_equal(got, want) and sg == sw


def test_config5_full_size_matches_oracle():
    """BASELINE config 5 at full size: 100k nodes x 100k pods in 1,000-pod batches,
    every decision, the RNG position and the committed totals against the
    incremental oracle (its node loop split over OMP_NUM_THREADS threads: ~15 s on
    the GPU box's host). Also the window path against the exact one-pod-at-a-time
    kernel (two different kernels), committed totals == the sum of the placed pods'
    requests, and no node with a capacity above it."""
    import os

    case = Case("config5", 100000, 100000)
    wind = DeviceScheduler(case.cfg, device=0)
    got, sg = run_batch(wind, case, chunk=1000)
    assert wind.last_batch_stats()["windows"] > 0
    gc, gm = wind.read_requested()
    wind.close()
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))
    orc = OracleScheduler(case.cfg)
    orc.set_cluster(case.view.arrays)
    want, sw = orc.batch_mt(case.batch, 1234, threads)
    wc, wm = orc.read_requested()
    orc.close()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"window vs oracle: first mismatches at {bad[:8]}: {got[bad[:8]]} vs {want[bad[:8]]}"
    assert sg == sw and np.array_equal(gc, wc) and np.array_equal(gm, wm)
    exact = DeviceScheduler(case.cfg, device=0)
    exact.set_window(0)
    ref, sr = run_batch(exact, case, chunk=1000)
    exact.close()
    assert np.array_equal(got, ref) and sg == sr
    ok = got >= 0
    assert ok.sum() > len(got) // 2
    sc, sm = np.zeros_like(gc), np.zeros_like(gm)
    np.add.at(sc, got[ok], case.batch.pods["milli_cpu"][ok].astype(np.int64))
    np.add.at(sm, got[ok], case.batch.pods["memory"][ok].astype(np.int64))
    assert np.array_equal(sc, gc) and np.array_equal(sm, gm)
    nodes = case.view.arrays.nodes
    cap_c, cap_m = nodes["cap_milli_cpu"].astype(np.int64), nodes["cap_memory"].astype(np.int64)
    assert ((cap_c == 0) | (gc <= cap_c)).all() and ((cap_m == 0) | (gm <= cap_m)).all()


def test_failed_batch_requires_resync_and_retry_is_accepted(monkeypatch):
    """A batch that fails after its device work started (injected: KSG_DEBUG &
    16384) leaves the context diverged: the retry with the same uids is refused
    with a message naming ksg_set_cluster, and after ksg_set_cluster the same
    pods schedule exactly as the oracle's (the deferred-replay stash
    used to keep the failed batch's uids)."""
    from kubernetes_amd.engine import KsgError

    case = Case("config2", 600, 300)
    monkeypatch.setenv("KSG_DEBUG", "16384")  # (read by ksg_set_cluster)
    dev = DeviceScheduler(case.cfg, device=0)
    dev.set_cluster(case.view.arrays)
    monkeypatch.delenv("KSG_DEBUG")
    with pytest.raises(KsgError, match="injected"):
        dev.batch(case.batch, 5)
    with pytest.raises(KsgError, match="ksg_set_cluster"):
        dev.batch(case.batch, 5)
    with pytest.raises(KsgError, match="ksg_set_cluster"):
        dev.remove_pod(int(case.batch.pods[0]["uid"]))
    dev.set_cluster(case.view.arrays)
    got, sg = dev.batch(case.batch, 5)
    orc = OracleScheduler(case.cfg)
    orc.set_cluster(case.view.arrays)
    want, sw = orc.batch(case.batch, 5)
    assert np.array_equal(got, want) and sg == sw
    dev.close()


def test_debug_counters_write_only_the_requested_words(monkeypatch):
    """ksg_debug_counters copies min(n_words, KSG_DEBUG_COUNTER_WORDS) words and
    zero-fills the rest of the caller's buffer, never past n_words (ABI version 3;
    VERDICT round 4 "silent ABI widening"): a short buffer keeps its canary tail,
    a long one gets the 64 stamped words then zeros. KSG_DEBUG=8 (the stamped
    resolver build) places exactly what the oracle places."""
    import ctypes as C
    case = Case("config2", 600, 400)
    monkeypatch.setenv("KSG_DEBUG", "8")  # (read by ksg_create / ksg_set_cluster)
    dev, orc = _pair(case)
    dev.set_cluster(case.view.arrays)
    monkeypatch.delenv("KSG_DEBUG")
    got, sg = dev.batch(case.batch, 5)
    orc.set_cluster(case.view.arrays)
    want, sw = orc.batch(case.batch, 5)
    assert np.array_equal(got, want) and sg == sw
    W = abi.KSG_DEBUG_COUNTER_WORDS
    full = dev.debug_counters()
    assert full.shape == (W,) and full.sum() > 0  # (the stamps ran)
    short = np.full(16, -7, np.int32)
    assert dev._lib.ksg_debug_counters(dev._ctx, abi.ptr(short), 8) == abi.KSG_OK
    assert np.array_equal(short[:8], full[:8]) and (short[8:] == -7).all()
    long_ = np.full(W + 16, -7, np.int32)
    assert dev._lib.ksg_debug_counters(dev._ctx, abi.ptr(long_), W + 8) == abi.KSG_OK
    assert np.array_equal(long_[:W], full) and (long_[W:W + 8] == 0).all() and (long_[W + 8:] == -7).all()
    assert dev._lib.ksg_debug_counters(dev._ctx, C.c_void_p(None), 0) == abi.KSG_OK
    dev.close()
