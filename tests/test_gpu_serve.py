"""The resident begin/commit server (ksg_serve.hip) against the C oracle.

ksg_schedule_begin / ksg_schedule_commit on one rank are served by a resident
workgroup polling mapped host memory. These sequences drive it through every
request kind and hand-over: begin + commit with fail codes, abandoned begins,
FitErrors, ksg_add_pod / ksg_remove_pod between pods (queued mirror patches
applied by the server), ksg_evaluate and ksg_schedule_batch in the middle (the
server leaves the stream and is relaunched), and an idle timeout short enough
that the server returns between requests, including between a begin and its
commit (the commit rescans the pod the host left in the request block). Every
result is compared with the oracle: return code, max score, tie count, fail
codes, chosen node, committed totals.
"""
import numpy as np
import pytest

from kubernetes_amd import abi
from kubernetes_amd.engine import DeviceScheduler, PodBatch
from oracle.pyoracle import OracleScheduler
from tests.helpers import Case

pytestmark = pytest.mark.gpu


def _drive(case, dev, orc, seed, n_pods, *, evaluate_every=0, batch_at=(), churn=0.0, abandon=0.1):
    rng = np.random.default_rng(seed)
    n = case.view.arrays.n_nodes
    live = []  # uids placed by commit / add_pod, removable
    i = 0
    while i < n_pods:
        if i in batch_at:  # a short batch through the window path in between
            sub = PodBatch(case.batch.pods[i:i + 40], case.batch.ids)
            g, sg = dev.batch(sub, 1234 + i)
            w, sw = orc.batch(sub, 1234 + i)
            assert np.array_equal(g, w) and sg == sw, f"batch at {i}"
            live.extend(int(case.batch.pods[i + q]["uid"]) for q in range(len(g)) if g[q] >= 0)
            i += 40
            continue
        if evaluate_every and i % evaluate_every == 0:
            rcg, fg, sg = dev.evaluate(case.batch, i)
            rco, fo, so = orc.evaluate(case.batch, i)
            assert rcg == rco and np.array_equal(fg, fo)
            assert np.array_equal(sg[fg == 0], so[fo == 0])
        if churn and rng.random() < churn:
            if live and rng.random() < 0.5:
                uid = live.pop(int(rng.integers(0, len(live))))
                dev.remove_pod(uid)
                orc.remove_pod(uid)
            else:  # an existing pod reported by the store (some hosts are not nodes)
                host = int(rng.integers(0, n + 3))
                dev.add_pod(host, case.batch, i)
                orc.add_pod(host, case.batch, i)
                live.append(int(case.batch.pods[i]["uid"]))
                i += 1
                continue
        want_fail = bool(rng.random() < 0.7)
        rg, mg, kg, fg = dev.begin(case.batch, i, want_fail=want_fail)
        ro, mo, ko, fo = orc.begin(case.batch, i, want_fail=want_fail)
        assert (rg, kg) == (ro, ko), f"pod {i}: gpu {(rg, kg)} oracle {(ro, ko)}"
        if want_fail:
            assert np.array_equal(fg, fo), f"pod {i}: fail codes"
        if rg == abi.KSG_OK:
            assert mg == mo, f"pod {i}: max score"
            if rng.random() < abandon:  # the next begin abandons this one
                i += 1
                continue
            ix = int(rng.integers(0, kg))
            ng, no = dev.commit(ix), orc.commit(ix)
            assert ng == no, f"pod {i}: node gpu {ng} oracle {no}"
            live.append(int(case.batch.pods[i]["uid"]))
        i += 1
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)


@pytest.mark.parametrize("name,nn,npods,grid", [
    ("config1", 500, 500, False),     # one workgroup, R = 1, register-cached totals
    ("config2", 2000, 500, False),    # R = 2
    ("config2", 2000, 500, True),     # the grid server: 8 scan workgroups
    ("config2", 5000, 500, False),    # R = 8 (config 2's node count)
    ("config2", 5000, 500, True),
    ("config4", 900, 400, False),     # ServiceAffinity + ServiceAntiAffinity
    ("config4", 900, 400, True),      # ... on the grid server: the domain counts exchanged (round 5)
    ("config4", 5000, 300, True),     # ... config 4's node count, 20 scan workgroups
    ("config3", 15000, 200, False),   # R = 16
    ("config3", 15000, 200, True),
    ("config2", 30000, 120, True),    # past the one-workgroup server's 16,384 nodes (4 nodes per thread)
    ("config5", 100000, 40, True),    # config 5's node count (98 scan workgroups of 1,024 nodes)
])
def test_serve_begin_commit_matches_oracle(name, nn, npods, grid, monkeypatch):
    monkeypatch.setenv("KSG_SERVE_GRID", "1" if grid else "0")
    case = Case(name, nn, npods)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    _drive(case, dev, orc, seed=nn + npods, n_pods=npods)
    st = dev.serve_stats()
    assert st["eligible"] and st["launches"] >= 1 and st["requests"] >= npods, st
    assert st["grid"] == grid, st
    dev.close()


@pytest.mark.parametrize("family,nn,npods,grid", [
    ("four_anti", 900, 300, True),   # 50 domains: the grid server, anti priorities past its two in registers
    ("four_anti", 3000, 200, True),  # (12 scan workgroups)
    ("many_anti", 900, 300, False),  # 84 domains > KSG_GSRV_MAXD: the one-workgroup server instead
])
def test_serve_anti_priorities_grid_or_fallback(family, nn, npods, grid, monkeypatch):
    """Several ServiceAntiAffinity priorities through begin / commit with the grid server
    asked for: up to KSG_GSRV_MAXD label domains it serves them, the
    priorities past KSG_GSRV_ANTI_REG loading their domains from HBM (ksg_serve.hip); past
    that many domains srv_grid() falls back to the one-workgroup server. Both match the oracle."""
    from tests.families import FamilyCase

    monkeypatch.setenv("KSG_SERVE_GRID", "1")
    case = FamilyCase(family, nn, npods)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    _drive(case, dev, orc, seed=nn + 3, n_pods=npods, churn=0.05)
    st = dev.serve_stats()
    assert st["eligible"] and st["requests"] >= npods, st
    assert st["grid"] == grid, st
    dev.close()


@pytest.mark.parametrize("name,nn,npods", [("config2", 1500, 400), ("config4", 700, 300), ("config2", 3000, 300)])
def test_serve_interleaved_with_add_remove_evaluate_batch(name, nn, npods):
    """Mirror patches through the server, and evaluate / batch taking the stream."""
    case = Case(name, nn, npods)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    _drive(case, dev, orc, seed=5, n_pods=npods, evaluate_every=37, batch_at=(100, 250), churn=0.2)
    st = dev.serve_stats()
    assert st["launches"] >= 3, st  # relaunched after each evaluate / batch
    dev.close()


@pytest.mark.parametrize("nn,grid", [(900, False), (900, True), (2500, True)])
def test_serve_idle_timeout_relaunch(nn, grid, monkeypatch):
    """A 1-us idle limit: the server returns between nearly every pair of
    requests, between a begin and its commit too (the relaunched server is
    offered every request after the last one the host saw served)."""
    monkeypatch.setenv("KSG_SERVE_IDLE_US", "1")
    monkeypatch.setenv("KSG_SERVE_GRID", "1" if grid else "0")
    case = Case("config2", nn, 300)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    _drive(case, dev, orc, seed=11, n_pods=300, churn=0.1)
    st = dev.serve_stats()
    assert st["launches"] > 100, st
    dev.close()


def test_serve_matches_launch_per_call_path(monkeypatch):
    """KSG_SERVE=0 (round-2 path: scan + decide launches) and the server agree."""
    case = Case("config2", 3000, 300)
    devs = []
    for serve in ("1", "0"):
        monkeypatch.setenv("KSG_SERVE", serve)
        d = DeviceScheduler(case.cfg, device=0)
        d.set_cluster(case.view.arrays)
        devs.append(d)
    assert devs[0].serve_stats()["eligible"] and not devs[1].serve_stats()["eligible"]
    rng = np.random.default_rng(2)
    for i in range(300):
        a = devs[0].begin(case.batch, i, want_fail=True)
        b = devs[1].begin(case.batch, i, want_fail=True)
        assert a[:3] == b[:3] and np.array_equal(a[3], b[3])
        if a[0] == abi.KSG_OK:
            ix = int(rng.integers(0, a[2]))
            assert devs[0].commit(ix) == devs[1].commit(ix)
    for d in devs:
        d.close()


@pytest.mark.parametrize("name,nn,npods,churn", [("config2", 2000, 300, 0.0), ("config1", 700, 300, 0.2),
                                                 ("config2", 5000, 200, 0.1), ("config4", 3000, 250, 0.1)])
def test_serve_grid_four_nodes_per_thread(name, nn, npods, churn, monkeypatch):
    """The grid server's 4-nodes-per-thread scan workgroups (the default past
    16,384 nodes) forced at small sizes: partial last workgroups, fail codes,
    tie words past the 64-B part, patches in between."""
    monkeypatch.setenv("KSG_SERVE_GRID_NPT4_MIN", "0")
    case = Case(name, nn, npods)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    _drive(case, dev, orc, seed=nn, n_pods=npods, churn=churn)
    st = dev.serve_stats()
    assert st["grid"] and st["requests"] >= npods, st
    dev.close()


@pytest.mark.parametrize("name,nn,grid", [("config2", 900, False), ("config4", 700, False), ("config2", 2500, True)])
def test_serve_pending_begin_survives_stream_users(name, nn, grid, monkeypatch):
    """Calls that take the stream between a server-served begin and its commit
    (read_requested, kubelet admission, a rejected evaluate / batch) stop the
    server; the commit must still apply the pending pod on the node the begin's
    tie words give (srv_stop dropped the pending begin and the
    commit ran the launch-per-call decide on stale device records)."""
    from kubernetes_amd.engine import KsgError

    monkeypatch.setenv("KSG_SERVE_GRID", "1" if grid else "0")
    case = Case(name, nn, 120)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    rng = np.random.default_rng(nn)
    sets = np.zeros(1, abi.ADMISSION_SET_DTYPE)
    sets[0]["n_pods"] = 1  # pod 0 against an unlimited capacity
    one = PodBatch(case.batch.pods[:1], case.batch.ids)
    for i in range(120):
        rg, mg, kg, _ = dev.begin(case.batch, i)
        ro, mo, ko, _ = orc.begin(case.batch, i)
        assert (rg, kg) == (ro, ko), f"pod {i}"
        if rg != abi.KSG_OK:
            continue
        assert mg == mo
        kind = i % 4
        if kind == 0:
            dev.read_requested()
        elif kind == 1:
            assert dev.admit(sets, one, np.zeros(0, np.uint32), 1)[0] == 1
        elif kind == 2:
            with pytest.raises(KsgError, match="pending"):
                dev.evaluate(case.batch, i)
        else:
            with pytest.raises(KsgError, match="pending"):
                dev.batch(PodBatch(case.batch.pods[i + 1:i + 3], case.batch.ids), 7)
        ix = int(rng.integers(0, kg))
        assert dev.commit(ix) == orc.commit(ix), f"pod {i}"
        gc, gm = dev.read_requested()
        wc, wm = orc.read_requested()
        assert np.array_equal(gc, wc) and np.array_equal(gm, wm), f"pod {i}: committed totals"
    assert dev.serve_stats()["eligible"]
    dev.close()


@pytest.mark.parametrize("grid", [False, True])
def test_serve_commit_then_idle_exit(grid, monkeypatch):
    """A commit answered inside the idle window, then a pause longer than the idle
    limit, then a begin: the relaunched server must not be offered the answered
    COMMIT again (the one-workgroup server applied it twice)."""
    import time

    monkeypatch.setenv("KSG_SERVE_IDLE_US", "2000")
    monkeypatch.setenv("KSG_SERVE_GRID", "1" if grid else "0")
    case = Case("config2", 1200, 40)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    orc.set_cluster(case.view.arrays)
    rng = np.random.default_rng(3)
    for i in range(40):
        rg, _, kg, _ = dev.begin(case.batch, i)
        ro, _, ko, _ = orc.begin(case.batch, i)
        assert (rg, kg) == (ro, ko), f"pod {i}"
        if rg == abi.KSG_OK:
            ix = int(rng.integers(0, kg))
            assert dev.commit(ix) == orc.commit(ix), f"pod {i}"
        time.sleep(0.01)  # > KSG_SERVE_IDLE_US: the server answers the commit, then returns
    gc, gm = dev.read_requested()
    wc, wm = orc.read_requested()
    assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    assert dev.serve_stats()["launches"] > 20
    dev.close()


@pytest.mark.parametrize("grid", [False, True])
def test_serve_rejects_malformed_requests(grid, monkeypatch):
    """A BEGIN and a COMMIT whose payload layout is out of range (KSG_DEBUG bits 23
    / 22 corrupt the next one the host posts) are rejected by the server's layout
    check (req_bad) instead of being read: the begin fails with KSG_ERR_STATE and
    the context stays usable; the rejected commit (posted without waiting) is
    reported by the next call and leaves the context diverged until
    ksg_set_cluster, after which scheduling matches the oracle again (round 3's
    illegal-address faults in both servers came from request payloads read
    outside their layout; ADVICE r3: a rejected commit must diverge the context)."""
    from kubernetes_amd.engine import KsgError

    monkeypatch.setenv("KSG_SERVE_GRID", "1" if grid else "0")
    case = Case("config2", 1500, 60)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    monkeypatch.setenv("KSG_DEBUG", str((1 << 22) | (1 << 23)))  # (read by ksg_set_cluster)
    dev.set_cluster(case.view.arrays)
    monkeypatch.delenv("KSG_DEBUG")
    orc.set_cluster(case.view.arrays)
    with pytest.raises(KsgError, match="rejected begin"):
        dev.begin(case.batch, 0)
    rg, _, kg, _ = dev.begin(case.batch, 0)  # the same pod again: served
    ro, _, ko, _ = orc.begin(case.batch, 0)
    assert (rg, kg) == (ro, ko) and rg == abi.KSG_OK
    dev.commit(0)  # corrupted on the way: rejected by the server, reported by the next call
    with pytest.raises(KsgError, match="rejected commit"):
        dev.begin(case.batch, 1)
    with pytest.raises(KsgError, match="ksg_set_cluster"):
        dev.begin(case.batch, 1)
    dev.set_cluster(case.view.arrays)
    _drive(case, dev, orc, seed=1, n_pods=60, abandon=0.0)
    dev.close()
