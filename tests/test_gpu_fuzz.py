"""Randomised GPU parity: many small seeded clusters that stress the window
resolver's corner cases against the C oracle, bit-exact.

Knobs drawn per case: node count (incl. one or two 64-node words), tight
capacities (FitErrors, requested > capacity), dense host ports / GCE PDs (key
conflicts between pods of one window), few services (service flags, maxCount
changes, ServiceAffinity peers), zero-request pods, and every policy family
(DefaultProvider, resources only, ServiceAffinity + ServiceAntiAffinity,
LabelsPresence / LabelPreference / anti-affinity with weights). Each case runs
at windows 0 (exact kernel), 5, 64 and 128.
"""
import numpy as np
import pytest

from kubernetes_amd import factory, ingest, workload
from kubernetes_amd.api import Quantity
from kubernetes_amd.engine import DeviceScheduler
from oracle.pyoracle import OracleScheduler
from tests.families import FAMILIES, FamilyCase

pytestmark = pytest.mark.gpu

POLICIES = {
    "default": workload.config_default,
    "basic": workload.config1,
    "config4": workload.config4,
    "labels": lambda: factory.create_from_config({
        "predicates": [{"name": "PodFitsResources"}, {"name": "PodFitsPorts"}, {"name": "MatchNodeSelector"},
                       {"name": "HasZone", "argument": {"labelsPresence": {"labels": ["zone"], "presence": True}}}],
        "priorities": [{"name": "LeastRequestedPriority", "weight": 2},
                       {"name": "ServiceSpreadingPriority", "weight": 3},
                       {"name": "PreferRack", "weight": 1,
                        "argument": {"labelPreference": {"label": "rack", "presence": True}}},
                       {"name": "RackSpread", "weight": 2, "argument": {"serviceAntiAffinity": {"label": "rack"}}}],
    }),
}


def _case(seed):
    rng = workload._SM(1000 + seed)
    nn = [40, 64, 65, 130, 700, 2100][rng.below(6)]
    npods = 150 + rng.below(250)
    policy = list(POLICIES)[seed % len(POLICIES)]
    n_apps = [1, 3, 10, 40][rng.below(4)]
    port_frac = [0.0, 0.1, 0.6][rng.below(3)]
    pd_frac = [0.0, 0.05, 0.5][rng.below(3)]
    sel_frac = [0.0, 0.2, 0.7][rng.below(3)]
    tight = rng.below(3) == 0
    nodes = workload.make_nodes(nn, rng)
    if tight:
        for n in nodes:
            n.spec.capacity["cpu"] = Quantity.from_milli(1000 + 500 * rng.below(4))
    pods = workload.make_pods(npods, rng, n_apps=n_apps, port_frac=port_frac, pd_frac=pd_frac, sel_frac=sel_frac)
    for i, p in enumerate(pods):  # some zero-request pods (fit anywhere, predicates.go:129-132)
        if rng.below(20) == 0:
            c = p.spec.containers[0]
            c.resources.limits["cpu"] = Quantity.from_milli(0)
            c.resources.limits["memory"] = Quantity.from_int(0)
    for p in pods:  # dense keys: a small pool so pods of one window collide
        for c in p.spec.containers:
            for cp in c.ports:
                cp.host_port = 9000 + (cp.host_port % 3)
        for v in p.spec.volumes:
            if v.gce_persistent_disk is not None:
                v.gce_persistent_disk.pd_name = f"pd-{int(v.gce_persistent_disk.pd_name.split('-')[1]) % 5}"
    cfg = POLICIES[policy]()
    cfg.max_conflict_keys = 64
    w = workload.Workload(f"fuzz{seed}", nodes, pods, workload.make_services(n_apps), cfg, [])
    it = ingest.Interner()
    for k in w.config.label_keys():
        it.key_id(k)
    view = ingest.ClusterView(w.nodes, w.services, it)
    batch = ingest.ingest_pods(view, w.pods, aff_labels=w.config.affinity_labels())
    return w.config.compile(it.key_id), view.arrays, batch, (nn, npods, policy, n_apps, port_frac, pd_frac, tight)


@pytest.mark.parametrize("seed", range(64))
def test_fuzz_windows_match_oracle(seed):
    cfg, arrays, batch, desc = _case(seed)
    orc = OracleScheduler(cfg)
    orc.set_cluster(arrays)
    want, sw = orc.batch(batch, 4242 + seed)
    wc, wm = orc.read_requested()
    for window in (0, 5, 64, 128):
        dev = DeviceScheduler(cfg, device=0)
        dev.set_window(window)
        dev.set_cluster(arrays)
        got, sg = dev.batch(batch, 4242 + seed)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"{desc} window {window}: first mismatches at {bad[:6]}: {got[bad[:6]]} vs {want[bad[:6]]}"
        assert sg == sw, (desc, window)
        gc, gm = dev.read_requested()
        assert np.array_equal(gc, wc) and np.array_equal(gm, wm), (desc, window)
        dev.close()


# ---- input families the BASELINE configs never produce (tests/families.py) ----------
@pytest.mark.parametrize("family", FAMILIES)
def test_family_windows_match_oracle(family):
    case = FamilyCase(family, 700, 500)
    orc = case.load(OracleScheduler(case.cfg))
    want, sw = orc.batch(case.batch, 777)
    wc, wm = orc.read_requested()
    assert (want >= 0).sum() > len(want) // 2
    for window in (0, 5, 64, 128):
        dev = case.load(DeviceScheduler(case.cfg, device=0))
        dev.set_window(window)
        got, sg = dev.batch(case.batch, 777)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"{family} window {window}: first mismatches at {bad[:6]}: {got[bad[:6]]} vs {want[bad[:6]]}"
        assert sg == sw, (family, window)
        gc, gm = dev.read_requested()
        assert np.array_equal(gc, wc) and np.array_equal(gm, wm), (family, window)
        if family in ("many_anti", "past_caps") and window:
            # six / twenty ServiceAntiAffinity priorities: the window path (phase A keeps the
            # first four priorities' domains in registers and loads the rest)
            assert dev.last_batch_stats()["windows"] > 0, (family, window)
        if family == "negative" and window:
            # negative LeastRequested / ServiceSpreading weights break the window path's
            # monotonicity: every batch must have taken the exact kernel
            assert dev.last_batch_stats()["windows"] == 0
        dev.close()


# ---- interleavings: the resolver's waves hand off through LDS flags, so a
# missing wait would show up only under some interleaving (a single drawn-node
# mailbox the committer could overwrite while running ahead through no-commit
# pods differed in ~1 of 5 runs of `namespaces` in round 2). Instead of
# repeating runs, each case runs once per fixed delay pattern: KSG_DEBUG bits
# 16..19 make one wave role (committer, x-checker, checkers, producers) sleep
# ~512 cycles per pod (ksg_plain.hip; round 4: also the ServiceAntiAffinity
# resolvers of ksg_window.hip, the register-slot re-rank and the LDS-slot one),
# which pushes every hand-off onto its other side (the role that is usually
# ahead falls behind, and vice versa)
_SKEWS = (0, 1, 2, 4, 8, 1 | 4, 2 | 8, 2 | 4)


@pytest.mark.parametrize("family", FAMILIES)
def test_family_interleavings_match_oracle(family, monkeypatch):
    case = FamilyCase(family, 700, 500)
    orc = case.load(OracleScheduler(case.cfg))
    want, _ = orc.batch(case.batch, 777)
    for window in (5, 64):
        for skew in _SKEWS:
            monkeypatch.setenv("KSG_DEBUG", str(skew << 16))  # (read by ksg_set_cluster)
            dev = case.load(DeviceScheduler(case.cfg, device=0))
            dev.set_window(window)
            got, _ = dev.batch(case.batch, 777)
            dev.close()
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, f"{family} window {window} skew {skew}: first mismatches at {bad[:6]}"


@pytest.mark.parametrize("seed", range(0, 64, 4))
def test_fuzz_interleavings_match_oracle(seed, monkeypatch):
    cfg, arrays, batch, desc = _case(seed)
    orc = OracleScheduler(cfg)
    orc.set_cluster(arrays)
    want, _ = orc.batch(batch, 4242 + seed)
    for window in (5, 64):
        for skew in _SKEWS[::2] if seed % 8 else _SKEWS:
            monkeypatch.setenv("KSG_DEBUG", str(skew << 16))
            dev = DeviceScheduler(cfg, device=0)
            dev.set_window(window)
            dev.set_cluster(arrays)
            got, _ = dev.batch(batch, 4242 + seed)
            dev.close()
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, f"{desc} window {window} skew {skew}: first mismatches at {bad[:6]}"


@pytest.mark.parametrize("resolver", ["rerank", "ldsslot"])
def test_anti_affinity_resolver_interleavings_match_oracle(resolver, monkeypatch):
    """Config 4's ServiceAffinity + ServiceAntiAffinity at 900 nodes under every
    skew: the register-slot re-rank resolver (ksg_win_resolve2_kernel<..., ANTI>)
    and, with KSG_DEBUG & 4096, the LDS-slot one (ksg_win_resolve_kernel)."""
    from tests.helpers import Case

    case = Case("config4", 900, 600)
    orc = OracleScheduler(case.cfg)
    orc.set_cluster(case.view.arrays)
    want, sw = orc.batch(case.batch, 31)
    extra = 4096 if resolver == "ldsslot" else 0
    for window in (5, 64, 128):
        for skew in _SKEWS:
            monkeypatch.setenv("KSG_DEBUG", str((skew << 16) | extra))
            dev = DeviceScheduler(case.cfg, device=0)
            dev.set_window(window)
            dev.set_cluster(case.view.arrays)
            got, sg = dev.batch(case.batch, 31)
            windows = dev.last_batch_stats()["windows"]
            dev.close()
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, f"{resolver} window {window} skew {skew}: first mismatches at {bad[:6]}"
            assert sg == sw and windows > 0
