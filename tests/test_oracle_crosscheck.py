"""Cross-checks the two oracle layers on whole scheduling sequences.

ref_model (object-level Python transcription, pinned by tests/golden) vs the C
restatement (oracle/ksg_oracle.c, driven through the product ingest), then the C
restatement's faithful mode (MapPodsToMachines regroup + greedy capacity check +
sort, as the reference) vs its incremental mode (closed forms) at larger sizes.
Every successful pod is assumed on its host before the next one, as
scheduleOne + AssumePod do (plugin/pkg/scheduler/scheduler.go:86-118).
"""
import copy

import numpy as np
import pytest

from kubernetes_amd import abi, factory, ingest, workload
from kubernetes_amd.api import Pod, PodStatus
from kubernetes_amd.scheduler import SplitMix64Rand
from oracle import ref_model as R
from oracle.pyoracle import OracleScheduler
from tests import families
from tests.families import FAMILIES
from tests.helpers import Case


def _policy_labels():
    """Exercises LabelsPresence + LabelPreference + weights != 1 (plugins.go:81-183)."""
    return factory.create_from_config({
        "predicates": [{"name": "PodFitsResources"}, {"name": "MatchNodeSelector"},
                       {"name": "HasZone", "argument": {"labelsPresence": {"labels": ["zone"], "presence": True}}},
                       {"name": "NoK9", "argument": {"labelsPresence": {"labels": ["k9"], "presence": False}}}],
        "priorities": [{"name": "LeastRequestedPriority", "weight": 1},
                       {"name": "PreferRackLabel", "weight": 3,
                        "argument": {"labelPreference": {"label": "rack", "presence": True}}},
                       {"name": "AvoidK0", "weight": 2,
                        "argument": {"labelPreference": {"label": "k0", "presence": False}}},
                       {"name": "ZoneSpreadX", "weight": 2,
                        "argument": {"serviceAntiAffinity": {"label": "rack"}}}],
    })


# LabelPreference priorities and single-key LabelsPresence predicates of _policy_many_labels:
# past two slot passes' worth of the config's slots (ksg_add_static_config runs two passes)
N_PREF = 2 * abi.MAX_LABEL_PREF + 4
N_U = 2 * abi.MAX_PRESENCE + 1


def _policy_many_labels():
    """More LabelsPresence predicates / keys and LabelPreference priorities than
    ksg_config's slots: the rest are evaluated on the device in slot passes
    (ksg_add_static_config)."""
    preds = [{"name": "PodFitsResources"}, {"name": "MatchNodeSelector"},
             {"name": "HasZone", "argument": {"labelsPresence": {"labels": ["zone"], "presence": True}}},
             {"name": "HasRegionRack", "argument": {"labelsPresence": {"labels": ["region", "rack"], "presence": True}}},
             # one key past a slot's keys in one predicate
             {"name": "NoA", "argument": {"labelsPresence": {"labels": [f"a{j}" for j in range(abi.MAX_PRESENCE_KEYS + 1)],
                                                            "presence": False}}}]
    preds += [{"name": f"NoU{j:02d}", "argument": {"labelsPresence": {"labels": [f"u{j}"], "presence": False}}}
              for j in range(N_U)]
    prios = [{"name": "LeastRequestedPriority", "weight": 1}]
    prios += [{"name": f"Pref{j:02d}", "weight": 1 + j % 5,
               "argument": {"labelPreference": {"label": f"t{j}", "presence": j % 3 != 0}}}
              for j in range(N_PREF)]
    return factory.create_from_config({"predicates": preds, "priorities": prios})


def _workload(name, nn, npods, tight=False, existing=0, seed=7):
    if name == "policy_many_labels":
        rng = workload._SM(seed)
        nodes = workload.make_nodes(nn, rng, dense_labels=2)
        for i, n in enumerate(nodes):  # t_j on every (j + 2)-th node; u_j, a4 on a few
            for j in range(N_PREF):
                if i % (j + 2) == 0:
                    n.metadata.labels[f"t{j}"] = "x"
            for j in range(N_U):
                if i % (j + 23) == 7:
                    n.metadata.labels[f"u{j}"] = "x"
            if i % 13 == 5:
                n.metadata.labels["a4"] = "y"
        pods = workload.make_pods(npods, rng, n_apps=10)
        w = workload.Workload(name, nodes, pods, workload.make_services(10), _policy_many_labels(), [])
    elif name == "policy_labels":
        rng = workload._SM(seed)
        nodes = workload.make_nodes(nn, rng, dense_labels=2)
        for i, n in enumerate(nodes):  # some nodes lack zone / carry k9
            if i % 7 == 0:
                n.metadata.labels.pop("zone")
            if i % 11 == 0:
                n.metadata.labels["k9"] = "x"
        pods = workload.make_pods(npods, rng, n_apps=10)
        w = workload.Workload(name, nodes, pods, workload.make_services(10), _policy_labels(), [])
    else:
        w = workload.build(name, n_nodes=nn, n_pods=npods, seed=seed)
    if tight:  # small nodes: FitErrors and cap-exceeding LeastRequested inputs
        for n in w.nodes:
            n.spec.capacity["cpu"] = n.spec.capacity["cpu"].__class__.from_milli(1500)
    if existing:
        w.existing = w.pods[:existing]
        w.pods = w.pods[existing:]
        names = [n.metadata.name for n in w.nodes]
        for i, p in enumerate(w.existing):
            p.status = PodStatus(host=names[(i * 7) % len(names)] if i % 5 else "gone-node")
    return w


def _ref_sequence(w, rng_seed):
    lister = R.PodLister(list(w.existing))
    svcs = R.ServiceLister(w.services)
    preds, prios = R.from_config(w.config, w.nodes, lister, svcs)
    rnd = SplitMix64Rand(rng_seed)
    sched = R.GenericScheduler(preds, prios, lister, rnd)
    out = []
    for p in w.pods:
        try:
            host = sched.schedule(p, w.nodes)
        except R.FitError:
            out.append(("nofit", None))
            continue
        except KeyError:
            out.append(("error", None))
            continue
        q = copy.copy(p)
        q.status = PodStatus(host=host)
        lister.pods.append(q)  # AssumePod
        out.append(("ok", host))
    return out, rnd.state


def _c_sequence(w, rng_seed, faithful):
    it = ingest.Interner()
    for k in w.config.label_keys():
        it.key_id(k)
    view = ingest.ClusterView(w.nodes, w.services, it)
    aff = w.config.affinity_labels()
    orc = OracleScheduler(w.config.compile(it.key_id), faithful=faithful)
    orc.set_cluster(view.arrays)
    if w.existing:
        b = ingest.ingest_pods(view, w.existing, aff_labels=aff)
        for i, p in enumerate(w.existing):
            orc.add_pod(view.host_id(p.status.host), b, i)
    batch = ingest.ingest_pods(view, w.pods, uids=list(range(10 ** 6, 10 ** 6 + len(w.pods))), aff_labels=aff)
    out, st = orc.batch(batch, rng_seed)
    orc.close()
    res = []
    for o in out:
        if o >= 0:
            res.append(("ok", view.names[o]))
        elif o == abi.KSG_OUT_NOFIT:
            res.append(("nofit", None))
        else:
            res.append(("error", None))
    return res, st


@pytest.mark.parametrize("name,nn,npods,tight,existing", [
    ("config1", 40, 120, False, 0),
    ("config1", 12, 80, True, 0),
    ("config2", 50, 150, False, 0),
    ("config2", 30, 120, True, 30),
    ("config4", 48, 150, False, 0),
    ("config4", 32, 120, True, 20),
    ("policy_labels", 40, 120, False, 0),
    ("policy_labels", 24, 100, True, 15),
])
def test_ref_model_vs_c_oracle(name, nn, npods, tight, existing):
    w = _workload(name, nn, npods, tight, existing)
    want, st_w = _ref_sequence(w, 99)
    for faithful in (True, False):
        got, st_g = _c_sequence(w, 99, faithful)
        bad = [i for i in range(len(want)) if want[i] != got[i]]
        assert not bad, f"faithful={faithful} first mismatches {[(i, want[i], got[i]) for i in bad[:5]]}"
        assert st_g == st_w
    if tight:
        assert any(k == "nofit" for k, _ in want)


@pytest.mark.parametrize("name,nn,npods", [("config2", 400, 1200), ("config4", 300, 900), ("config1", 500, 1000)])
def test_faithful_vs_incremental(name, nn, npods):
    c = Case(name, nn, npods)
    a = OracleScheduler(c.cfg, faithful=True)
    b = OracleScheduler(c.cfg, faithful=False)
    for o in (a, b):
        o.set_cluster(c.view.arrays)
    oa, sa = a.batch(c.batch, 5)
    ob, sb = b.batch(c.batch, 5)
    assert np.array_equal(oa, ob) and sa == sb
    ra, rb = a.read_requested(), b.read_requested()
    assert all(np.array_equal(x, y) for x, y in zip(ra, rb))


@pytest.mark.parametrize("family", FAMILIES)
def test_families_ref_model_vs_c_oracle(family):
    """tests/families.py: overlapping services, two namespaces, negative and large
    weights, pre-existing pods on "" / unknown hosts, invalid ServiceAffinity values."""
    w = families.build(family, 40, 110)
    want, st_w = _ref_sequence(w, 31)
    for faithful in (True, False):
        got, st_g = _c_sequence(w, 31, faithful)
        bad = [i for i in range(len(want)) if want[i] != got[i]]
        assert not bad, f"faithful={faithful} first mismatches {[(i, want[i], got[i]) for i in bad[:5]]}"
        assert st_g == st_w
    assert sum(k == "ok" for k, _ in want) > len(want) // 2


@pytest.mark.parametrize("name,nn,npods,threads", [("config2", 700, 1500, 4), ("config1", 500, 1000, 8),
                                                     ("config2", 130, 600, 3)])
def test_incremental_node_sharded_threads(name, nn, npods, threads):
    """The nproc-thread CPU baseline (orc_schedule_batch_mt, node-rank shards per pod)
    makes the single-threaded incremental restatement's decisions."""
    c = Case(name, nn, npods)
    a = OracleScheduler(c.cfg)
    b = OracleScheduler(c.cfg)
    for o in (a, b):
        o.set_cluster(c.view.arrays)
    oa, sa = a.batch(c.batch, 11)
    ob, sb = b.batch_mt(c.batch, 11, threads)
    assert np.array_equal(oa, ob) and sa == sb
    assert all(np.array_equal(x, y) for x, y in zip(a.read_requested(), b.read_requested()))
