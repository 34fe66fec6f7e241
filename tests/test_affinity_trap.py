"""ServiceAffinity under SelectorFromSet's invalid-label trap.

CheckServiceAffinity builds its selector with labels.Set(affinityLabels).AsSelector()
(pkg/scheduler/predicates.go:311-315) -> SelectorFromSet (pkg/labels/labels.go:60-61),
which returns the EMPTY selector -- matching every node -- as soon as one key fails
IsQualifiedName or one value fails IsValidLabelValue (pkg/labels/selector.go:654-668,
NewRequirement :91-115). The affinity map takes each label's value from the pod's own
nodeSelector, else from the node of the first service peer (:261-307), so the trap can
come from either side, and it applies per ServiceAffinity predicate.

The reference's own tables (TestServiceAffinity, predicates_test.go:466-603) never hold
an invalid value, so these rows are derived from the cited reference code; the expected
fit sets are written out by hand and every engine must give them: the object-level
restatement (oracle/ref_model.py), the C restatement in both modes through the product
ingest, and the HIP library through the C ABI (-m gpu).
"""
import re

import pytest

from kubernetes_amd import abi, factory
from kubernetes_amd.api import ObjectMeta, Pod, PodSpec, PodStatus, Service, ServiceSpec, make_node
from oracle import ref_model as R
from oracle.pyoracle import OracleScheduler
from tests.golden_util import run_engine

SEL = {"app": "web"}


def _node(name, **labels):
    return make_node(name, 4000, 8 << 30, labels=labels or None)


def _pod(name="", node_selector=None, status_host="", labels=SEL):
    return Pod(metadata=ObjectMeta(name=name, namespace="ns", labels=dict(labels) if labels else None),
               spec=PodSpec(node_selector=node_selector), status=PodStatus(host=status_host))


def _cfg(*groups):
    preds = [{"name": "trap-aff-" + "-".join(re.sub("[^a-zA-Z0-9]", "", l) for l in g),
              "argument": {"serviceAffinity": {"labels": list(g)}}} for g in groups]
    return factory.create_from_config({"predicates": preds,
                                       "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]})


NODES3 = [_node("n1", region="r1", zone="z1"), _node("n2", region="r2", zone="z2"),
          _node("n3", region="r1", zone="z2")]
SVC = [Service(metadata=ObjectMeta(name="web", namespace="ns"), spec=ServiceSpec(selector=SEL))]

# (id, groups, nodes, existing pods, pod, expected fitting node names)
CASES = [
    ("valid-control", [("region",)], NODES3, [], _pod(node_selector={"region": "r1"}), {"n1", "n3"}),
    ("pod-invalid-value", [("region",)], NODES3, [], _pod(node_selector={"region": "bad value!"}),
     {"n1", "n2", "n3"}),
    ("pod-invalid-value-two-nodes", [("region",)], NODES3[:2], [], _pod(node_selector={"region": "bad value!"}),
     {"n1", "n2"}),
    ("peer-invalid-value", [("region",)],
     [_node("n1", region="bad value!"), _node("n2", region="r2"), _node("n3", region="r1")],
     [_pod("peer", status_host="n1")], _pod(), {"n1", "n2", "n3"}),
    ("peer-valid-control", [("region",)], NODES3, [_pod("peer", status_host="n2")], _pod(), {"n2"}),
    # one predicate over two labels: the pod's invalid region empties the whole selector
    ("mixed-one-predicate", [("region", "zone")], NODES3, [_pod("peer", status_host="n2")],
     _pod(node_selector={"region": "bad!"}), {"n1", "n2", "n3"}),
    # two predicates: only the one holding the invalid value matches everything
    ("mixed-two-predicates", [("region",), ("zone",)], NODES3, [],
     _pod(node_selector={"region": "bad!", "zone": "z2"}), {"n2", "n3"}),
    ("mixed-two-predicates-peer", [("region",), ("zone",)],
     [_node("n1", region="r1", zone="z1"), _node("n2", region="r2", zone="bad zone!"),
      _node("n3", region="r2", zone="z1")],
     [_pod("peer", status_host="n2")], _pod(), {"n2", "n3"}),
    # a label in two predicates: still required through the valid one
    ("shared-label", [("region", "zone"), ("zone",)], NODES3, [],
     _pod(node_selector={"region": "bad!", "zone": "z2"}), {"n2", "n3"}),
    # an invalid label KEY in the Policy: any affinity map holding it is rejected
    ("invalid-policy-key-pod", [("bad key!",)], [_node("n1"), _node("n2")], [],
     _pod(node_selector={"bad key!": "x"}), {"n1", "n2"}),
    ("invalid-policy-key-peer", [("bad key!",)],
     [make_node("n1", 4000, 8 << 30, labels={"bad key!": "x"}), _node("n2")],
     [_pod("peer", status_host="n1")], _pod(), {"n1", "n2"}),
    # no selector value, no peer: Everything()
    ("no-peer", [("region",)], NODES3, [], _pod(), {"n1", "n2", "n3"}),
]


def _ref_fits(groups, nodes, existing, pod):
    cfg = _cfg(*groups)
    lister = R.PodLister(existing)
    preds, _ = R.from_config(cfg, nodes, lister, R.ServiceLister(SVC))
    filtered, _ = R.find_nodes_that_fit(pod, lister, preds, nodes)
    return {n.metadata.name for n in filtered}


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_ref_model(case):
    _, groups, nodes, existing, pod, want = case
    assert _ref_fits(groups, nodes, existing, pod) == want


def _oracle(faithful):
    return lambda cfg: OracleScheduler(cfg, faithful=faithful)


def _device(cfg):
    from kubernetes_amd.engine import DeviceScheduler

    return DeviceScheduler(cfg, device=0)


ENGINES = [pytest.param(_oracle(True), id="oracle-faithful"), pytest.param(_oracle(False), id="oracle-incremental"),
           pytest.param(_device, id="hip", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_engines(engine, case):
    _, groups, nodes, existing, pod, want = case
    rc, got = run_engine(engine, _cfg(*groups), nodes, existing, SVC, pod)
    assert rc == abi.KSG_OK
    fits = {h for h, (f, _) in got.items() if f == abi.FAIL_NONE}
    assert fits == want, got
    assert all(f in (abi.FAIL_NONE, abi.FAIL_SERVICEAFFINITY) for f, _ in got.values())


def test_groups_compiled():
    cfg = _cfg(("region",), ("zone",), ("region", "zone")).compile(lambda k: {"region": 0, "zone": 1}[k])
    assert cfg.n_aff_labels == 2
    assert sorted(cfg.aff_group_mask[g] for g in range(cfg.n_aff_groups)) == [1, 2, 3]
