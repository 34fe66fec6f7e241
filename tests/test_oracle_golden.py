"""Pins the object-level restatement (oracle/ref_model.py) and the host ingest helpers
(kubernetes_amd.resource / labels) to the reference's own test tables
(tests/golden/*.json, restated by tests/golden/make_golden.py)."""
from fractions import Fraction

import pytest

from kubernetes_amd import labels as L
from kubernetes_amd.api import Node, ObjectMeta, Pod
from kubernetes_amd.resource import QuantityError, parse_quantity
from kubernetes_amd.scheduler import SplitMix64Rand
from oracle import ref_model as R
from tests.golden_util import load, mk_node, mk_pod, mk_service

G = load("scheduler_golden.json")
Q = load("quantity_golden.json")
LB = load("labels_golden.json")


def _ids(sec):
    return [c.get("test", c.get("name", str(i))) for i, c in enumerate(G[sec])]


# ---- priorities -------------------------------------------------------------------
@pytest.mark.parametrize("c", G["least_requested"], ids=_ids("least_requested"))
def test_least_requested(c):
    nodes = [mk_node(n) for n in c["nodes"]]
    got = R.least_requested_priority(mk_pod(c["pod"]), R.PodLister([mk_pod(p) for p in c["pods"]]), nodes)
    assert [list(x) for x in got] == c["expected"]  # reflect.DeepEqual: node order


@pytest.mark.parametrize("c", G["node_label_priority"], ids=_ids("node_label_priority"))
def test_node_label_priority(c):
    nodes = [mk_node(n) for n in c["nodes"]]
    fn = R.new_node_label_priority(c["label"], c["presence"])
    got = fn(Pod(), R.PodLister([]), nodes)
    assert sorted(map(list, got)) == sorted(c["expected"])


@pytest.mark.parametrize("c", G["service_spread"], ids=_ids("service_spread"))
def test_service_spread(c):
    fn = R.new_service_spread_priority(R.ServiceLister([mk_service(s, i) for i, s in enumerate(c["services"])]))
    got = fn(mk_pod(c["pod"]), R.PodLister([mk_pod(p) for p in c["pods"]]), [mk_node(n) for n in c["nodes"]])
    assert [list(x) for x in got] == c["expected"]


@pytest.mark.parametrize("c", G["zone_spread"], ids=_ids("zone_spread"))
def test_zone_spread(c):
    fn = R.new_service_anti_affinity_priority(
        R.ServiceLister([mk_service(s, i) for i, s in enumerate(c["services"])]), "zone")
    got = fn(mk_pod(c["pod"]), R.PodLister([mk_pod(p) for p in c["pods"]]), [mk_node(n) for n in c["nodes"]])
    assert sorted(map(list, got)) == sorted(c["expected"])


# ---- predicates ---------------------------------------------------------------------
@pytest.mark.parametrize("c", G["pod_fits_resources"], ids=_ids("pod_fits_resources"))
def test_pod_fits_resources(c):
    fit = R.new_resource_fit_predicate(R.NodeInfo([mk_node(c["node"])]))
    assert fit(mk_pod(c["pod"]), [mk_pod(p) for p in c["existing"]], c["node"]["name"]) == c["fits"]


@pytest.mark.parametrize("c", G["pod_fits_host"], ids=_ids("pod_fits_host"))
def test_pod_fits_host(c):
    assert R.pod_fits_host(mk_pod(c["pod"]), [], c["node"]) == c["fits"]


@pytest.mark.parametrize("c", G["pod_fits_ports"], ids=[f"{i}-{t}" for i, t in enumerate(_ids("pod_fits_ports"))])
def test_pod_fits_ports(c):
    assert R.pod_fits_ports(mk_pod(c["pod"]), [mk_pod(p) for p in c["existing"]], "machine") == c["fits"]


@pytest.mark.parametrize("c", G["get_used_ports"])
def test_get_used_ports(c):
    assert sorted(R.get_used_ports(*[mk_pod(p) for p in c["pods"]])) == c["ports"]


@pytest.mark.parametrize("c", G["disk_conflicts"], ids=_ids("disk_conflicts"))
def test_disk_conflicts(c):
    assert R.no_disk_conflict(mk_pod(c["pod"]), [mk_pod(p) for p in c["existing"]], "machine") == c["fits"]


@pytest.mark.parametrize("c", G["pod_fits_selector"], ids=_ids("pod_fits_selector"))
def test_pod_fits_selector(c):
    info = R.NodeInfo([Node(metadata=ObjectMeta(name="machine", labels=c["labels"]))])
    assert R.new_selector_match_predicate(info)(mk_pod(c["pod"]), [], "machine") == c["fits"]


@pytest.mark.parametrize("c", G["node_label_presence"], ids=_ids("node_label_presence"))
def test_node_label_presence(c):
    info = R.NodeInfo([Node(metadata=ObjectMeta(name="machine", labels=c["node_labels"]))])
    assert R.new_node_label_predicate(info, c["labels"], c["presence"])(Pod(), [], "machine") == c["fits"]


@pytest.mark.parametrize("c", G["service_affinity"], ids=_ids("service_affinity"))
def test_service_affinity(c):
    fn = R.new_service_affinity_predicate(R.PodLister([mk_pod(p) for p in c["pods"]]),
                                          R.ServiceLister([mk_service(s, i) for i, s in enumerate(c["services"])]),
                                          R.NodeInfo([mk_node(n) for n in c["nodes"]]), c["labels"])
    assert fn(mk_pod(c["pod"]), [], c["node"]) == c["fits"]


# ---- generic scheduler ------------------------------------------------------------
def _false(pod, existing, node):
    return False


def _true(pod, existing, node):
    return True


def _matches(pod, existing, node):
    return pod.metadata.name == node


def _numeric(pod, lister, nodes):
    return [(n.metadata.name, int(n.metadata.name)) for n in nodes]


def _reverse_numeric(pod, lister, nodes):
    res = _numeric(pod, lister, nodes)
    mx = max(float(s) for _, s in res) if res else 0.0
    mn = min(float(s) for _, s in res) if res else float("inf")
    return [(h, int(mx + mn - float(s))) for h, s in res]


PREDS = {"false": _false, "true": _true, "matches": _matches, "match": _matches}
PRIOS = {"EqualPriority": R.equal_priority, "numericPriority": _numeric, "reverseNumericPriority": _reverse_numeric}


class _OddFirst:
    """The one known bit of Go's rand.NewSource(0): its first Int() is odd
    (generic_scheduler_test.go:180-186 picks machine1 of the ties [machine2, machine1])."""

    def int(self):
        return 1


@pytest.mark.parametrize("c", G["select_host"])
def test_select_host(c):
    s = R.GenericScheduler({}, [], R.PodLister([]), SplitMix64Rand(0))
    lst = [tuple(x) for x in c["list"]]
    for _ in range(10):
        if c["expects_err"]:
            with pytest.raises(ValueError):
                s.select_host(lst)
        else:
            assert s.select_host(lst) in c["possible_hosts"]


@pytest.mark.parametrize("c", G["generic_scheduler"], ids=_ids("generic_scheduler"))
def test_generic_scheduler(c):
    nodes = [Node(metadata=ObjectMeta(name=n)) for n in c["nodes"]]
    pod = Pod(metadata=ObjectMeta(name=c["pod_name"]))
    preds = {p: PREDS[p] for p in c["predicates"]}
    prios = [(PRIOS[n], w) for n, w in c["prioritizers"]]
    for seed in range(4):
        s = R.GenericScheduler(preds, prios, R.PodLister([]), SplitMix64Rand(seed))
        if c["expects_err"]:
            with pytest.raises(R.FitError):
                s.schedule(pod, nodes)
        else:
            assert s.schedule(pod, nodes) in c["expected_hosts"]
    if "go_rand_seed0_host" in c:
        s = R.GenericScheduler(preds, prios, R.PodLister([]), _OddFirst())
        assert s.schedule(pod, nodes) == c["go_rand_seed0_host"]


@pytest.mark.parametrize("c", G["find_fit"], ids=_ids("find_fit"))
def test_find_fit(c):
    nodes = [Node(metadata=ObjectMeta(name=n)) for n in c["nodes"]]
    preds = {p: PREDS[p] for p in c["predicates"]}
    _, failed = R.find_nodes_that_fit(Pod(metadata=ObjectMeta(name=c["pod_name"])), R.PodLister([]), preds, nodes)
    assert {k: sorted(v) for k, v in failed.items()} == c["failed"]


def test_no_minions():
    s = R.GenericScheduler({"true": _true}, [], R.PodLister([]), SplitMix64Rand(0))
    with pytest.raises(R.NoMinions):
        s.schedule(Pod(), [])


# ---- quantity / labels (host ingest) ---------------------------------------------------
def _frac(s):
    n, d = s.split("/")
    return Fraction(int(n), int(d))


@pytest.mark.parametrize("c", Q["parse"], ids=[c["input"] for c in Q["parse"]])
def test_quantity_parse(c):
    want = _frac(c["amount"])
    q = parse_quantity(c["input"])
    assert (q.amount, q.format) == (want, c["format"])
    qn = parse_quantity("-" + c["input"])  # TestQuantityParse also runs every row negated and with "+"
    assert (qn.amount, qn.format) == (-want, c["format"])
    qp = parse_quantity("+" + c["input"])
    assert (qp.amount, qp.format) == (want, c["format"])


@pytest.mark.parametrize("s", Q["invalid"])
def test_quantity_invalid(s):
    with pytest.raises(QuantityError):
        parse_quantity(s)


@pytest.mark.parametrize("c", Q["milli_value"], ids=[c["input"] for c in Q["milli_value"]])
def test_quantity_milli_value(c):
    assert parse_quantity(c["input"]).milli_value() == c["milli"]


@pytest.mark.parametrize("c", Q["value"], ids=[c["input"] for c in Q["value"]])
def test_quantity_value(c):
    assert parse_quantity(c["input"]).value() == c["value"]


def test_set_matches():
    for c in LB["set_matches"]:
        assert L.selector_from_set(c["selector"]).matches(c["labels"]) == c["matches"], c


def test_label_validation():
    assert all(L.is_qualified_name(v) for v in LB["qualified_name_good"])
    assert not any(L.is_qualified_name(v) for v in LB["qualified_name_bad"])
    assert all(L.is_valid_label_value(v) for v in LB["label_value_good"])
    assert not any(L.is_valid_label_value(v) for v in LB["label_value_bad"])


def test_selector_from_set_invalid_matches_everything():
    """selector.go:654-668: an invalid key or value -> empty selector (matches all)."""
    assert L.selector_from_set({"foo": "=blah"}).matches({"foo": "bar"})
    assert L.selector_from_set({"bad key!": "x"}).empty()
