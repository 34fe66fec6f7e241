#!/usr/bin/env python3
"""Writes tests/golden/*.json: the reference's own test tables for the hot path, as data.

The reference is Go and there is no Go toolchain here, so the
Go tests cannot be run. Their tables of inputs and expected outputs are the
known answers that pin the oracle. This script restates each table as plain
data. Each section names the Go test (file:line under pkg/) that holds it. Run
it to regenerate the fixtures:

    python tests/golden/make_golden.py

Encoding (our own, used by tests/golden_cases.py):
  node    {"name", "cpu_milli", "memory", "labels"}    cpu_milli/memory absent = no capacity
  pod     {"name", "ns", "labels", "host", "status_host", "node_selector",
           "containers": [{"cpu", "memory", "ports"}], "pds": [pd names]}
          container quantities are strings for ParseQuantity. NewMilliQuantity(v)
          is written "<v>m" and NewQuantity(v) is written "<v>". The amounts are equal.
  service {"ns", "selector"}
  host priority lists are [[host, score], ...]
"""
from __future__ import annotations

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


# ---- constructors --------------------------------------------------------------
def node(name, cpu_milli=None, memory=None, labels=None):
    d = {"name": name}
    if cpu_milli is not None:
        d["cpu_milli"] = cpu_milli
        d["memory"] = memory
    if labels is not None:
        d["labels"] = labels
    return d


def pod(name="", ns="", labels=None, host="", status_host="", node_selector=None, containers=(), pds=()):
    return {"name": name, "ns": ns, "labels": labels, "host": host, "status_host": status_host,
            "node_selector": node_selector, "containers": list(containers), "pds": list(pds)}


def ctr(cpu=None, memory=None, ports=()):
    c = {"ports": list(ports)}
    if cpu is not None:
        c["cpu"] = cpu
    if memory is not None:
        c["memory"] = memory
    return c


def svc(selector, ns=""):
    return {"ns": ns, "selector": selector}


def resource_pod(*reqs):
    """newResourcePod (predicates_test.go:55-72): NewMilliQuantity cpu, NewQuantity memory."""
    return pod(containers=[ctr(f"{c}m", f"{m}") for c, m in reqs])


def port_pod(host, *ports):
    """newPod (scheduler_test.go:62-78): Status.Host + one container with these HostPorts."""
    return pod(status_host=host, containers=[ctr(ports=ports)])


# ---- priorities_test.go ---------------------------------------------------------
def least_requested():
    """TestLeastRequested (priorities_test.go:40-264). Expected lists are in node order."""
    l1 = {"foo": "bar", "baz": "blah"}
    l2 = {"bar": "foo", "baz": "blah"}
    cpu_only = [ctr("1000m"), ctr("2000m")]
    cpu_mem = [ctr("1000m", "2000"), ctr("2000m", "3000")]
    m = lambda a, b, c, d: [node("machine1", a, b), node("machine2", c, d)]
    P = lambda host, spec, labels=None: pod(status_host=host, containers=spec, labels=labels)
    return [
        {"test": "nothing scheduled, nothing requested", "pod": pod(), "pods": [],
         "nodes": m(4000, 10000, 4000, 10000), "expected": [["machine1", 10], ["machine2", 10]]},
        {"test": "nothing scheduled, resources requested, differently sized machines", "pod": pod(containers=cpu_mem),
         "pods": [], "nodes": m(4000, 10000, 6000, 10000), "expected": [["machine1", 3], ["machine2", 5]]},
        {"test": "no resources requested, pods scheduled", "pod": pod(),
         "pods": [P("machine1", [], l2), P("machine1", [], l1), P("machine2", [], l1), P("machine2", [], l1)],
         "nodes": m(4000, 10000, 4000, 10000), "expected": [["machine1", 10], ["machine2", 10]]},
        {"test": "no resources requested, pods scheduled with resources", "pod": pod(),
         "pods": [P("machine1", cpu_only, l2), P("machine1", cpu_only, l1), P("machine2", cpu_only, l1),
                  P("machine2", cpu_mem, l1)],
         "nodes": m(10000, 20000, 10000, 20000), "expected": [["machine1", 7], ["machine2", 5]]},
        {"test": "resources requested, pods scheduled with resources", "pod": pod(containers=cpu_mem),
         "pods": [P("machine1", cpu_only), P("machine2", cpu_mem)],
         "nodes": m(10000, 20000, 10000, 20000), "expected": [["machine1", 5], ["machine2", 4]]},
        {"test": "resources requested, pods scheduled with resources, differently sized machines",
         "pod": pod(containers=cpu_mem), "pods": [P("machine1", cpu_only), P("machine2", cpu_mem)],
         "nodes": m(10000, 20000, 10000, 50000), "expected": [["machine1", 5], ["machine2", 6]]},
        {"test": "requested resources exceed minion capacity", "pod": pod(containers=cpu_only),
         "pods": [P("machine1", cpu_only), P("machine2", cpu_mem)],
         "nodes": m(4000, 10000, 4000, 10000), "expected": [["machine1", 5], ["machine2", 2]]},
        {"test": "zero minion resources, pods scheduled with resources", "pod": pod(),
         "pods": [P("", cpu_only), P("", cpu_mem)],
         "nodes": m(0, 0, 0, 0), "expected": [["machine1", 0], ["machine2", 0]]},
    ]


def node_label_priority():
    """TestNewNodeLabelPriority (priorities_test.go:269-366). Compared after sorting."""
    nodes = [node("machine1", labels={"foo": "bar"}), node("machine2", labels={"bar": "foo"}),
             node("machine3", labels={"bar": "baz"})]
    rows = [
        ("baz", True, [0, 0, 0], "no match found, presence true"),
        ("baz", False, [10, 10, 10], "no match found, presence false"),
        ("foo", True, [10, 0, 0], "one match found, presence true"),
        ("foo", False, [0, 10, 10], "one match found, presence false"),
        ("bar", True, [0, 10, 10], "two matches found, presence true"),
        ("bar", False, [10, 0, 0], "two matches found, presence false"),
    ]
    return [{"test": t, "nodes": nodes, "label": l, "presence": p,
             "expected": [[f"machine{i + 1}", s] for i, s in enumerate(sc)]} for l, p, sc, t in rows]


# ---- spreading_test.go ----------------------------------------------------------
def service_spread():
    """TestServiceSpreadPriority (spreading_test.go:27-171). Expected lists are in node order."""
    l1 = {"foo": "bar", "baz": "blah"}
    l2 = {"bar": "foo", "baz": "blah"}
    z1, z2 = "machine1", "machine2"
    P = lambda host, labels=None, ns="": pod(status_host=host, labels=labels, ns=ns)
    nodes = [node("machine1"), node("machine2")]
    return [
        {"test": "nothing scheduled", "pod": pod(), "pods": [], "services": [], "nodes": nodes,
         "expected": [[z1, 10], [z2, 10]]},
        {"test": "no services", "pod": pod(labels=l1), "pods": [P(z1)], "services": [], "nodes": nodes,
         "expected": [[z1, 10], [z2, 10]]},
        {"test": "different services", "pod": pod(labels=l1), "pods": [P(z1, l2)],
         "services": [svc({"key": "value"})], "nodes": nodes, "expected": [[z1, 10], [z2, 10]]},
        {"test": "two pods, one service pod", "pod": pod(labels=l1), "pods": [P(z1, l2), P(z2, l1)],
         "services": [svc(l1)], "nodes": nodes, "expected": [[z1, 10], [z2, 0]]},
        {"test": "five pods, one service pod in no namespace", "pod": pod(labels=l1),
         "pods": [P(z1, l2), P(z1, l1, "default"), P(z1, l1, "ns1"), P(z2, l1), P(z2, l2)],
         "services": [svc(l1)], "nodes": nodes, "expected": [[z1, 10], [z2, 0]]},
        {"test": "four pods, one service pod in default namespace", "pod": pod(labels=l1, ns="default"),
         "pods": [P(z1, l1), P(z1, l1, "ns1"), P(z2, l1, "default"), P(z2, l2)],
         "services": [svc(l1, "default")], "nodes": nodes, "expected": [[z1, 10], [z2, 0]]},
        {"test": "five pods, one service pod in specific namespace", "pod": pod(labels=l1, ns="ns1"),
         "pods": [P(z1, l1), P(z1, l1, "default"), P(z1, l1, "ns2"), P(z2, l1, "ns1"), P(z2, l2)],
         "services": [svc(l1, "ns1")], "nodes": nodes, "expected": [[z1, 10], [z2, 0]]},
        {"test": "three pods, two service pods on different machines", "pod": pod(labels=l1),
         "pods": [P(z1, l2), P(z1, l1), P(z2, l1)], "services": [svc(l1)], "nodes": nodes,
         "expected": [[z1, 0], [z2, 0]]},
        {"test": "four pods, three service pods", "pod": pod(labels=l1),
         "pods": [P(z1, l2), P(z1, l1), P(z2, l1), P(z2, l1)], "services": [svc(l1)], "nodes": nodes,
         "expected": [[z1, 5], [z2, 0]]},
        {"test": "service with partial pod label matches", "pod": pod(labels=l1),
         "pods": [P(z1, l2), P(z1, l1), P(z2, l1)], "services": [svc({"baz": "blah"})], "nodes": nodes,
         "expected": [[z1, 0], [z2, 5]]},
    ]


def zone_spread():
    """TestZoneSpreadPriority (spreading_test.go:173-341): ServiceAntiAffinity{label: zone}.
    The node list comes from a Go map (makeLabeledMinionList), so results are compared sorted."""
    l1 = {"foo": "bar", "baz": "blah"}
    l2 = {"bar": "foo", "baz": "blah"}
    nozone, zone1, zone2 = {"name": "value"}, {"zone": "zone1"}, {"zone": "zone2"}
    nodes = [node("machine01", labels=nozone), node("machine02", labels=nozone),
             node("machine11", labels=zone1), node("machine12", labels=zone1),
             node("machine21", labels=zone2), node("machine22", labels=zone2)]
    h0, h1, h2 = "machine01", "machine11", "machine21"
    P = lambda host, labels=None, ns="": pod(status_host=host, labels=labels, ns=ns)

    def exp(a, b):
        return [["machine11", a], ["machine12", a], ["machine21", b], ["machine22", b],
                ["machine01", 0], ["machine02", 0]]
    return [
        {"test": "nothing scheduled", "pod": pod(), "pods": [], "services": [], "expected": exp(10, 10)},
        {"test": "no services", "pod": pod(labels=l1), "pods": [P(h1)], "services": [], "expected": exp(10, 10)},
        {"test": "different services", "pod": pod(labels=l1), "pods": [P(h1, l2)],
         "services": [svc({"key": "value"})], "expected": exp(10, 10)},
        {"test": "three pods, one service pod", "pod": pod(labels=l1), "pods": [P(h0, l2), P(h1, l2), P(h2, l1)],
         "services": [svc(l1)], "expected": exp(10, 0)},
        {"test": "three pods, two service pods on different machines", "pod": pod(labels=l1),
         "pods": [P(h1, l2), P(h1, l1), P(h2, l1)], "services": [svc(l1)], "expected": exp(5, 5)},
        {"test": "three service label match pods in different namespaces", "pod": pod(labels=l1, ns="default"),
         "pods": [P(h1, l1), P(h1, l1, "default"), P(h2, l1), P(h2, l1, "ns1")],
         "services": [svc(l1, "default")], "expected": exp(0, 10)},
        {"test": "four pods, three service pods", "pod": pod(labels=l1),
         "pods": [P(h1, l2), P(h1, l1), P(h2, l1), P(h2, l1)], "services": [svc(l1)], "expected": exp(6, 3)},
        {"test": "service with partial pod label matches", "pod": pod(labels=l1),
         "pods": [P(h1, l2), P(h1, l1), P(h2, l1)], "services": [svc({"baz": "blah"})], "expected": exp(3, 6)},
        {"test": "service pod on non-zoned minion", "pod": pod(labels=l1),
         "pods": [P(h0, l1), P(h1, l1), P(h2, l1), P(h2, l1)], "services": [svc(l1)], "expected": exp(7, 5)},
    ]


def with_nodes(cases, nodes):
    for c in cases:
        c["nodes"] = nodes
    return cases


# ---- predicates_test.go ---------------------------------------------------------
def pod_fits_resources():
    """TestPodFitsResources (predicates_test.go:74-134): node capacity makeResources(10, 20)."""
    rows = [
        (pod(), [(10, 20)], True, "no resources requested always fits"),
        (resource_pod((1, 1)), [(10, 20)], False, "too many resources fails"),
        (resource_pod((1, 1)), [(5, 5)], True, "both resources fit"),
        (resource_pod((1, 2)), [(5, 19)], False, "one resources fits"),
        (resource_pod((5, 1)), [(5, 19)], True, "equal edge case"),
    ]
    return [{"test": t, "pod": p, "existing": [resource_pod(e) for e in ex], "node": node("machine", 10, 20),
             "fits": f} for p, ex, f, t in rows]


def pod_fits_host():
    """TestPodFitsHost (predicates_test.go:136-180)."""
    return [
        {"test": "no host specified", "pod": pod(), "node": "foo", "fits": True},
        {"test": "host matches", "pod": pod(host="foo"), "node": "foo", "fits": True},
        {"test": "host doesn't match", "pod": pod(host="bar"), "node": "foo", "fits": False},
    ]


def pod_fits_ports():
    """TestPodFitsPorts (predicates_test.go:182-237)."""
    return [
        {"test": "nothing running", "pod": pod(), "existing": [], "fits": True},
        {"test": "other port", "pod": port_pod("m1", 8080), "existing": [port_pod("m1", 9090)], "fits": True},
        {"test": "same port", "pod": port_pod("m1", 8080), "existing": [port_pod("m1", 8080)], "fits": False},
        {"test": "second port", "pod": port_pod("m1", 8000, 8080), "existing": [port_pod("m1", 8080)],
         "fits": False},
        {"test": "second port", "pod": port_pod("m1", 8000, 8080), "existing": [port_pod("m1", 8001, 8080)],
         "fits": False},
    ]


def get_used_ports():
    """TestGetUsedPorts (predicates_test.go:239-273)."""
    return [
        {"pods": [port_pod("m1", 9090)], "ports": [9090]},
        {"pods": [port_pod("m1", 9090), port_pod("m1", 9091)], "ports": [9090, 9091]},
        {"pods": [port_pod("m1", 9090), port_pod("m2", 9091)], "ports": [9090, 9091]},
    ]


def disk_conflicts():
    """TestDiskConflicts (predicates_test.go:275-322)."""
    foo = pod(pds=["foo"])
    bar = pod(pds=["bar"])
    return [
        {"test": "nothing", "pod": pod(), "existing": [], "fits": True},
        {"test": "one state", "pod": pod(), "existing": [foo], "fits": True},
        {"test": "same state", "pod": foo, "existing": [foo], "fits": False},
        {"test": "different state", "pod": bar, "existing": [foo], "fits": True},
    ]


def pod_fits_selector():
    """TestPodFitsSelector (predicates_test.go:324-404)."""
    return [
        {"test": "no selector", "pod": pod(), "labels": None, "fits": True},
        {"test": "missing labels", "pod": pod(node_selector={"foo": "bar"}), "labels": None, "fits": False},
        {"test": "same labels", "pod": pod(node_selector={"foo": "bar"}), "labels": {"foo": "bar"}, "fits": True},
        {"test": "node labels are superset", "pod": pod(node_selector={"foo": "bar"}),
         "labels": {"foo": "bar", "baz": "blah"}, "fits": True},
        {"test": "node labels are subset", "pod": pod(node_selector={"foo": "bar", "baz": "blah"}),
         "labels": {"foo": "bar"}, "fits": False},
    ]


def node_label_presence():
    """TestNodeLabelPresence (predicates_test.go:406-464): node labels {foo: bar, bar: foo}."""
    rows = [
        (["baz"], True, False, "label does not match, presence true"),
        (["baz"], False, True, "label does not match, presence false"),
        (["foo", "baz"], True, False, "one label matches, presence true"),
        (["foo", "baz"], False, False, "one label matches, presence false"),
        (["foo", "bar"], True, True, "all labels match, presence true"),
        (["foo", "bar"], False, False, "all labels match, presence false"),
    ]
    return [{"test": t, "labels": l, "presence": p, "node_labels": {"foo": "bar", "bar": "foo"}, "fits": f}
            for l, p, f, t in rows]


def service_affinity():
    """TestServiceAffinity (predicates_test.go:466-603): five labelled nodes."""
    sel = {"foo": "bar"}
    l1 = {"region": "r1", "zone": "z11"}
    l2 = {"region": "r1", "zone": "z12"}
    l3 = {"region": "r2", "zone": "z21"}
    l4 = {"region": "r2", "zone": "z22"}
    nodes = [node("machine1", labels=l1), node("machine2", labels=l2), node("machine3", labels=l3),
             node("machine4", labels=l4), node("machine5", labels=l4)]
    P = lambda host, ns="": pod(status_host=host, labels=sel, ns=ns)
    rows = [
        (pod(), [], [], "machine1", ["region"], True, "nothing scheduled"),
        (pod(node_selector={"region": "r1"}), [], [], "machine1", ["region"], True, "pod with region label match"),
        (pod(node_selector={"region": "r2"}), [], [], "machine1", ["region"], False,
         "pod with region label mismatch"),
        (pod(labels=sel), [P("machine1")], [svc(sel)], "machine1", ["region"], True, "service pod on same minion"),
        (pod(labels=sel), [P("machine2")], [svc(sel)], "machine1", ["region"], True,
         "service pod on different minion, region match"),
        (pod(labels=sel), [P("machine3")], [svc(sel)], "machine1", ["region"], False,
         "service pod on different minion, region mismatch"),
        (pod(labels=sel, ns="ns1"), [P("machine3", "ns1")], [svc(sel, "ns2")], "machine1", ["region"], True,
         "service in different namespace, region mismatch"),
        (pod(labels=sel, ns="ns1"), [P("machine3", "ns2")], [svc(sel, "ns1")], "machine1", ["region"], True,
         "pod in different namespace, region mismatch"),
        (pod(labels=sel, ns="ns1"), [P("machine3", "ns1")], [svc(sel, "ns1")], "machine1", ["region"], False,
         "service and pod in same namespace, region mismatch"),
        (pod(labels=sel), [P("machine2")], [svc(sel)], "machine1", ["region", "zone"], False,
         "service pod on different minion, multiple labels, not all match"),
        (pod(labels=sel), [P("machine5")], [svc(sel)], "machine4", ["region", "zone"], True,
         "service pod on different minion, multiple labels, all match"),
    ]
    return [{"test": t, "pod": p, "pods": ps, "services": ss, "node": n, "labels": l, "fits": f, "nodes": nodes}
            for p, ps, ss, n, l, f, t in rows]


# ---- generic_scheduler_test.go --------------------------------------------------
def select_host():
    """TestSelectHost (generic_scheduler_test.go:96-160): any member of possible_hosts."""
    return [
        {"list": [["machine1.1", 1], ["machine2.1", 2]], "possible_hosts": ["machine2.1"], "expects_err": False},
        {"list": [["machine1.1", 1], ["machine1.2", 2], ["machine1.3", 2], ["machine2.1", 2]],
         "possible_hosts": ["machine1.2", "machine1.3", "machine2.1"], "expects_err": False},
        {"list": [["machine1.1", 3], ["machine1.2", 3], ["machine2.1", 2], ["machine3.1", 1], ["machine1.3", 3]],
         "possible_hosts": ["machine1.1", "machine1.2", "machine1.3"], "expects_err": False},
        {"list": [], "possible_hosts": [], "expects_err": True},
    ]


def generic_scheduler():
    """TestGenericScheduler (generic_scheduler_test.go:162-245). Predicates / priorities are the
    test's own functions: false, true, matches (pod.Name == node), numeric (score = int(name)),
    reverseNumeric (max + min - score). go_rand_seed0_host is the host Go's rand.NewSource(0)
    picks. Only the 1-bit fact "first Int() is odd" is known (tie order machine2, machine1).
    Our tests use an injected source, and expected_hosts lists every host a source may yield."""
    return [
        {"name": "test 1", "predicates": ["false"], "prioritizers": [["EqualPriority", 1]],
         "nodes": ["machine1", "machine2"], "pod_name": "", "expects_err": True},
        {"name": "test 2", "predicates": ["true"], "prioritizers": [["EqualPriority", 1]],
         "nodes": ["machine1", "machine2"], "pod_name": "", "expects_err": False,
         "go_rand_seed0_host": "machine1", "expected_hosts": ["machine1", "machine2"]},
        {"name": "test 3", "predicates": ["matches"], "prioritizers": [["EqualPriority", 1]],
         "nodes": ["machine1", "machine2"], "pod_name": "machine2", "expects_err": False,
         "expected_hosts": ["machine2"]},
        {"name": "test 4", "predicates": ["true"], "prioritizers": [["numericPriority", 1]],
         "nodes": ["3", "2", "1"], "pod_name": "", "expects_err": False, "expected_hosts": ["3"]},
        {"name": "test 5", "predicates": ["matches"], "prioritizers": [["numericPriority", 1]],
         "nodes": ["3", "2", "1"], "pod_name": "2", "expects_err": False, "expected_hosts": ["2"]},
        {"name": "test 6", "predicates": ["true"],
         "prioritizers": [["numericPriority", 1], ["reverseNumericPriority", 2]],
         "nodes": ["3", "2", "1"], "pod_name": "2", "expects_err": False, "expected_hosts": ["1"]},
        {"name": "test 7", "predicates": ["true", "false"], "prioritizers": [["numericPriority", 1]],
         "nodes": ["3", "2", "1"], "pod_name": "", "expects_err": True},
    ]


def find_fit():
    """TestFindFitAllError / TestFindFitSomeError (generic_scheduler_test.go:247-297)."""
    return [
        {"name": "all error", "predicates": ["true", "false"], "nodes": ["3", "2", "1"], "pod_name": "",
         "failed": {"3": ["false"], "2": ["false"], "1": ["false"]}},
        {"name": "some error", "predicates": ["true", "match"], "nodes": ["3", "2", "1"], "pod_name": "1",
         "failed": {"3": ["match"], "2": ["match"]}},
    ]


# ---- pkg/api/resource/quantity_test.go ------------------------------------------
def _dec(i, exp):
    """dec(i, exponent) = i * 10^exponent as an exact fraction string."""
    from fractions import Fraction
    f = Fraction(i) * (Fraction(10) ** exp)
    return f"{f.numerator}/{f.denominator}"


def quantity():
    """TestQuantityParse (quantity_test.go:60-238); TestMilliNewSet / TestNewSet round trips
    (quantity_test.go:387-463) restated as parse -> MilliValue/Value of their strings."""
    MAX = "9223372036854775807/1"
    D, B, E = "DecimalSI", "BinarySI", "DecimalExponent"
    Ki = 1024
    parse = [
        ("0", _dec(0, 0), D), ("0m", _dec(0, 0), D), ("0Ki", _dec(0, 0), B), ("0k", _dec(0, 0), D),
        ("0Mi", _dec(0, 0), B), ("0M", _dec(0, 0), D), ("0Gi", _dec(0, 0), B), ("0G", _dec(0, 0), D),
        ("0Ti", _dec(0, 0), B), ("0T", _dec(0, 0), D),
        ("1Ki", _dec(Ki, 0), B), ("8Ki", _dec(8 * Ki, 0), B), ("7Mi", _dec(7 * Ki ** 2, 0), B),
        ("6Gi", _dec(6 * Ki ** 3, 0), B), ("5Ti", _dec(5 * Ki ** 4, 0), B), ("4Pi", _dec(4 * Ki ** 5, 0), B),
        ("3Ei", _dec(3 * Ki ** 6, 0), B), ("10Ti", _dec(10 * Ki ** 4, 0), B), ("100Ti", _dec(100 * Ki ** 4, 0), B),
        ("3m", _dec(3, -3), D), ("9", _dec(9, 0), D), ("8k", _dec(8, 3), D), ("7M", _dec(7, 6), D),
        ("6G", _dec(6, 9), D), ("5T", _dec(5, 12), D), ("40T", _dec(4, 13), D), ("300T", _dec(3, 14), D),
        ("2P", _dec(2, 15), D), ("1E", _dec(1, 18), D),
        ("1E-3", _dec(1, -3), E), ("1e3", _dec(1, 3), E), ("1E6", _dec(1, 6), E), ("1e9", _dec(1, 9), E),
        ("1E12", _dec(1, 12), E), ("1e15", _dec(1, 15), E), ("1E18", _dec(1, 18), E),
        ("1e14", _dec(1, 14), E), ("1e13", _dec(1, 13), E), ("100.035k", _dec(100035, 0), D),
        ("0.001", _dec(1, -3), D), ("0.0005k", _dec(5, -1), D), ("0.005", _dec(5, -3), D),
        ("0.05", _dec(5, -2), D), ("0.5", _dec(5, -1), D), ("0.00050k", _dec(5, -1), D),
        ("0.00500", _dec(5, -3), D), ("0.05000", _dec(5, -2), D), ("0.50000", _dec(5, -1), D),
        ("0.5e0", _dec(5, -1), E), ("0.5e-1", _dec(5, -2), E), ("0.5e-2", _dec(5, -3), E),
        ("10.035M", _dec(10035, 3), D),
        ("1.2e3", _dec(12, 2), E), ("1.3E+6", _dec(13, 5), E), ("1.40e9", _dec(14, 8), E),
        ("1.53E12", _dec(153, 10), E), ("1.6e15", _dec(16, 14), E), ("1.7E18", _dec(17, 17), E),
        ("9.01", _dec(901, -2), D), ("8.1k", _dec(81, 2), D), ("7.123456M", _dec(7123456, 0), D),
        ("6.987654321G", _dec(6987654321, 0), D), ("5.444T", _dec(5444, 9), D), ("40.1T", _dec(401, 11), D),
        ("300.2T", _dec(3002, 11), D), ("2.5P", _dec(25, 14), D), ("1.01E", _dec(101, 16), D),
        ("3.001m", _dec(4, -3), D), ("1.1E-3", _dec(2, -3), E), ("0.0001", _dec(1, -3), D),
        ("0.0005", _dec(1, -3), D), ("0.00050", _dec(1, -3), D), ("0.5e-3", _dec(1, -3), E),
        ("0.9m", _dec(1, -3), D), ("0.12345", _dec(124, -3), D), ("0.12354", _dec(124, -3), D),
        ("9Ei", MAX, B), ("9223372036854775807Ki", MAX, B), ("12E", MAX, D),
        ("100.035Ki", _dec(10243584, -2), B), ("0.5Mi", _dec(Ki * Ki // 2, 0), B),
        ("0.05Gi", _dec(536870912, -1), B), ("0.025Ti", _dec(274877906944, -1), B),
        ("0.000001Ki", _dec(2, -3), D), (".001", _dec(1, -3), D), (".0001k", _dec(100, -3), D),
        ("1.", _dec(1, 0), D), ("1.G", _dec(1, 9), D),
    ]
    invalid = ["1.1.M", "1+1.0M", "0.1mi", "0.1am", "aoeu", ".5i", "1i", "-3.01i"]
    milli = [("1m", 1), ("1", 1000), ("1234", 1234000), ("1e3", 1000000)]
    value = [("1", 1), ("1k", 1000), ("1234k", 1234000), ("1Ki", 1024), ("1e6", 1000000), ("1Mi", 1024 * 1024)]
    return {"parse": [{"input": i, "amount": a, "format": f} for i, a, f in parse],
            "invalid": invalid,
            "milli_value": [{"input": i, "milli": v} for i, v in milli],
            "value": [{"input": i, "value": v} for i, v in value]}


# ---- pkg/labels, pkg/util/validation -------------------------------------------
def labels():
    """TestSetMatches (labels/selector_test.go:130-144), the equality cases of TestSelectorMatches
    (:96-116), TestNilMapIsValid (:146-154), TestLabelHas/Get (labels_test.go:38-70),
    TestIsQualifiedName / TestIsValidLabelValue (util/validation_test.go:157-225)."""
    ls = {"foo": "bar", "baz": "blah"}
    matches = [
        ({}, ls, True), ({"foo": "bar"}, ls, True), ({"baz": "blah"}, ls, True),
        ({"foo": "bar", "baz": "blah"}, ls, True),
        ({"x": "y"}, {"x": "y"}, True), ({"x": "y", "z": "w"}, {"x": "y", "z": "w"}, True),
        ({"notin": "in"}, {"notin": "in"}, True),
        ({"x": "y"}, {"x": "z"}, False), ({"x": "y", "z": "w"}, {"x": "w", "z": "w"}, False),
        ({"foo": "blah"}, ls, False), ({"baz": "bar"}, ls, False),
        ({"foo": "bar", "foobar": "bar", "baz": "blah"}, ls, False),
        (None, ls, True),
    ]
    return {
        "set_matches": [{"selector": s, "labels": l, "matches": m} for s, l, m in matches],
        "qualified_name_good": ["simple", "now-with-dashes", "1-starts-with-num", "1234", "simple/simple",
                                "now-with-dashes/simple", "now-with-dashes/now-with-dashes", "now.with.dots/simple",
                                "now-with.dashes-and.dots/simple", "1-num.2-num/3-num", "1234/5678",
                                "1.2.3.4/5678", "UppercaseIsOK123"],
        "qualified_name_bad": ["nospecialchars%^=@", "cantendwithadash-", "only/one/slash", "a" * 254,
                               "-cantstartwithadash"],
        "label_value_good": ["simple", "now-with-dashes", "1-starts-with-num", "end-with-num-1", "1234", "a" * 63, ""],
        "label_value_bad": ["nospecialchars%^=@", "Tama-nui-te-rā.is.Māori.sun", "\\backslashes\\are\\bad",
                            "-starts-with-dash", "ends-with-dash-", ".starts.with.dot", "ends.with.dot.", "a" * 64],
    }


def modeler():
    """plugin/pkg/scheduler/modeler_test.go:52-75 (TestModeler): (namespace, name) ids."""
    return {"source": "plugin/pkg/scheduler/modeler_test.go:52-75", "cases": [
        {"queued": [], "scheduled": [["default", "foo"], ["custom", "foo"]], "assumed": [["default", "foo"]],
         "expect": [["default", "foo"], ["custom", "foo"]]},
        {"queued": [], "scheduled": [["default", "foo"]], "assumed": [["default", "foo"], ["custom", "foo"]],
         "expect": [["default", "foo"], ["custom", "foo"]]},
        {"queued": [["custom", "foo"]], "scheduled": [["default", "foo"]],
         "assumed": [["default", "foo"], ["custom", "foo"]], "expect": [["default", "foo"]]},
    ]}


def kubelet():
    """pkg/kubelet/kubelet_test.go TestHandleNodeSelector (:2929-2976) and TestHandleMemExceeded
    (:2979-3032): handleNotFittingPods (kubelet.go:1745-1771) marks the not-fitting pod failed.
    machine = cadvisor MachineInfo (CapacityFromMachineInfo, kubelet/util.go:48-58); created =
    CreationTimestamp order key (seconds); rejected = the pods whose status becomes PodFailed."""
    mem90 = [ctr(memory="90")]
    return {"source": "pkg/kubelet/kubelet_test.go:2929-3032", "cases": [
        {"test": "TestHandleNodeSelector", "machine": {"num_cores": 0, "memory_capacity": 0},
         "node_labels": {"key": "B"},
         "pods": [dict(pod("podA", "foo", node_selector={"key": "A"}), created=0),
                  dict(pod("podB", "foo", node_selector={"key": "B"}), created=0)],
         "rejected": {"foo/podA": "nodeSelectorMismatching"}},
        {"test": "TestHandleMemExceeded", "machine": {"num_cores": 0, "memory_capacity": 100},
         "node_labels": None,
         "pods": [dict(pod("newpod", "foo", containers=mem90), created=1),
                  dict(pod("oldpod", "foo", containers=mem90), created=0)],
         "rejected": {"foo/newpod": "capacityExceeded"}},
    ]}


def main():
    out = {
        "source": "smarterclayton/kubernetes v0.13.0-dev, pkg/scheduler/*_test.go (tables restated as data)",
        "least_requested": least_requested(),
        "node_label_priority": node_label_priority(),
        "service_spread": service_spread(),
        "zone_spread": zone_spread(),
        "pod_fits_resources": pod_fits_resources(),
        "pod_fits_host": pod_fits_host(),
        "pod_fits_ports": pod_fits_ports(),
        "get_used_ports": get_used_ports(),
        "disk_conflicts": disk_conflicts(),
        "pod_fits_selector": pod_fits_selector(),
        "node_label_presence": node_label_presence(),
        "service_affinity": service_affinity(),
        "select_host": select_host(),
        "generic_scheduler": generic_scheduler(),
        "find_fit": find_fit(),
    }
    zs = out["zone_spread"]
    with_nodes(zs, [node("machine01", labels={"name": "value"}), node("machine02", labels={"name": "value"}),
                    node("machine11", labels={"zone": "zone1"}), node("machine12", labels={"zone": "zone1"}),
                    node("machine21", labels={"zone": "zone2"}), node("machine22", labels={"zone": "zone2"})])
    with open(os.path.join(HERE, "scheduler_golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    with open(os.path.join(HERE, "modeler_golden.json"), "w") as f:
        json.dump(modeler(), f, indent=1, sort_keys=True)
        f.write("\n")
    with open(os.path.join(HERE, "kubelet_golden.json"), "w") as f:
        json.dump(kubelet(), f, indent=1, sort_keys=True)
        f.write("\n")
    with open(os.path.join(HERE, "quantity_golden.json"), "w") as f:
        json.dump({"source": "pkg/api/resource/quantity_test.go", **quantity()}, f, indent=1, sort_keys=True)
        f.write("\n")
    with open(os.path.join(HERE, "labels_golden.json"), "w") as f:
        json.dump({"source": "pkg/labels/*_test.go, pkg/util/validation_test.go", **labels()}, f, indent=1,
                  sort_keys=True, ensure_ascii=True)
        f.write("\n")


if __name__ == "__main__":
    main()
