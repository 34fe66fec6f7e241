"""Loads tests/golden/*.json into kubernetes_amd.api objects and runs a case through an
engine (the C oracle or the HIP library) via the product's own ingest.

The fixtures are the reference's Go test tables restated as data by
tests/golden/make_golden.py.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

from kubernetes_amd import abi, factory, ingest
from kubernetes_amd.api import (Container, ContainerPort, GCEPersistentDiskVolumeSource, Node, NodeSpec, ObjectMeta,
                                Pod, PodSpec, PodStatus, ResourceList, ResourceRequirements, Service, ServiceSpec,
                                Volume, make_node)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name: str) -> dict:
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def mk_node(d: dict, labels=None) -> Node:
    lab = d.get("labels") if labels is None else labels
    if "cpu_milli" in d:
        return make_node(d["name"], d["cpu_milli"], d["memory"], labels=lab)
    return Node(metadata=ObjectMeta(name=d["name"], labels=lab))


def mk_pod(d: dict) -> Pod:
    ctrs = []
    for c in d.get("containers", []):
        lim = {}
        if "cpu" in c:
            lim["cpu"] = c["cpu"]
        if "memory" in c:
            lim["memory"] = c["memory"]
        ctrs.append(Container(ports=[ContainerPort(host_port=p) for p in c.get("ports", [])],
                              resources=ResourceRequirements(ResourceList(lim))))
    vols = [Volume(gce_persistent_disk=GCEPersistentDiskVolumeSource(pd_name=n)) for n in d.get("pds", [])]
    return Pod(metadata=ObjectMeta(name=d.get("name", ""), namespace=d.get("ns", ""), labels=d.get("labels")),
               spec=PodSpec(containers=ctrs, volumes=vols, node_selector=d.get("node_selector"),
                            host=d.get("host", "")),
               status=PodStatus(host=d.get("status_host", "")))


def mk_service(d: dict, i: int = 0) -> Service:
    return Service(metadata=ObjectMeta(name=f"svc{i}", namespace=d.get("ns", "")),
                   spec=ServiceSpec(selector=d.get("selector")))


def run_engine(engine_cls, config: factory.SchedulerConfig, nodes: Sequence[Node], existing: Sequence[Pod],
               services: Sequence[Service], pod: Pod) -> Tuple[int, Dict[str, Tuple[int, int]]]:
    """Ingest a case and evaluate `pod` once.

    Returns (rc, {node name: (fail code, combined score)}). Existing pods are added in lister
    order on their Status.Host; a host outside the node list gets an external id."""
    it = ingest.Interner()
    for k in config.label_keys():
        it.key_id(k)
    view = ingest.ClusterView(nodes, services, it)
    aff = config.affinity_labels()
    cfg = config.compile(it.key_id)
    eng = engine_cls(cfg)
    try:
        eng.set_cluster(view.arrays)
        if existing:
            b = ingest.ingest_pods(view, existing, aff_labels=aff)
            for i, p in enumerate(existing):
                eng.add_pod(view.host_id(p.status.host), b, i)
        pb = ingest.ingest_pods(view, [pod], uids=[10 ** 6], aff_labels=aff)
        rc, fails, scores = eng.evaluate(pb, 0)
        return rc, {view.names[i]: (int(fails[i]), int(scores[i])) for i in range(len(view.names))}
    finally:
        eng.close()


# ---- configs for single-function golden cases ---------------------------------------
def cfg_priority(kind: str, label: str = "", presence: bool = False) -> factory.SchedulerConfig:
    """No predicates and one priority of weight 1: the combined score is that priority's score."""
    if kind in ("LeastRequestedPriority", "ServiceSpreadingPriority"):
        return factory.create_from_keys([], [kind])
    if kind == "ServiceAntiAffinity":
        name = f"golden-anti-{label}"
        pol = {"priorities": [{"name": name, "weight": 1, "argument": {"serviceAntiAffinity": {"label": label}}}]}
    else:
        name = f"golden-pref-{label}-{int(presence)}"
        pol = {"priorities": [{"name": name, "weight": 1,
                               "argument": {"labelPreference": {"label": label, "presence": presence}}}]}
    return factory.create_from_config(pol)


def cfg_predicate(kind: str, labels: Sequence[str] = (), presence: bool = False) -> factory.SchedulerConfig:
    """One predicate and LeastRequested (any priority works: only the fit code is read)."""
    if kind in ("PodFitsPorts", "PodFitsResources", "NoDiskConflict", "MatchNodeSelector", "HostName"):
        return factory.create_from_keys([kind], ["LeastRequestedPriority"])
    if kind == "ServiceAffinity":
        name = "golden-aff-" + "-".join(labels)
        arg = {"serviceAffinity": {"labels": list(labels)}}
    else:
        name = "golden-presence-" + "-".join(labels) + f"-{int(presence)}"
        arg = {"labelsPresence": {"labels": list(labels), "presence": presence}}
    return factory.create_from_config({"predicates": [{"name": name, "argument": arg}],
                                       "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]})


# ---- case adapters: each golden section -> (config, nodes, existing, services, pod, check) ----
def priority_cases(g: dict):
    """Yield (id, config, nodes, existing, services, pod, expected {host: score}, ordered)."""
    for c in g["least_requested"]:
        yield ("least_requested/" + c["test"], cfg_priority("LeastRequestedPriority"),
               [mk_node(n) for n in c["nodes"]], [mk_pod(p) for p in c["pods"]], [], mk_pod(c["pod"]),
               dict(map(tuple, c["expected"])))
    for c in g["service_spread"]:
        yield ("service_spread/" + c["test"], cfg_priority("ServiceSpreadingPriority"),
               [mk_node(n) for n in c["nodes"]], [mk_pod(p) for p in c["pods"]],
               [mk_service(s, i) for i, s in enumerate(c["services"])], mk_pod(c["pod"]),
               dict(map(tuple, c["expected"])))
    for c in g["zone_spread"]:
        yield ("zone_spread/" + c["test"], cfg_priority("ServiceAntiAffinity", "zone"),
               [mk_node(n) for n in c["nodes"]], [mk_pod(p) for p in c["pods"]],
               [mk_service(s, i) for i, s in enumerate(c["services"])], mk_pod(c["pod"]),
               dict(map(tuple, c["expected"])))
    for c in g["node_label_priority"]:
        yield ("node_label_priority/" + c["test"], cfg_priority("LabelPreference", c["label"], c["presence"]),
               [mk_node(n) for n in c["nodes"]], [], [], Pod(), dict(map(tuple, c["expected"])))


def predicate_cases(g: dict):
    """Yield (id, config, nodes, existing, services, pod, node name, fits)."""
    for c in g["pod_fits_resources"]:
        nd = c["node"]
        ex = [mk_pod(p) for p in c["existing"]]
        for p in ex:
            p.status.host = nd["name"]
        yield ("pod_fits_resources/" + c["test"], cfg_predicate("PodFitsResources"), [mk_node(nd)], ex, [],
               mk_pod(c["pod"]), nd["name"], c["fits"])
    for c in g["pod_fits_host"]:
        yield ("pod_fits_host/" + c["test"], cfg_predicate("HostName"), [Node(metadata=ObjectMeta(name=c["node"]))],
               [], [], mk_pod(c["pod"]), c["node"], c["fits"])
    for kind, sec in (("PodFitsPorts", "pod_fits_ports"), ("NoDiskConflict", "disk_conflicts")):
        for c in g[sec]:
            ex = [mk_pod(p) for p in c["existing"]]
            for p in ex:  # the Go tests pass these as the node's existing pods
                p.status.host = "machine"
            yield (f"{sec}/" + c["test"], cfg_predicate(kind), [Node(metadata=ObjectMeta(name="machine"))], ex, [],
                   mk_pod(c["pod"]), "machine", c["fits"])
    for c in g["pod_fits_selector"]:
        yield ("pod_fits_selector/" + c["test"], cfg_predicate("MatchNodeSelector"),
               [Node(metadata=ObjectMeta(name="machine", labels=c["labels"]))], [], [], mk_pod(c["pod"]), "machine",
               c["fits"])
    for c in g["node_label_presence"]:
        yield ("node_label_presence/" + c["test"], cfg_predicate("LabelsPresence", c["labels"], c["presence"]),
               [Node(metadata=ObjectMeta(name="machine", labels=c["node_labels"]))], [], [], Pod(), "machine",
               c["fits"])
    for c in g["service_affinity"]:
        yield ("service_affinity/" + c["test"], cfg_predicate("ServiceAffinity", c["labels"]),
               [mk_node(n) for n in c["nodes"]], [mk_pod(p) for p in c["pods"]],
               [mk_service(s, i) for i, s in enumerate(c["services"])], mk_pod(c["pod"]), c["node"], c["fits"])
