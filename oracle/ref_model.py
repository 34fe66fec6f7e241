"""Object-level restatement of pkg/scheduler (smarterclayton/kubernetes v0.13.0-dev).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Pure Python over
kubernetes_amd.api objects; every function names the reference lines it
transcribes (paths under /root/reference). Used for small cases: it is pinned
by the golden vectors transcribed from the reference's Go tests
(tests/golden/scheduler_golden.json) and in turn pins the C restatement and the
host ingest (tests/test_oracle_crosscheck.py).

Go map iteration order is the only nondeterminism in the reference on this
path; it is canonicalised here as in the product:
  * predicates run in sorted-name order (findNodesThatFit, generic_scheduler.go:109),
    except that predicates which can return an error (ServiceAffinity's peer
    lookup, predicates.go:293-297) run first: when the first service peer sits
    on a host outside the node list, Schedule returns that error (one of the
    outcomes Go's random map order allows, and the one the kernels implement);
  * services[0] = first matching service in ServiceLister order (spreading.go:54);
  * nsServicePods[0] = first matching pod in PodLister order (predicates.go:293).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from kubernetes_amd.api import Node, Pod, Service
from kubernetes_amd.labels import everything, selector_from_set, set_get, set_has


class FitError(Exception):
    def __init__(self, pod, failed):
        super().__init__("failed to find fit")
        self.pod = pod
        self.failed_predicates = failed


class NoMinions(Exception):
    pass


# ---- listers (pkg/scheduler/listers.go:27-93) -------------------------------
class PodLister:
    def __init__(self, pods: Sequence[Pod]):
        self.pods = list(pods)

    def list(self, selector=None) -> List[Pod]:
        sel = selector or everything()
        return [p for p in self.pods if sel.matches(p.metadata.labels)]


class ServiceLister:
    def __init__(self, services: Sequence[Service]):
        self.services = list(services)

    def get_pod_services(self, pod: Pod) -> List[Service]:
        """FakeServiceLister.GetPodServices (listers.go:59-78)."""
        out = [s for s in self.services
               if s.metadata.namespace == pod.metadata.namespace
               and selector_from_set(s.spec.selector).matches(pod.metadata.labels)]
        if not out:
            raise LookupError("Could not find service for pod")
        return out


class NodeInfo:
    """StaticNodeInfo / FakeNodeListInfo: GetNodeInfo by name (predicates.go:31-42)."""

    def __init__(self, nodes: Sequence[Node]):
        self.nodes = list(nodes)

    def get(self, name: str) -> Node:
        for n in self.nodes:
            if n.metadata.name == name:
                return n
        raise KeyError(f"failed to find node: {name}")


# ---- predicates (pkg/scheduler/predicates.go) --------------------------------
def is_volume_conflict(volume, pod: Pod) -> bool:  # predicates.go:52-66
    if volume.gce_persistent_disk is None:
        return False
    pd = volume.gce_persistent_disk.pd_name
    return any(v.gce_persistent_disk is not None and v.gce_persistent_disk.pd_name == pd for v in pod.spec.volumes)


def no_disk_conflict(pod: Pod, existing: List[Pod], node: str) -> bool:  # predicates.go:73-83
    for v in pod.spec.volumes:
        for e in existing:
            if is_volume_conflict(v, e):
                return False
    return True


def get_resource_request(pod: Pod) -> Tuple[int, int]:  # predicates.go:94-102
    cpu = mem = 0
    for c in pod.spec.containers:
        mem += c.resources.limits.memory().value()
        cpu += c.resources.limits.cpu().milli_value()
    return cpu, mem


def _i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def check_pods_exceeding_capacity(pods: List[Pod], capacity) -> Tuple[List[Pod], List[Pod]]:  # :104-124
    total_cpu = capacity.cpu().milli_value()
    total_mem = capacity.memory().value()
    req_cpu = req_mem = 0
    fitting, not_fitting = [], []
    for p in pods:
        pc, pm = get_resource_request(p)
        fits_cpu = total_cpu == 0 or _i64(total_cpu - req_cpu) >= pc
        fits_mem = total_mem == 0 or _i64(total_mem - req_mem) >= pm
        if not fits_cpu or not fits_mem:
            not_fitting.append(p)
            continue
        req_cpu = _i64(req_cpu + pc)
        req_mem = _i64(req_mem + pm)
        fitting.append(p)
    return fitting, not_fitting


def new_resource_fit_predicate(info: NodeInfo):  # predicates.go:127-152
    def pod_fits_resources(pod: Pod, existing: List[Pod], node: str) -> bool:
        cpu, mem = get_resource_request(pod)
        if cpu == 0 and mem == 0:
            return True
        n = info.get(node)
        _, exceeding = check_pods_exceeding_capacity(list(existing) + [pod], n.spec.capacity)
        return len(exceeding) == 0
    return pod_fits_resources


def pod_matches_node_labels(pod: Pod, node: Node) -> bool:  # predicates.go:161-167
    if not pod.spec.node_selector:
        return True
    return selector_from_set(pod.spec.node_selector).matches(node.metadata.labels)


def new_selector_match_predicate(info: NodeInfo):  # predicates.go:154-179
    def pod_selector_matches(pod: Pod, existing: List[Pod], node: str) -> bool:
        return pod_matches_node_labels(pod, info.get(node))
    return pod_selector_matches


def pod_fits_host(pod: Pod, existing: List[Pod], node: str) -> bool:  # predicates.go:181-186
    if len(pod.spec.host) == 0:
        return True
    return pod.spec.host == node


def new_node_label_predicate(info: NodeInfo, labels: Sequence[str], presence: bool):  # predicates.go:194-229
    def check_node_label_presence(pod: Pod, existing: List[Pod], node: str) -> bool:
        ml = info.get(node).metadata.labels
        for l in labels:
            exists = set_has(ml, l)
            if (exists and not presence) or (not exists and presence):
                return False
        return True
    return check_node_label_presence


def new_service_affinity_predicate(pod_lister: PodLister, service_lister: ServiceLister, info: NodeInfo,
                                   labels: Sequence[str]):  # predicates.go:238-324
    def check_service_affinity(pod: Pod, existing: List[Pod], node: str) -> bool:
        affinity = {}
        ns = pod.spec.node_selector or {}
        labels_exist = True
        for l in labels:
            if l in ns:
                affinity[l] = ns[l]
            else:
                labels_exist = False
        if not labels_exist:
            try:
                services = service_lister.get_pod_services(pod)
            except LookupError:
                services = None
            if services:
                sel = selector_from_set(services[0].spec.selector)
                peers = [p for p in pod_lister.list(sel) if p.metadata.namespace == pod.metadata.namespace]
                if peers:
                    other = info.get(peers[0].status.host)  # raises: the Go predicate returns err
                    for l in labels:
                        if l in affinity:
                            continue
                        if set_has(other.metadata.labels, l):
                            affinity[l] = set_get(other.metadata.labels, l)
        sel = everything() if not affinity else selector_from_set(affinity)
        return sel.matches(info.get(node).metadata.labels)
    check_service_affinity.may_error = True
    return check_service_affinity


def get_used_ports(*pods: Pod) -> Dict[int, bool]:  # predicates.go:340-350
    ports = {}
    for p in pods:
        for c in p.spec.containers:
            for cp in c.ports:
                ports[cp.host_port] = True
    return ports


def pod_fits_ports(pod: Pod, existing: List[Pod], node: str) -> bool:  # predicates.go:326-338
    existing_ports = get_used_ports(*existing)
    for wport in get_used_ports(pod):
        if wport == 0:
            continue
        if existing_ports.get(wport):
            return False
    return True


def map_pods_to_machines(lister: PodLister) -> Dict[str, List[Pod]]:  # predicates.go:354-375
    out: Dict[str, List[Pod]] = {}
    for p in lister.list(everything()):
        out.setdefault(p.status.host, []).append(p)
    return out


# ---- priorities (pkg/scheduler/priorities.go, spreading.go) -------------------
def calculate_score(requested: int, capacity: int) -> int:  # priorities.go:27-37
    if capacity == 0:
        return 0
    if requested > capacity:
        return 0
    prod = _i64((capacity - requested) * 10)
    q = abs(prod) // abs(capacity)
    return q if (prod >= 0) == (capacity > 0) else -q


def calculate_occupancy(pod: Pod, node: Node, pods: List[Pod]) -> Tuple[str, int]:  # priorities.go:43-76
    tc = tm = 0
    for e in pods:
        for c in e.spec.containers:
            tc += c.resources.limits.cpu().milli_value()
            tm += c.resources.limits.memory().value()
    for c in pod.spec.containers:
        tc += c.resources.limits.cpu().milli_value()
        tm += c.resources.limits.memory().value()
    cs = calculate_score(_i64(tc), node.spec.capacity.cpu().milli_value())
    ms = calculate_score(_i64(tm), node.spec.capacity.memory().value())
    return node.metadata.name, int((cs + ms) / 2)


def least_requested_priority(pod: Pod, pod_lister: PodLister, nodes: List[Node]):  # priorities.go:82-91
    m = map_pods_to_machines(pod_lister)
    return [calculate_occupancy(pod, n, m.get(n.metadata.name, [])) for n in nodes]


def new_node_label_priority(label: str, presence: bool):  # priorities.go:98-134
    def calculate_node_label_priority(pod: Pod, pod_lister: PodLister, nodes: List[Node]):
        out = []
        for n in nodes:
            exists = set_has(n.metadata.labels, label)
            ok = (exists and presence) or (not exists and not presence)
            out.append((n.metadata.name, 10 if ok else 0))
        return out
    return calculate_node_label_priority


def _f32_score(num: int, den: int) -> int:
    """int(10 * (float32(num) / float32(den))) (spreading.go:79-83, 156-160)."""
    q = np.float32(num) / np.float32(den)
    return int(np.float32(10) * np.float32(q))


def _ns_service_pods(pod: Pod, service_lister: ServiceLister, pod_lister: PodLister) -> List[Pod]:
    try:
        services = service_lister.get_pod_services(pod)
    except LookupError:
        return []
    sel = selector_from_set(services[0].spec.selector)
    return [p for p in pod_lister.list(sel) if p.metadata.namespace == pod.metadata.namespace]


def new_service_spread_priority(service_lister: ServiceLister):  # spreading.go:24-86
    def calculate_spread_priority(pod: Pod, pod_lister: PodLister, nodes: List[Node]):
        ns_pods = _ns_service_pods(pod, service_lister, pod_lister)
        counts: Dict[str, int] = {}
        max_count = 0
        for p in ns_pods:
            counts[p.status.host] = counts.get(p.status.host, 0) + 1
            max_count = max(max_count, counts[p.status.host])
        out = []
        for n in nodes:
            score = 10
            if max_count > 0:
                score = _f32_score(max_count - counts.get(n.metadata.name, 0), max_count)
            out.append((n.metadata.name, score))
        return out
    return calculate_spread_priority


def new_service_anti_affinity_priority(service_lister: ServiceLister, label: str):  # spreading.go:93-168
    def calculate_anti_affinity_priority(pod: Pod, pod_lister: PodLister, nodes: List[Node]):
        ns_pods = _ns_service_pods(pod, service_lister, pod_lister)
        other, labeled = [], {}
        for n in nodes:
            if set_has(n.metadata.labels, label):
                labeled[n.metadata.name] = set_get(n.metadata.labels, label)
            else:
                other.append(n.metadata.name)
        pod_counts: Dict[str, int] = {}
        for p in ns_pods:
            if p.status.host in labeled:
                v = labeled[p.status.host]
                pod_counts[v] = pod_counts.get(v, 0) + 1
        nsp = len(ns_pods)
        out = []
        for name, v in labeled.items():
            score = 10
            if nsp > 0:
                score = _f32_score(nsp - pod_counts.get(v, 0), nsp)
            out.append((name, score))
        out.extend((name, 0) for name in other)
        return out
    return calculate_anti_affinity_priority


def equal_priority(pod: Pod, pod_lister: PodLister, nodes: List[Node]):  # generic_scheduler.go:180-195
    return [(n.metadata.name, 1) for n in nodes]


# ---- generic scheduler (pkg/scheduler/generic_scheduler.go) ------------------
Predicate = Callable[[Pod, List[Pod], str], bool]
PriorityFn = Callable[[Pod, PodLister, List[Node]], List[Tuple[str, int]]]


def find_nodes_that_fit(pod: Pod, pod_lister: PodLister, predicates: Dict[str, Predicate],
                        nodes: List[Node]):  # generic_scheduler.go:100-128
    filtered, failed = [], {}
    m = map_pods_to_machines(pod_lister)
    for n in nodes:
        fits = True
        for name in sorted(predicates, key=lambda k: (not getattr(predicates[k], "may_error", False), k)):
            if not predicates[name](pod, m.get(n.metadata.name, []), n.metadata.name):
                fits = False
                failed.setdefault(n.metadata.name, set()).add(name)
                break
        if fits:
            filtered.append(n)
    return filtered, failed


def prioritize_nodes(pod: Pod, pod_lister: PodLister, configs: List[Tuple[PriorityFn, int]],
                     nodes: List[Node]) -> List[Tuple[str, int]]:  # generic_scheduler.go:136-165
    if len(configs) == 0:
        return equal_priority(pod, pod_lister, nodes)
    combined: Dict[str, int] = {}
    for fn, weight in configs:
        if weight == 0:
            continue
        for host, score in fn(pod, pod_lister, nodes):
            # Go int (int64) arithmetic wraps
            v = combined.get(host, 0) + score * weight
            combined[host] = ((v + (1 << 63)) % (1 << 64)) - (1 << 63)
    return list(combined.items())


def get_best_hosts(sorted_list: List[Tuple[str, int]]) -> List[str]:  # generic_scheduler.go:167-177
    return [h for h, s in sorted_list if s == sorted_list[0][1]]


class GenericScheduler:
    """genericScheduler (generic_scheduler.go:46-96, 197-204). `random` needs .int()."""

    def __init__(self, predicates: Dict[str, Predicate], prioritizers: List[Tuple[PriorityFn, int]],
                 pod_lister: PodLister, random):
        self.predicates = predicates
        self.prioritizers = prioritizers
        self.pods = pod_lister
        self.random = random

    def select_host(self, plist: List[Tuple[str, int]]) -> str:
        if not plist:
            raise ValueError("empty priorityList")
        # sort.Sort(sort.Reverse(...)) with Less = (score, host) ascending (types.go:42-47)
        srt = sorted(plist, key=lambda hs: (hs[1], hs[0].encode()), reverse=True)
        hosts = get_best_hosts(srt)
        ix = self.random.int() % len(hosts)
        return hosts[ix]

    def schedule(self, pod: Pod, nodes: List[Node]) -> str:
        if len(nodes) == 0:
            raise NoMinions("no minions available to schedule pods")
        filtered, failed = find_nodes_that_fit(pod, self.pods, self.predicates, nodes)
        plist = prioritize_nodes(pod, self.pods, self.prioritizers, filtered)
        if len(plist) == 0:
            raise FitError(pod, failed)
        return self.select_host(plist)


def default_provider(nodes: Sequence[Node], pod_lister: PodLister, service_lister: ServiceLister):
    """DefaultProvider (algorithmprovider/defaults/defaults.go:30-72) bound to listers."""
    info = NodeInfo(nodes)
    preds = {
        "PodFitsPorts": pod_fits_ports,
        "PodFitsResources": new_resource_fit_predicate(info),
        "NoDiskConflict": no_disk_conflict,
        "MatchNodeSelector": new_selector_match_predicate(info),
        "HostName": pod_fits_host,
    }
    # priorities in sorted name order (plugins.go:235-248)
    prios = [(equal_priority, 0), (least_requested_priority, 1), (new_service_spread_priority(service_lister), 1)]
    return preds, prios


def from_config(config, nodes: Sequence[Node], pod_lister: PodLister, service_lister: ServiceLister):
    """Bind a kubernetes_amd.factory.SchedulerConfig to these functions, as the factory's
    getFitPredicateFunctions / getPriorityFunctionConfigs do (plugins.go:220-248)."""
    info = NodeInfo(nodes)
    preds: Dict[str, Predicate] = {}
    for name, d in config.predicates.items():
        if d.kind == "PodFitsPorts":
            preds[name] = pod_fits_ports
        elif d.kind == "PodFitsResources":
            preds[name] = new_resource_fit_predicate(info)
        elif d.kind == "NoDiskConflict":
            preds[name] = no_disk_conflict
        elif d.kind == "MatchNodeSelector":
            preds[name] = new_selector_match_predicate(info)
        elif d.kind == "HostName":
            preds[name] = pod_fits_host
        elif d.kind == "ServiceAffinity":
            preds[name] = new_service_affinity_predicate(pod_lister, service_lister, info, d.labels)
        elif d.kind == "LabelsPresence":
            preds[name] = new_node_label_predicate(info, d.labels, d.presence)
        else:
            raise ValueError(d.kind)
    prios: List[Tuple[PriorityFn, int]] = []
    for d in config.priorities:
        if d.kind == "LeastRequestedPriority":
            fn = least_requested_priority
        elif d.kind == "ServiceSpreadingPriority":
            fn = new_service_spread_priority(service_lister)
        elif d.kind == "EqualPriority":
            fn = equal_priority
        elif d.kind == "ServiceAntiAffinity":
            fn = new_service_anti_affinity_priority(service_lister, d.label)
        elif d.kind == "LabelPreference":
            fn = new_node_label_priority(d.label, d.presence)
        else:
            raise ValueError(d.kind)
        prios.append((fn, d.weight))
    return preds, prios
