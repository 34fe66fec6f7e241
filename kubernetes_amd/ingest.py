"""Host ingest: api objects -> interned C-ABI arrays.

What the reference evaluates with strings and big decimals on every predicate
call is converted once here:
  * node rank = index in byte-wise ascending name order, so the reference's
    tie order "score desc, host desc" (types.go:42-47) becomes "rank desc";
  * capacities / limits -> int64 via Quantity.MilliValue (cpu) and Value
    (memory) (resource_helpers.go:29-42, predicates.go:94-102);
  * label (key,value) pairs, label keys, host ports, GCE PD names -> dense ids;
  * nodeSelector -> pair ids, honouring SelectorFromSet's "invalid => match
    everything" trap (selector.go:654-668); a value no node carries -> pair 0;
  * services a pod matches: same namespace and SelectorFromSet(selector)
    matches the pod's labels (cache/listers.go:109-129); services[0] is the
    first matching service in ServiceLister order (the reference iterates a Go
    map here; SURVEY.md 8(a) trap ii).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np

from . import abi
from .api import Node, Pod, Service
from .engine import ClusterArrays, PodBatch
from .labels import is_qualified_name, is_valid_label_value, selector_from_set


def pair_is_valid(key: str, value: str) -> bool:
    """NewRequirement(key, =, {value}) succeeds (selector.go:91-115, 638-650)."""
    return is_qualified_name(key) and is_valid_label_value(value)


class Interner:
    """Persistent id spaces shared by the config, the cluster and every pod."""

    def __init__(self):
        self.label_keys: Dict[str, int] = {}
        self.pairs: Dict[tuple, int] = {}
        self.pair_key: List[int] = [0xFFFFFFFF]  # pair 0: "no node has it"
        self.conflict: Dict[tuple, int] = {}
        self.ext_hosts: Dict[str, int] = {}

    def key_id(self, key: str) -> int:
        kid = self.label_keys.get(key)
        if kid is None:
            kid = self.label_keys[key] = len(self.label_keys)
        return kid

    def pair_id(self, key: str, value: str, create: bool) -> int:
        pid = self.pairs.get((key, value))
        if pid is None:
            if not create:
                return 0
            pid = self.pairs[(key, value)] = len(self.pair_key)
            kid = self.key_id(key)
            # SelectorFromSet rejects this (key, value) (selector.go:654-668): flagged so
            # a ServiceAffinity selector built from a peer node's label matches everything
            if not pair_is_valid(key, value):
                kid |= abi.PAIR_INVALID
            self.pair_key.append(kid)
        return pid

    def conflict_id(self, kind: str, value) -> int:
        cid = self.conflict.get((kind, value))
        if cid is None:
            cid = self.conflict[(kind, value)] = len(self.conflict)
        return cid


class ClusterView:
    """A node list + service list, interned. Holds name->rank for pod ingest."""

    def __init__(self, nodes: Sequence[Node], services: Sequence[Service], interner: Interner):
        self.interner = interner
        self.nodes = sorted(nodes, key=lambda n: n.metadata.name.encode())
        self.names = [n.metadata.name for n in self.nodes]
        self.rank = {name: i for i, name in enumerate(self.names)}
        self.services = list(services)
        self._svc_sel = [(s.metadata.namespace, selector_from_set(s.spec.selector)) for s in self.services]
        # GetPodServices index: a service can only match a pod that carries its
        # selector's first requirement; empty selectors (incl. SelectorFromSet's
        # invalid-label trap) match every pod of the namespace
        self._svc_first: Dict[tuple, List[int]] = {}
        self._svc_all: Dict[str, List[int]] = {}
        for i, (sns, sel) in enumerate(self._svc_sel):
            if sel.empty():
                self._svc_all.setdefault(sns, []).append(i)
            else:
                k, v = sel.requirements[0]
                self._svc_first.setdefault((sns, k, v), []).append(i)
        arr = np.zeros(len(self.nodes), dtype=abi.NODE_DTYPE)
        pairs: List[int] = []
        for i, n in enumerate(self.nodes):
            cap = n.spec.capacity
            arr[i]["cap_milli_cpu"] = cap.cpu().milli_value()
            arr[i]["cap_memory"] = cap.memory().value()
            arr[i]["label_off"] = len(pairs)
            labels = n.metadata.labels or {}
            for k in sorted(labels):
                pairs.append(interner.pair_id(k, labels[k], create=True))
            arr[i]["n_labels"] = len(labels)
        self.arrays = ClusterArrays(
            nodes=arr,
            node_pairs=np.asarray(pairs, dtype=np.uint32),
            pair_keys=np.asarray(interner.pair_key, dtype=np.uint32),
            n_services=len(self.services),
            names=self.names,
        )

    # ---- pods ---------------------------------------------------------------
    def host_id(self, host: str) -> int:
        """Status.Host -> node rank, or an id >= N for hosts not in the node list."""
        r = self.rank.get(host)
        if r is not None:
            return r
        ext = self.interner.ext_hosts
        if host not in ext:
            ext[host] = len(ext)
        return len(self.names) + ext[host]

    def pod_services(self, pod: Pod) -> List[int]:
        """Indices (service-list order) of the services selecting the pod: same
        namespace, selector matches its labels (GetPodServices, listers.go:63-91)."""
        ns = pod.metadata.namespace
        labels = pod.metadata.labels or {}
        cand = list(self._svc_all.get(ns, ()))
        for k, v in labels.items():
            c = self._svc_first.get((ns, k, v))
            if c:
                cand.extend(c)
        if not cand:
            return []
        sel = self._svc_sel
        return sorted(i for i in set(cand) if sel[i][1].matches(labels))


class PodBatchBuilder:
    """Accumulates interned pods (pending or existing) into a PodBatch."""

    def __init__(self, view: ClusterView, aff_labels: Sequence[str] = ()):
        self.view = view
        self.aff_labels = list(aff_labels)
        self.rows: List[tuple] = []
        self.ids: List[int] = []

    def add(self, pod: Pod, uid: int) -> int:
        v = self.view
        it = v.interner
        cpu = mem = 0
        ports: List[int] = []
        for c in pod.spec.containers:  # getResourceRequest (predicates.go:94-102)
            lim = c.resources.limits
            mem += lim.memory().value()
            cpu += lim.cpu().milli_value()
            for p in c.ports:  # getUsedPorts (predicates.go:340-350); port 0 never checked
                if p.host_port != 0:
                    ports.append(it.conflict_id("port", int(p.host_port)))
        pds = [it.conflict_id("pd", vol.gce_persistent_disk.pd_name)
               for vol in pod.spec.volumes if vol.gce_persistent_disk is not None]
        ns = pod.spec.node_selector
        sel: List[int] = []
        if ns:  # PodMatchesNodeLabels (predicates.go:161-167)
            s = selector_from_set(ns)
            sel = [it.pair_id(k, val, create=False) for k, val in s.requirements]
        svcs = v.pod_services(pod)
        host = pod.spec.host
        host_code = -1 if host == "" else v.rank.get(host, -2)
        aff = [-1] * abi.MAX_AFF
        for j, l in enumerate(self.aff_labels):  # CheckServiceAffinity (predicates.go:261-271)
            if ns and l in ns:
                # an invalid value empties the predicate's selector (predicates.go:314)
                aff[j] = it.pair_id(l, ns[l], create=False) if pair_is_valid(l, ns[l]) else abi.AFF_INVALID
        base = len(self.ids)
        self.ids.extend(ports)
        self.ids.extend(pds)
        self.ids.extend(sel)
        self.ids.extend(svcs)
        self.rows.append((
            uid, cpu, mem, host_code, svcs[0] if svcs else -1,
            base, len(ports),
            base + len(ports), len(pds),
            base + len(ports) + len(pds), len(sel),
            base + len(ports) + len(pds) + len(sel), len(svcs),
            tuple(aff),
        ))
        return len(self.rows) - 1

    def build(self) -> PodBatch:
        arr = np.zeros(len(self.rows), dtype=abi.POD_DTYPE)
        for i, r in enumerate(self.rows):
            arr[i] = r
        return PodBatch(arr, np.asarray(self.ids, dtype=np.uint32))


def ingest_pods(view: ClusterView, pods: Sequence[Pod], uids: Optional[Sequence[int]] = None,
                aff_labels: Sequence[str] = ()) -> PodBatch:
    b = PodBatchBuilder(view, aff_labels)
    for i, p in enumerate(pods):
        b.add(p, uids[i] if uids is not None else i + 1)
    return b.build()
