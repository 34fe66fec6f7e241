"""The kubelet's admission re-check with the scheduler's predicates, on the device.

Reference (pkg/kubelet/kubelet.go):
  handleNotFittingPods                          :1745-1771
    checkHostPortConflicts                      :1697-1713  kubelet-only (validation.AccumulateUniquePorts):
                                                            not a scheduler predicate, not reimplemented
    checkNodeSelectorMatching                   :1731-1744  -> scheduler.PodMatchesNodeLabels (predicates.go:161-167)
    checkCapacityExceeded                       :1716-1729  -> sort.Sort(podsByCreationTime) +
                                                               scheduler.CheckPodsExceedingCapacity (predicates.go:104-124)
  CapacityFromMachineInfo                       pkg/kubelet/util.go:48-58

Both predicates run in ksg_admit_kernel (ksg_admit.hip) through the C ABI
(ksg_pod_matches_node_labels / ksg_check_pods_exceeding_capacity / ksg_admit_pods);
many nodes' sets go in one launch (`admit_many`). There is no host evaluation.
podsByCreationTime is sorted with a stable sort: Go's sort.Sort gives no order
among equal timestamps (it is stable only below 12 pods); ties keep list order here.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .api import Node, Pod, ResourceList
from .engine import DeviceScheduler, PodBatch
from .ingest import Interner
from .labels import selector_from_set
from .resource import Quantity


@dataclass
class MachineInfo:
    """cadvisor MachineInfo fields CapacityFromMachineInfo reads."""
    num_cores: int = 0
    memory_capacity: int = 0


def capacity_from_machine_info(info: MachineInfo) -> ResourceList:  # kubelet/util.go:48-58
    return ResourceList(cpu=Quantity.from_milli(int(info.num_cores) * 1000), memory=Quantity.from_int(info.memory_capacity))


def pods_by_creation_time(pods: Sequence[Pod]) -> List[Pod]:  # kubelet.go:1684-1694
    return sorted(pods, key=lambda p: p.metadata.creation_timestamp)


class KubeletAdmission:
    """The scheduler predicates of handleNotFittingPods over many nodes at once."""

    def __init__(self, engine: Optional[DeviceScheduler] = None, device: int = 0, build_only: bool = False):
        """build_only: intern sets into ABI arrays (build()) without a device context."""
        if engine is None and not build_only:
            from .factory import create_from_keys

            engine = DeviceScheduler(create_from_keys([], []).compile(lambda k: 0), device=device)
        self.engine = engine
        self.interner = Interner()

    def close(self):
        if self.engine is not None:
            self.engine.close()

    # ---- ingest -------------------------------------------------------------
    def _pod_rows(self, pods: Sequence[Pod], rows: list, ids: list):
        it = self.interner
        for p in pods:
            cpu = mem = 0
            for c in p.spec.containers:  # getResourceRequest (predicates.go:94-102)
                cpu += c.resources.limits.cpu().milli_value()
                mem += c.resources.limits.memory().value()
            sel = []
            if p.spec.node_selector:  # SelectorFromSet: invalid => matches everything
                sel = [it.pair_id(k, v, create=False) for k, v in selector_from_set(p.spec.node_selector).requirements]
            rows.append((0, cpu, mem, -1, -1, 0, 0, 0, 0, len(ids), len(sel), 0, 0, (-1,) * abi.MAX_AFF))
            ids.extend(sel)

    def build(self, sets: Sequence[Tuple[Optional[Node], ResourceList, Sequence[Pod]]]):
        """Intern (node, capacity, pods-in-order) sets into the ABI arrays:
        -> (ADMISSION_SET_DTYPE[n_sets], PodBatch, node label pairs)."""
        it = self.interner
        pairs: List[int] = []
        set_rows = []
        for node, cap, _ in sets:  # intern every node's labels first: selectors look them up
            labels = (node.metadata.labels or {}) if node is not None else {}
            set_rows.append((len(pairs), len(labels)))
            pairs.extend(it.pair_id(k, labels[k], create=True) for k in sorted(labels))
        rows: list = []
        ids: List[int] = []
        arr = np.zeros(len(sets), abi.ADMISSION_SET_DTYPE)
        for s, (node, cap, pods) in enumerate(sets):
            arr[s] = (cap.cpu().milli_value(), cap.memory().value(), len(rows), len(pods), *set_rows[s])
            self._pod_rows(pods, rows, ids)
        parr = np.zeros(len(rows), abi.POD_DTYPE)
        for i, r in enumerate(rows):
            parr[i] = r
        return arr, PodBatch(parr, np.asarray(ids, np.uint32)), np.asarray(pairs, np.uint32)

    def admit_many(self, sets: Sequence[Tuple[Optional[Node], ResourceList, Sequence[Pod]]], mode: int = 3):
        """One device pass over (node, capacity, pods-in-order) sets. -> codes per set:
        mode 3: KSG_ADMIT_* (selector, then capacity over the matching pods); mode 1:
        1 = fits (capacity only); mode 2: 1 = nodeSelector matches."""
        arr, batch, pairs = self.build(sets)
        out = self.engine.admit(arr, batch, pairs, mode)
        res, at = [], 0
        for _, _, pods in sets:
            res.append(out[at:at + len(pods)])
            at += len(pods)
        return res

    # ---- the kubelet's checks, one node -------------------------------------
    def check_node_selector_matching(self, pods: Sequence[Pod], node: Node) -> Tuple[List[Pod], List[Pod]]:
        (m,) = self.admit_many([(node, ResourceList(), pods)], mode=2)
        return [p for p, ok in zip(pods, m) if ok], [p for p, ok in zip(pods, m) if not ok]

    def check_capacity_exceeded(self, pods: Sequence[Pod], capacity: ResourceList) -> Tuple[List[Pod], List[Pod]]:
        pods = pods_by_creation_time(pods)
        (f,) = self.admit_many([(None, capacity, pods)], mode=1)
        return [p for p, ok in zip(pods, f) if ok], [p for p, ok in zip(pods, f) if not ok]

    def handle_not_fitting_pods(self, pods: Sequence[Pod], node: Node, capacity: ResourceList) -> Dict[str, str]:
        """-> {namespace/name: event reason} for the pods the kubelet fails
        ("nodeSelectorMismatching", "capacityExceeded"), in the kubelet's order."""
        return self.handle_many([(node, capacity, pods)])[0]

    def handle_many(self, sets: Sequence[Tuple[Node, ResourceList, Sequence[Pod]]]) -> List[Dict[str, str]]:
        ordered = [(n, c, pods_by_creation_time(pods)) for n, c, pods in sets]
        out = []
        for (_, _, pods), codes in zip(ordered, self.admit_many(ordered, mode=3)):
            why = {}
            for p, code in zip(pods, codes):
                if code == abi.ADMIT_NODESELECTOR:
                    why[p.key()] = "nodeSelectorMismatching"
                elif code == abi.ADMIT_CAPACITY:
                    why[p.key()] = "capacityExceeded"
            out.append(why)
        return out
