"""Extensions beyond this reference vintage: taints / tolerations, extended
(scalar) resources and BalancedResourceAllocation.

smarterclayton/kubernetes v0.13 has none of these; BASELINE.json's configs name
them. Their semantics follow the published kube-scheduler v1.10 algorithms
(api/core/v1 Toleration.ToleratesTaint, algorithm/predicates
PodToleratesNodeTaints + PodFitsResources' ScalarResources, algorithm/priorities
TaintTolerationPriority + NormalizeReduce, BalancedResourceAllocation). No
reference or test table exists here to pin them: PARITY IS UNPINNED, the C
restatement of the tests' checker is the only one. They are off unless a
context enables them (DeviceScheduler.set_extensions), and they run on the exact
one-pod-at-a-time kernels.

This module turns taints, tolerations and extended resources into the ABI's
interned form: every distinct node taint gets an id, each node lists its taint
ids, and each pod lists the taint ids its tolerations do NOT tolerate (hard:
NoSchedule / NoExecute; soft: PreferNoSchedule against the tolerations whose
effect is empty or PreferNoSchedule).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import abi

NO_SCHEDULE = "NoSchedule"
PREFER_NO_SCHEDULE = "PreferNoSchedule"
NO_EXECUTE = "NoExecute"


@dataclass(frozen=True)
class Taint:
    key: str
    value: str = ""
    effect: str = NO_SCHEDULE


@dataclass(frozen=True)
class Toleration:
    key: str = ""
    operator: str = ""  # "" / "Equal" / "Exists"
    value: str = ""
    effect: str = ""    # "": every effect


def tolerates(t: Toleration, taint: Taint) -> bool:
    """Toleration.ToleratesTaint (v1.10): effect empty or equal, key empty or
    equal, then Exists tolerates any value and Equal (or "") needs the value."""
    if t.effect and t.effect != taint.effect:
        return False
    if t.key and t.key != taint.key:
        return False
    if t.operator in ("", "Equal"):
        return t.value == taint.value
    if t.operator == "Exists":
        return True
    return False


def tolerated_by_any(tols: Sequence[Toleration], taint: Taint) -> bool:
    return any(tolerates(t, taint) for t in tols)


@dataclass
class ExtConfig:
    """Which extensions a context runs (compiled to abi.KsgExtConfig)."""
    taints: bool = False
    scalar_resources: Sequence[str] = ()   # extended resource names, e.g. ("nvidia.com/gpu",)
    w_taint_toleration: int = 0
    w_balanced: int = 0

    def compile(self, max_taints: int) -> abi.KsgExtConfig:
        if len(self.scalar_resources) > abi.MAX_SCALAR:
            raise ValueError(f"at most {abi.MAX_SCALAR} extended resources")
        e = abi.KsgExtConfig()
        e.filters = (abi.EXT_TAINTS if self.taints else 0) | (abi.EXT_SCALAR if self.scalar_resources else 0)
        e.w_taint_toleration = int(self.w_taint_toleration)
        e.w_balanced = int(self.w_balanced)
        e.n_scalar = len(self.scalar_resources)
        e.max_taints = max_taints
        return e


class ExtInterner:
    """Interns node taints; builds the node-side arrays and the pods' records."""

    def __init__(self, cfg: ExtConfig):
        self.cfg = cfg
        self.taint_id: Dict[Taint, int] = {}
        self.taints: List[Taint] = []

    def intern(self, t: Taint) -> int:
        if t not in self.taint_id:
            self.taint_id[t] = len(self.taints)
            self.taints.append(t)
        return self.taint_id[t]

    def node_arrays(self, node_taints: Sequence[Sequence[Taint]],
                    node_scalar: Optional[Dict[str, Sequence[int]]] = None):
        """-> (scalar_cap int64[n_scalar, N], taint_off, taint_n, taint_ids) for set_node_ext."""
        n = len(node_taints)
        off = np.zeros(n, np.uint32)
        cnt = np.zeros(n, np.uint32)
        ids: List[int] = []
        for i, ts in enumerate(node_taints):
            off[i] = len(ids)
            for t in ts:
                ids.append(self.intern(t))
            cnt[i] = len(ts)
        cap = np.zeros((max(len(self.cfg.scalar_resources), 1), n), np.int64)
        for r, name in enumerate(self.cfg.scalar_resources):
            if node_scalar and name in node_scalar:
                cap[r] = np.asarray(node_scalar[name], np.int64)
        return cap[: len(self.cfg.scalar_resources)], off, cnt, np.asarray(ids, np.uint32)

    def pod_records(self, ids: np.ndarray, tolerations: Sequence[Sequence[Toleration]],
                    scalar: Optional[Sequence[Dict[str, int]]] = None):
        """-> (POD_EXT_DTYPE[n], ids extended with the pods' untolerated taint lists).
        Call after node_arrays (every node taint interned)."""
        n = len(tolerations)
        rec = np.zeros(n, abi.POD_EXT_DTYPE)
        extra: List[int] = []
        base = len(ids)
        soft_tols_of = lambda tols: [t for t in tols if t.effect in ("", PREFER_NO_SCHEDULE)]
        for i, tols in enumerate(tolerations):
            hard = [self.taint_id[t] for t in self.taints if t.effect in (NO_SCHEDULE, NO_EXECUTE)
                    and not tolerated_by_any(tols, t)]
            stols = soft_tols_of(tols)
            soft = [self.taint_id[t] for t in self.taints if t.effect == PREFER_NO_SCHEDULE
                    and not tolerated_by_any(stols, t)]
            rec[i]["hard_off"] = base + len(extra)
            rec[i]["n_hard"] = len(hard)
            extra.extend(hard)
            rec[i]["soft_off"] = base + len(extra)
            rec[i]["n_soft"] = len(soft)
            extra.extend(soft)
            if scalar is not None:
                for r, name in enumerate(self.cfg.scalar_resources):
                    rec[i]["scalar"][r] = int(scalar[i].get(name, 0))
        all_ids = np.concatenate([np.asarray(ids, np.uint32), np.asarray(extra, np.uint32)])
        return rec, all_ids
