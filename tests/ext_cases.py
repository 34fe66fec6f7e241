"""Seeded workloads with the extensions (taints / tolerations, extended
resources, BalancedResourceAllocation) on top of a BASELINE-shaped cluster.
Parity unpinned (kubernetes_amd/extensions.py): the C restatement is the checker."""
from __future__ import annotations

from kubernetes_amd import workload
from kubernetes_amd.engine import PodBatch
from kubernetes_amd.extensions import (NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, ExtConfig, ExtInterner, Taint,
                                       Toleration)
from tests.helpers import Case

GPU = "nvidia.com/gpu"


class ExtCase:
    def __init__(self, name="config2", nn=700, npods=900, seed=11, w_taint=1, w_bal=1, taints=True, gpus=True,
                 base_policy=None):
        self.case = Case(name, nn, npods)
        rng = workload._SM(seed)
        self.ecfg = ExtConfig(taints=taints, scalar_resources=(GPU, "example.com/fpga") if gpus else (),
                              w_taint_toleration=w_taint, w_balanced=w_bal)
        pool = [Taint("dedicated", "db", NO_SCHEDULE), Taint("dedicated", "ml", NO_SCHEDULE),
                Taint("maint", "", NO_EXECUTE), Taint("spot", "true", PREFER_NO_SCHEDULE),
                Taint("slow-disk", "", PREFER_NO_SCHEDULE), Taint("zone-drain", "z1", PREFER_NO_SCHEDULE)]
        node_taints = []
        for _ in range(nn):
            k = rng.below(4)
            node_taints.append(list({pool[rng.below(len(pool))] for _ in range(k)}))
        node_scalar = {GPU: [[0, 0, 4, 8][rng.below(4)] for _ in range(nn)],
                       "example.com/fpga": [rng.below(3) for _ in range(nn)]}
        tol_pool = [Toleration("dedicated", "Equal", "db", NO_SCHEDULE), Toleration("dedicated", "Exists"),
                    Toleration("maint", "Exists", "", NO_EXECUTE), Toleration("spot", "Equal", "true"),
                    Toleration("", "Exists"), Toleration("slow-disk", "Exists", "", PREFER_NO_SCHEDULE),
                    Toleration("zone-drain", "Equal", "z2")]
        tols, scal = [], []
        for _ in range(npods):
            k = rng.below(3) if rng.below(10) else 0
            tols.append([tol_pool[rng.below(len(tol_pool) - 1) if rng.below(20) else len(tol_pool) - 2]
                         for _ in range(k)])
            g = [0, 0, 0, 1, 2][rng.below(5)]
            scal.append({GPU: g, "example.com/fpga": 1 if rng.below(10) == 0 else 0})
        self.inter = ExtInterner(self.ecfg)
        self.node_arrays = self.inter.node_arrays(node_taints, node_scalar if gpus else None)
        rec, ids = self.inter.pod_records(self.case.batch.ids, tols, scal)
        self.batch = PodBatch(self.case.batch.pods, ids, rec)
        self.cfg = self.case.cfg
        self.kcfg = self.ecfg.compile(max(len(self.inter.taints), 1))

    def load(self, sched):
        sched.set_extensions(self.kcfg)
        sched.set_cluster(self.case.view.arrays)
        sched.set_node_ext(*self.node_arrays)
        return sched
