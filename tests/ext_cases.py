"""Seeded workloads with the extensions (taints / tolerations, extended
resources, BalancedResourceAllocation) on top of a BASELINE-shaped cluster
(kubernetes_amd.workload.extension_data). Parity unpinned
(kubernetes_amd/extensions.py): the C restatement is the checker."""
from __future__ import annotations

from kubernetes_amd import workload
from kubernetes_amd.engine import PodBatch
from kubernetes_amd.extensions import ExtInterner
from tests.helpers import Case


class ExtCase:
    def __init__(self, name="config2", nn=700, npods=900, seed=11, w_taint=1, w_bal=1, taints=True, gpus=True):
        self.case = Case(name, nn, npods)
        self.ecfg, node_taints, node_scalar, tols, scal = workload.extension_data(
            nn, npods, seed, taints=taints, gpus=gpus, w_taint=w_taint, w_bal=w_bal)
        self.inter = ExtInterner(self.ecfg)
        self.node_arrays = self.inter.node_arrays(node_taints, node_scalar)
        rec, ids = self.inter.pod_records(self.case.batch.ids, tols, scal)
        self.batch = PodBatch(self.case.batch.pods, ids, rec)
        self.cfg = self.case.cfg
        self.kcfg = self.ecfg.compile(max(len(self.inter.taints), 1))

    def load(self, sched):
        sched.set_extensions(self.kcfg)
        sched.set_cluster(self.case.view.arrays)
        sched.set_node_ext(*self.node_arrays)
        return sched
