"""Shared builders for parity tests: a workload -> (config, cluster arrays, pod batch)."""
from __future__ import annotations

import numpy as np

from kubernetes_amd import ingest, workload


class Case:
    def __init__(self, name, n_nodes=None, n_pods=None, seed=workload.WORKLOAD_SEED, existing=0):
        self.w = workload.build(name, n_nodes=n_nodes, n_pods=n_pods, seed=seed)
        self.it = ingest.Interner()
        for k in self.w.config.label_keys():
            self.it.key_id(k)
        self.view = ingest.ClusterView(self.w.nodes, self.w.services, self.it)
        aff = self.w.config.affinity_labels()
        self.batch = ingest.ingest_pods(self.view, self.w.pods, aff_labels=aff)
        self.cfg = self.w.config.compile(self.it.key_id)
        self.aff = aff


def run_batch(sched, case: Case, rng=workload.TIEBREAK_SEED, chunk=None):
    sched.set_cluster(case.view.arrays)
    if chunk is None:
        return sched.batch(case.batch, rng)
    outs = []
    for s in range(0, len(case.batch), chunk):
        sub = type(case.batch)(case.batch.pods[s:s + chunk], case.batch.ids)
        o, rng = sched.batch(sub, rng)
        outs.append(o)
    return np.concatenate(outs), rng
