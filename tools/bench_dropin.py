#!/usr/bin/env python3
"""Per-pod drop-in throughput: GPUScheduler.schedule (ksg_schedule_begin/commit, one
pod per call, as scheduleOne drives algorithm.Scheduler) with the two pod sources:

  relist   a plain PodLister re-listed and diffed on every call (the reference's own
           per-pod MapPodsToMachines cost structure, predicates.go:354-375);
  modeler  SimpleModeler's PodLister: the device mirror follows the stores' events
           (kubernetes_amd/modeler.py), O(events + assumed pods) per call.

Each scheduled pod is assumed (AssumePod) and later delivered by the scheduled-pod
"reflector", so the pod count the scheduler sees grows as it runs.
usage: python tools/bench_dropin.py [--nodes 5000] [--pods 2000]   (needs a GPU)
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubernetes_amd import workload  # noqa: E402
from kubernetes_amd.api import PodStatus  # noqa: E402
from kubernetes_amd.modeler import SimpleModeler, StoreToPodLister  # noqa: E402
from kubernetes_amd.scheduler import (FakeMinionLister, FakePodLister, FakeServiceLister, GPUScheduler,  # noqa: E402
                                      SplitMix64Rand)


def run(mode, w, n_pods):
    minions = FakeMinionLister(w.nodes)
    if mode == "modeler":
        q, s = StoreToPodLister(), StoreToPodLister()
        m = SimpleModeler(q, s)
        lister = m.pod_lister()
    else:
        plain = FakePodLister([])
        lister = plain
    g = GPUScheduler(w.config, lister, FakeServiceLister(w.services), SplitMix64Rand(7))
    hosts = []
    lag = []
    t0 = time.perf_counter()
    for p in w.pods[:n_pods]:
        h = g.schedule(p, minions)
        hosts.append(h)
        a = copy.copy(p)
        a.status = PodStatus(host=h)
        if mode == "modeler":
            m.assume_pod(a)
            lag.append(a)
            if len(lag) > 8:  # the reflector delivers the binding a few pods later
                s.store.add(copy.copy(lag.pop(0)))
        else:
            plain.pods.append(a)
    dt = time.perf_counter() - t0
    g.close()
    return n_pods / dt, hosts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=2000)
    args = ap.parse_args()
    w = workload.build("config2", n_nodes=args.nodes, n_pods=args.pods)
    run("modeler", w, 50)  # warm-up (library load, first launches)
    res = {}
    for mode in ("relist", "modeler"):
        rate, hosts = run(mode, w, args.pods)
        res[mode] = {"pods_per_s": rate}
        res[mode + "_hosts"] = hosts
    same = res.pop("relist_hosts") == res.pop("modeler_hosts")
    print(json.dumps({"metric": "drop-in GPUScheduler.schedule pods/s (one pod per call)",
                      "nodes": args.nodes, "pods": args.pods, "identical_decisions": same, **res}))


if __name__ == "__main__":
    main()
