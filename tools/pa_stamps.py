"""Phase-A wave stamps (KSG_DEBUG=64, ksg_window.hip): mean cycles per wave from its start to
every load landed (the scoring loop's start) and from there to its stores, and waves per
launch, over a few bench-shaped batches of one workload. Diagnostic only.
usage: python tools/pa_stamps.py [config5] [batches]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["KSG_DEBUG"] = str(int(os.environ.get("KSG_DEBUG", "0")) | 64)

import numpy as np  # noqa: E402

from kubernetes_amd import ingest, workload  # noqa: E402
from kubernetes_amd.engine import DeviceScheduler, PodBatch  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "config5"
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    w = workload.build(wl, n_pods=1000 * (nb + 1))
    it = ingest.Interner()
    for k in w.config.label_keys():
        it.key_id(k)
    view = ingest.ClusterView(w.nodes, w.services, it)
    batch = ingest.ingest_pods(view, w.pods, aff_labels=w.config.affinity_labels())
    s = DeviceScheduler(w.config.compile(it.key_id), device=0)
    s.set_cluster(view.arrays)
    rng = workload.TIEBREAK_SEED
    _, rng = s.batch(PodBatch(batch.pods[:1000], batch.ids, None), rng)  # (warm)
    c0 = s.debug_counters().astype(np.int64)
    launches = 0
    t = time.time()
    for b in range(1, nb + 1):
        _, rng = s.batch(PodBatch(batch.pods[1000 * b:1000 * (b + 1)], batch.ids, None), rng)
        launches += s.last_batch_stats()["windows"]
    c = s.debug_counters().astype(np.int64) - c0
    waves = int(c[50])
    print(f"{wl}: launches {launches} waves/launch {waves / max(launches, 1):.0f} "
          f"load cycles/wave {16 * c[48] / max(waves, 1):.0f} score cycles/wave {16 * c[49] / max(waves, 1):.0f} "
          f"({time.time() - t:.1f}s)")
    s.close()


if __name__ == "__main__":
    main()
