"""Debug helper: window path vs oracle on a small config, per window size."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.helpers import Case, run_batch
from kubernetes_amd.engine import DeviceScheduler, PodBatch
from oracle.pyoracle import OracleScheduler

name = sys.argv[1] if len(sys.argv) > 1 else "config1"
case = Case(name, 500, 60)
orc = OracleScheduler(case.cfg); want, sw = run_batch(orc, case)
for W in (1, 2, 3, 4, 6, 8, 16, 1024):
    dev = DeviceScheduler(case.cfg); dev.set_window(W)
    got, sg = run_batch(dev, case)
    bad = np.nonzero(got != want)[0]
    print(W, "stats", dev.last_batch_stats(), "first bad", bad[:5], got[bad[:5]], want[bad[:5]], flush=True)
    dev.close()
# per-pod k/m from oracle for first pods
orc = OracleScheduler(case.cfg); orc.set_cluster(case.view.arrays)
rng = 1234
for i in range(8):
    rc, m, k, _ = orc.begin(case.batch, i)
    print("pod", i, "M", m, "k", k, "req", case.batch.pods[i]["milli_cpu"], case.batch.pods[i]["memory"])
    o, rng = orc.batch(PodBatch(case.batch.pods[i:i+1], case.batch.ids), rng) if False else (None, rng)
