"""Debug helper: window path vs oracle; first mismatch, window stats, and the
state / scores right before it."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from kubernetes_amd.engine import DeviceScheduler, PodBatch
from oracle.pyoracle import OracleScheduler
from tests.helpers import Case, run_batch

name = sys.argv[1] if len(sys.argv) > 1 else "config1"
nn = int(sys.argv[2]) if len(sys.argv) > 2 else 500
npods = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
case = Case(name, nn, npods)
orc = OracleScheduler(case.cfg)
want, sw = run_batch(orc, case)
first = None
for W in (1024, 128, 16, 2):
    dev = DeviceScheduler(case.cfg)
    dev.set_window(W)
    got, sg = run_batch(dev, case)
    bad = np.nonzero(got != want)[0]
    print("W", W, "stats", dev.last_batch_stats(), "rng ok", sg == sw, "n bad", bad.size, "first", bad[:5],
          got[bad[:5]], want[bad[:5]], flush=True)
    if bad.size and first is None:
        first = (W, int(bad[0]))
    dev.close()
if first:
    W, b = first
    pre = PodBatch(case.batch.pods[:b], case.batch.ids)
    dev = DeviceScheduler(case.cfg)
    dev.set_window(W)
    dev.set_cluster(case.view.arrays)
    o2 = OracleScheduler(case.cfg)
    o2.set_cluster(case.view.arrays)
    g, rg = dev.batch(pre, 1234)
    w_, rw = o2.batch(pre, 1234)
    print("prefix", b, "same", np.array_equal(g, w_), "rng", rg == rw, "stats", dev.last_batch_stats())
    gc, gm = dev.read_requested()
    oc, om = o2.read_requested()
    for n in np.nonzero((gc != oc) | (gm != om))[0][:10]:
        print("  node", n, "gpu", gc[n], gm[n], "orc", oc[n], om[n])
    r1, f1, s1 = dev.evaluate(case.batch, b)
    r2, f2, s2 = o2.evaluate(case.batch, b)
    fit = f2 == 0
    print("  eval pod", b, "fail-diff", int((f1 != f2).sum()), "score-diff", int(((s1 != s2) & fit).sum()),
          "max", s2[fit].max() if fit.any() else None, "k", int((s2[fit] == s2[fit].max()).sum()) if fit.any() else 0)
    one = PodBatch(case.batch.pods[b:b + 1], case.batch.ids)
    print("  single pod", dev.batch(one, rg)[0], o2.batch(one, rw)[0])
