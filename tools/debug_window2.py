import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.helpers import Case
from kubernetes_amd.engine import DeviceScheduler, PodBatch
from oracle.pyoracle import OracleScheduler
case = Case("config1", 500, 60)
sub = PodBatch(case.batch.pods[:5], case.batch.ids)
for W in (0, 1):
    dev = DeviceScheduler(case.cfg); dev.set_window(W); dev.set_cluster(case.view.arrays)
    orc = OracleScheduler(case.cfg); orc.set_cluster(case.view.arrays)
    g, _ = dev.batch(sub, 1234); o, _ = orc.batch(sub, 1234)
    gc, gm = dev.read_requested(); oc, om = orc.read_requested()
    print("W", W, "out", g, o)
    for n in np.nonzero((gc != oc) | (gm != om))[0][:10]:
        print("  node", n, "gpu", gc[n], gm[n], "orc", oc[n], om[n])
    r1, f1, s1 = dev.evaluate(case.batch, 5); r2, f2, s2 = orc.evaluate(case.batch, 5)
    print("  eval pod5 fail-diff", int((f1 != f2).sum()), "score-diff", int(((s1 != s2) & (f1 == 0)).sum()), "max", s1[f1==0].max(), s2[f2==0].max())
