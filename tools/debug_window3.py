import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.helpers import Case
from kubernetes_amd.engine import DeviceScheduler, PodBatch
case = Case("config1", 500, 60)
dev = DeviceScheduler(case.cfg); dev.set_window(1024); dev.set_cluster(case.view.arrays)
out, _ = dev.batch(PodBatch(case.batch.pods[:8], case.batch.ids), 1234)
print(out)
