"""Debug: one small window batch with KSG_DEBUG=32; print the plain resolver's
inconsistency record (run on the GPU box)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
os.environ["KSG_DEBUG"] = "32"
from kubernetes_amd.engine import DeviceScheduler  # noqa: E402
from tests.helpers import Case  # noqa: E402

case = Case(sys.argv[1] if len(sys.argv) > 1 else "config1", int(sys.argv[2]) if len(sys.argv) > 2 else 500, 200)
dev = DeviceScheduler(case.cfg, device=0)
dev.set_window(int(sys.argv[3]) if len(sys.argv) > 3 else 16)
dev.set_cluster(case.view.arrays)
try:
    out, st = dev.batch(case.batch, 1234)
    print("ok", out[:20])
except Exception as e:  # noqa: BLE001
    print("error", e)
print("record", dev.debug_counters()[:20].tolist())
dev.close()
