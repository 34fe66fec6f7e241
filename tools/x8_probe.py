"""Timing-switch probe: config 2, 5,000 nodes x 3,000 pods under
KSG_DEBUG bit 27 (the committer does not wait for the verdicts) and bits 27 + 24 (the x-checker
also posts at once) -- decisions wrong by design; the run must end, with placements or with the
resolver's consistency halt (KSG_HALT_BAD), never a hang. usage: python tools/x8_probe.py"""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from tests.helpers import Case
from kubernetes_amd.engine import DeviceScheduler, PodBatch
import numpy as np
for bits in [(1 << 27), (1 << 27) | (1 << 24)]:
    os.environ["KSG_DEBUG"] = str(8 | bits)
    c = Case("config2", 5000, 3000)
    d = DeviceScheduler(c.cfg, device=0)
    d.set_cluster(c.view.arrays)
    try:
        o, r = d.batch(c.batch, 77)
        print(bits, "ok", int((o >= 0).sum()))
    except Exception as e:
        print(bits, "err", str(e)[:200])
    d.close()
