"""Run every fuzz case of tests/test_gpu_fuzz.py many times at windows 5, 37 and
128 and report each run that differs from the oracle (run on the GPU box).

usage: python tools/race_hunt.py <reps> [first_seed] [last_seed]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.engine import DeviceScheduler  # noqa: E402
from oracle.pyoracle import OracleScheduler  # noqa: E402
from tests.test_gpu_fuzz import _case  # noqa: E402

reps = int(sys.argv[1])
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else 63
t0 = time.time()
total = bad_runs = 0
for seed in range(lo, hi + 1):
    cfg, arrays, batch, desc = _case(seed)
    orc = OracleScheduler(cfg)
    orc.set_cluster(arrays)
    want, _ = orc.batch(batch, 4242 + seed)
    for window in (5, 37, 128):
        dev = DeviceScheduler(cfg, device=0)
        dev.set_window(window)
        for r in range(reps):
            dev.set_cluster(arrays)
            got, _ = dev.batch(batch, 4242 + seed)
            total += 1
            bad = np.nonzero(got != want)[0]
            if bad.size:
                bad_runs += 1
                print(f"seed {seed} {desc} window {window} rep {r}: {bad.size} mismatches from {bad[:4]}", flush=True)
        dev.close()
    print(f"seed {seed} done ({time.time() - t0:.0f}s)", flush=True)
print(f"{bad_runs}/{total} runs differ", flush=True)
