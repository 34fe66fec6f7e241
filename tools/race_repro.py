"""Repeat one input family through the window path many times in one process and
report every run that differs from the C oracle (run on the GPU box).

usage: python tools/race_repro.py <family> <window> <reps> [nn] [npods]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.engine import DeviceScheduler  # noqa: E402
from oracle.pyoracle import OracleScheduler  # noqa: E402
from tests.families import FamilyCase  # noqa: E402


def main():
    fam, window, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    nn = int(sys.argv[4]) if len(sys.argv) > 4 else 700
    npods = int(sys.argv[5]) if len(sys.argv) > 5 else 500
    case = FamilyCase(fam, nn, npods)
    orc = case.load(OracleScheduler(case.cfg))
    want, _ = orc.batch(case.batch, 777)
    bad_runs = 0
    t0 = time.time()
    for r in range(reps):
        dev = case.load(DeviceScheduler(case.cfg, device=0))
        dev.set_window(window)
        got, _ = dev.batch(case.batch, 777)
        bad = np.nonzero(got != want)[0]
        if bad.size:
            bad_runs += 1
            print(f"rep {r}: {bad.size} mismatches, first at {bad[:4]}: got {got[bad[:4]]} want {want[bad[:4]]}",
                  flush=True)
        dev.close()
    print(f"{fam} window {window} KSG_DEBUG={os.environ.get('KSG_DEBUG', '')} lib={os.environ.get('KSG_LIB', '')}:"
          f" {bad_runs}/{reps} runs differ ({time.time() - t0:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
