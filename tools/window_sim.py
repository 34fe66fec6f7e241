"""CPU model of the speculative window path: how often does a pod's sequential
decision differ from its snapshot prediction?

For each window (W pods from one snapshot) and each pod i, against the C
oracle: T0/M0 from the snapshot, the tie set/max against the sequential state.
A pod is
  * service-unclean: an earlier pod of the window raised its service's
    maxCount / gave it its first peer (the window must end: scores outside T0
    may rise);
  * a drop: clean, but its sequential tie set differs from T0 (some tie got
    worse; the choice may move);
  * predicted: neither (the result is the snapshot prediction).
Two window rules are modelled: `end-at-drop` (a window ends at the first
unclean pod or drop) and `fixup` (drops are repaired inside the window; only
unclean pods and exhausted tie sets end it).

  python tools/window_sim.py config2 5000 10000 128
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kubernetes_amd import workload  # noqa: E402
from kubernetes_amd.engine import PodBatch  # noqa: E402
from oracle.pyoracle import OracleScheduler  # noqa: E402
from tests.helpers import Case  # noqa: E402


def tie_set(rc, f, s):
    fit = f == 0
    if rc != 0 or not fit.any():
        return None, None
    m = s[fit].max()
    return m, np.nonzero(fit & (s == m))[0]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "config2"
    nn = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    npods = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    W = int(sys.argv[4]) if len(sys.argv) > 4 else 128
    rule = sys.argv[5] if len(sys.argv) > 5 else "fixup"
    case = Case(name, nn, npods)
    b = case.batch
    spread = case.cfg.w_service_spreading != 0
    aff = case.cfg.n_aff_labels > 0
    S = OracleScheduler(case.cfg)
    Cc = OracleScheduler(case.cfg)
    S.set_cluster(case.view.arrays)
    Cc.set_cluster(case.view.arrays)
    cnt = {}
    smax = {}
    peer = set()
    rng = workload.TIEBREAK_SEED
    pos = 0
    windows = []  # (pods, drops, reason)
    pred_hits = 0
    k0s = []
    dcount = []
    while pos < npods:
        snap_max = dict(smax)
        snap_peer = set(peer)
        placed = []
        drops = 0
        reason = "full"
        i = pos
        while i < min(pos + W, npods):
            p = b.pods[i]
            s = int(p["service"])
            unclean = s >= 0 and ((spread and smax.get(s, 0) != snap_max.get(s, 0)) or
                                  (aff and (s in peer) != (s in snap_peer)))
            rc0, f0, s0 = S.evaluate(b, i)
            rc1, f1, s1 = Cc.evaluate(b, i)
            m0, t0 = tie_set(rc0, f0, s0)
            m1, t1 = tie_set(rc1, f1, s1)
            drop = t0 is not None and not unclean and (m1 != m0 or not np.array_equal(t0, t1))
            if unclean:
                reason = "service"
                break
            if drop and rule == "end-at-drop" and i > pos:
                reason = "drop"
                break
            if drop and (m1 != m0):
                reason = "exhausted"
                if i > pos:
                    break
            if t0 is not None:
                k0s.append(len(t0))
            drops += bool(drop)
            if t0 is not None and not unclean and m1 == m0:
                dcount.append(len(t0) - len(t1))
            pred_hits += not drop
            o, rng = Cc.batch(PodBatch(b.pods[i:i + 1], b.ids), rng)
            node = int(o[0])
            placed.append((i, node))
            if node >= 0:
                svcs = b.ids[p["svcs_off"]:p["svcs_off"] + p["n_svcs"]]
                for sv in svcs:
                    sv = int(sv)
                    c = cnt.get((sv, node), 0) + 1
                    cnt[(sv, node)] = c
                    smax[sv] = max(smax.get(sv, 0), c)
                    peer.add(sv)
            i += 1
        for (j, node) in placed:
            if node >= 0:
                S.add_pod(node, b, j)
        windows.append((len(placed), drops, reason))
        pos += len(placed)
    ppw = np.array([w[0] for w in windows])
    dr = np.array([w[1] for w in windows])
    reasons = {}
    for w in windows:
        reasons[w[2]] = reasons.get(w[2], 0) + 1
    print(f"{name} N={nn} pods={npods} W={W} rule={rule}: windows {len(windows)}, pods/window {ppw.mean():.1f}, "
          f"drops {dr.sum()} ({dr.sum() / npods:.3f}/pod, {dr.mean():.2f}/window), reasons {reasons}, "
          f"k0 median {np.median(k0s):.0f} p10 {np.percentile(k0s, 10):.0f}")
    dc = np.array(dcount)
    print("drops per pod: " + " ".join(f"{q}:{(dc == q).mean():.3f}" for q in range(8)) + f" >=8:{(dc >= 8).mean():.3f} mean {dc.mean():.2f}")


if __name__ == "__main__":
    main()
