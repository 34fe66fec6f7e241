"""Concurrent updates through the C ABI (SURVEY.md 8(b) "Threading": one scheduling
thread per context plus reflector threads feeding pod adds / deletes, applied
between pods).

* Updates that arrive while a ksg_schedule_begin is pending are queued and applied
  right after the commit (or when the begin is abandoned): the decisions and the
  committed totals equal the oracle's with the same updates applied at that point.
* Stress: a reflector thread adds and removes pods on real nodes while the main
  thread schedules (ctypes drops the GIL, so the calls really overlap); after it
  has removed every pod it added, the requested totals equal exactly the sum of
  the pods the scheduler placed.
"""
import threading

import numpy as np
import pytest

from kubernetes_amd import abi
from kubernetes_amd.engine import DeviceScheduler, PodBatch
from oracle.pyoracle import OracleScheduler
from tests.helpers import Case

pytestmark = pytest.mark.gpu


def _with_uid(batch, i, uid):
    pods = batch.pods[i:i + 1].copy()
    pods["uid"] = uid
    return PodBatch(pods, batch.ids)


def test_updates_during_pending_begin_apply_after_commit():
    case = Case("config2", 700, 400)
    dev, orc = DeviceScheduler(case.cfg), OracleScheduler(case.cfg)
    try:
        for s in (dev, orc):
            s.set_cluster(case.view.arrays)
        n = case.view.arrays.n_nodes
        extra = Case("config2", 700, 300, seed=99)  # a second pod stream for the "reflector"
        rng = np.random.default_rng(5)
        live = []
        next_uid = 10 ** 9
        for i in range(len(case.batch)):
            rg, mg, kg, _ = dev.begin(case.batch, i)
            ro, mo, ko, _ = orc.begin(case.batch, i)
            assert (rg, mg, kg) == (ro, mo, ko), i
            # reflector events while the begin is pending: queued by the library
            ops = []
            for _ in range(int(rng.integers(0, 3))):
                if live and rng.random() < 0.4:
                    uid = live.pop(int(rng.integers(0, len(live))))
                    dev.remove_pod(uid)
                    ops.append(("rm", uid))
                else:
                    j = int(rng.integers(0, len(extra.batch)))
                    b = _with_uid(extra.batch, j, next_uid)
                    host = int(rng.integers(0, n + 3))
                    dev.add_pod(host, b, 0)
                    ops.append(("add", host, b))
                    live.append(next_uid)
                    next_uid += 1
            if rg == abi.KSG_OK:
                ix = int(rng.integers(0, kg))
                if i % 7 != 3 or i == len(case.batch) - 1:  # else abandoned: the next begin applies the queue
                    assert dev.commit(ix) == orc.commit(ix), i
            for op in ops:  # the oracle applies them where the library must have
                if op[0] == "rm":
                    orc.remove_pod(op[1])
                else:
                    orc.add_pod(op[1], op[2], 0)
        uc, um = dev.read_requested()
        wc, wm = orc.read_requested()
        assert np.array_equal(uc, wc) and np.array_equal(um, wm)
    finally:
        dev.close()
        orc.close()


def test_duplicate_and_unknown_uids_rejected_while_pending():
    case = Case("config2", 200, 20)
    dev = DeviceScheduler(case.cfg)
    try:
        dev.set_cluster(case.view.arrays)
        dev.add_pod(3, case.batch, 0)
        uid0 = int(case.batch.pods[0]["uid"])
        rg, _, _, _ = dev.begin(case.batch, 1)
        assert rg == abi.KSG_OK
        with pytest.raises(Exception):
            dev.add_pod(4, case.batch, 0)  # uid0 is live
        with pytest.raises(Exception):
            dev.add_pod(4, case.batch, 1)  # the pending pod's uid
        with pytest.raises(Exception):
            dev.remove_pod(123456789)
        dev.remove_pod(uid0)
        with pytest.raises(Exception):
            dev.remove_pod(uid0)  # already queued for removal
        dev.add_pod(5, case.batch, 0)  # re-add after the queued removal: allowed
        node = dev.commit(0)
        uc, _ = dev.read_requested()
        c0, c1 = (int(case.batch.pods[j]["milli_cpu"]) for j in (0, 1))
        want = np.zeros_like(uc)
        want[5] += c0
        want[node] += c1
        assert np.array_equal(uc, want)
    finally:
        dev.close()


@pytest.mark.parametrize("mode", ["begin_commit", "batch"])
def test_reflector_thread_stress(mode):
    case = Case("config2", 1500, 3000)
    churn = Case("config2", 1500, 2000, seed=123)
    dev = DeviceScheduler(case.cfg)
    dev.set_cluster(case.view.arrays)
    n = case.view.arrays.n_nodes
    errors = []
    stop = threading.Event()

    def reflector():
        rng = np.random.default_rng(9)
        live = []
        uid = 2 * 10 ** 9
        try:
            while not stop.is_set() or live:
                if live and (stop.is_set() or rng.random() < 0.45):
                    dev.remove_pod(live.pop(int(rng.integers(0, len(live)))))
                else:
                    j = int(rng.integers(0, len(churn.batch)))
                    dev.add_pod(int(rng.integers(0, n)), _with_uid(churn.batch, j, uid), 0)
                    live.append(uid)
                    uid += 1
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    t = threading.Thread(target=reflector)
    t.start()
    placed = []
    try:
        if mode == "batch":
            rng_state = 77
            for s in range(0, len(case.batch), 250):
                sub = PodBatch(case.batch.pods[s:s + 250], case.batch.ids)
                out, rng_state = dev.batch(sub, rng_state)
                placed.append(out)
        else:
            rng = np.random.default_rng(1)
            out = np.full(len(case.batch), -1, np.int32)
            for i in range(len(case.batch)):
                rg, _, kg, _ = dev.begin(case.batch, i)
                if rg == abi.KSG_OK:
                    out[i] = dev.commit(int(rng.integers(0, kg)))
            placed.append(out)
    finally:
        stop.set()
        t.join(timeout=60)
    assert not t.is_alive() and not errors, errors
    out = np.concatenate(placed)
    assert (out >= 0).sum() > len(out) // 2
    want_c = np.zeros(n, np.int64)
    want_m = np.zeros(n, np.int64)
    ok = out >= 0
    np.add.at(want_c, out[ok], case.batch.pods["milli_cpu"][ok].astype(np.int64))
    np.add.at(want_m, out[ok], case.batch.pods["memory"][ok].astype(np.int64))
    uc, um = dev.read_requested()
    dev.close()
    assert np.array_equal(uc, want_c) and np.array_equal(um, want_m)
