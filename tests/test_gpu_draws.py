"""ksg_schedule_batch_draws: the batch path with the caller's own rand.Int() values
(generic_scheduler.go:94 draws one per pod that finds a node). The batch must place
every pod where n sequential Schedule calls with the same values would: checked
against the C oracle's begin / commit(r % k) pod by pod, on the window path
(plain resolver, the anti-affinity re-rank) and the exact kernel."""
import numpy as np
import pytest

from kubernetes_amd import abi
from kubernetes_amd.engine import DeviceScheduler
from oracle.pyoracle import OracleScheduler
from tests.helpers import Case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,nn,npods,window", [("config2", 3000, 600, None), ("config4", 900, 400, None),
                                                  ("config1", 500, 500, None), ("config2", 1200, 200, 0)])
def test_batch_with_caller_draws_matches_sequential(name, nn, npods, window):
    case = Case(name, nn, npods)
    draws = np.random.default_rng(nn).integers(0, 1 << 63, size=npods + 7, dtype=np.uint64)
    dev = DeviceScheduler(case.cfg, device=0)
    orc = OracleScheduler(case.cfg)
    try:
        if window is not None:
            dev.set_window(window)
        dev.set_cluster(case.view.arrays)
        orc.set_cluster(case.view.arrays)
        out, used = dev.batch_draws(case.batch, draws)
        k_used = 0
        for i in range(npods):
            rc, _, k, _ = orc.begin(case.batch, i, want_fail=False)
            if rc == abi.KSG_OK:
                want = orc.commit(int(draws[k_used]) % k)
                k_used += 1
                assert out[i] == want, f"pod {i}"
            else:
                assert out[i] < 0, f"pod {i}: {out[i]}"
        assert used == k_used
        gc, gm = dev.read_requested()
        wc, wm = orc.read_requested()
        assert np.array_equal(gc, wc) and np.array_equal(gm, wm)
    finally:
        dev.close()


def test_caller_draws_rejects_short_or_negative_lists():
    case = Case("config1", 200, 20)
    dev = DeviceScheduler(case.cfg, device=0)
    try:
        dev.set_cluster(case.view.arrays)
        with pytest.raises(Exception):
            dev.batch_draws(case.batch, np.zeros(5, np.uint64))  # fewer values than pods
        with pytest.raises(Exception):
            dev.batch_draws(case.batch, np.full(20, 1 << 63, np.uint64))  # not rand.Int() values
    finally:
        dev.close()
