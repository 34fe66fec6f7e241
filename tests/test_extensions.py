"""Extensions beyond the reference vintage (taints / tolerations, extended
resources, BalancedResourceAllocation): host-side semantics and the C
restatement on CPU. PARITY UNPINNED: these predicates and priorities do not
exist in smarterclayton/kubernetes v0.13; the
cases below restate the published v1.10 behaviour by hand."""
import numpy as np
import pytest

from kubernetes_amd import abi
from kubernetes_amd.engine import PodBatch
from kubernetes_amd.extensions import (NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, ExtConfig, ExtInterner, Taint,
                                       Toleration, tolerates)
from oracle.pyoracle import OracleScheduler
from tests.ext_cases import ExtCase
from tests.helpers import Case


@pytest.mark.parametrize("tol,taint,want", [
    (Toleration("k", "Equal", "v", NO_SCHEDULE), Taint("k", "v", NO_SCHEDULE), True),
    (Toleration("k", "", "v"), Taint("k", "v", NO_EXECUTE), True),            # "" operator = Equal, "" effect = all
    (Toleration("k", "Equal", "w"), Taint("k", "v", NO_SCHEDULE), False),     # value differs
    (Toleration("k", "Exists"), Taint("k", "anything", PREFER_NO_SCHEDULE), True),
    (Toleration("", "Exists"), Taint("x", "y", NO_EXECUTE), True),            # empty key + Exists: every taint
    (Toleration("k", "Exists", "", NO_SCHEDULE), Taint("k", "v", NO_EXECUTE), False),  # effect differs
    (Toleration("j", "Exists"), Taint("k", "v", NO_SCHEDULE), False),         # key differs
    (Toleration("k", "Bogus", "v"), Taint("k", "v", NO_SCHEDULE), False),     # unknown operator
])
def test_tolerates(tol, taint, want):
    assert tolerates(tol, taint) is want


def test_pod_records_split_hard_and_soft():
    cfg = ExtConfig(taints=True, w_taint_toleration=1)
    it = ExtInterner(cfg)
    ts = [Taint("a", "1", NO_SCHEDULE), Taint("b", "", PREFER_NO_SCHEDULE), Taint("c", "", NO_EXECUTE)]
    it.node_arrays([ts])
    # tolerates a (NoSchedule) only; b is soft and untolerated; c hard and untolerated
    rec, ids = it.pod_records(np.zeros(0, np.uint32), [[Toleration("a", "Equal", "1", NO_SCHEDULE)],
                                                       [Toleration("", "Exists", "", NO_SCHEDULE)],
                                                       [Toleration("b", "Exists", "", NO_SCHEDULE)]])
    hard = lambda i: sorted(ids[rec[i]["hard_off"]: rec[i]["hard_off"] + rec[i]["n_hard"]].tolist())
    soft = lambda i: sorted(ids[rec[i]["soft_off"]: rec[i]["soft_off"] + rec[i]["n_soft"]].tolist())
    assert hard(0) == [2] and soft(0) == [1]
    assert hard(1) == [2] and soft(1) == [1]   # an empty-key NoSchedule toleration: not c (NoExecute)
    assert hard(2) == [0, 2] and soft(2) == [1]  # a NoSchedule toleration never tolerates a PreferNoSchedule taint


def _tiny(ext_cfg, node_taints, node_gpu, pod_tols, pod_gpu, cpu=(4000, 4000), mem=(8 << 30, 8 << 30)):
    case = Case("config1", 2, len(pod_tols))
    arr = case.view.arrays
    arr.nodes["cap_milli_cpu"][:] = cpu
    arr.nodes["cap_memory"][:] = mem
    it = ExtInterner(ext_cfg)
    na = it.node_arrays(node_taints, {"gpu": node_gpu})
    rec, ids = it.pod_records(case.batch.ids, pod_tols, [{"gpu": g} for g in pod_gpu])
    orc = OracleScheduler(case.cfg)
    orc.set_extensions(ext_cfg.compile(max(len(it.taints), 1)))
    orc.set_cluster(arr)
    orc.set_node_ext(*na)
    return orc, PodBatch(case.batch.pods, ids, rec)


def test_taint_filter_and_scalar_fit_codes():
    cfg = ExtConfig(taints=True, scalar_resources=("gpu",))
    orc, b = _tiny(cfg, [[Taint("d", "x", NO_SCHEDULE)], []], [0, 2], [[], [Toleration("d", "Equal", "x")]],
                   [1, 3])
    rc, fails, _ = orc.evaluate(b, 0)  # untolerated taint on node 0; node 1 has 2 GPUs for 1
    assert rc == abi.KSG_OK and fails.tolist() == [abi.FAIL_TAINTS, 0]
    rc, fails, _ = orc.evaluate(b, 1)  # tolerated; but 3 GPUs fit nowhere (0 and 2 allocatable)
    assert fails.tolist() == [abi.FAIL_SCALAR, abi.FAIL_SCALAR]


def test_balanced_allocation_and_taint_toleration_scores():
    # one pod of cpu 100..1000m / mem 128..2048Mi on two equal empty nodes; the pod's
    # request (config1 workload) fixes the fractions: score = int((1 - |fc - fm|) * 10)
    cfg = ExtConfig(taints=True, w_taint_toleration=1, w_balanced=1)
    orc, b = _tiny(cfg, [[Taint("s", "", PREFER_NO_SCHEDULE), Taint("t", "", PREFER_NO_SCHEDULE)], []], [0, 0],
                   [[]], [0])
    p = b.pods[0]
    fc, fm = p["milli_cpu"] / 4000.0, p["memory"] / float(8 << 30)
    bal = int((1.0 - abs(fc - fm)) * 10)
    lr = ((4000 - p["milli_cpu"]) * 10 // 4000 + ((8 << 30) - p["memory"]) * 10 // (8 << 30)) // 2
    rc, fails, scores = orc.evaluate(b, 0)
    # TaintToleration: counts 2 and 0, max 2 -> 10 - 10*2/2 = 0 and 10
    assert fails.tolist() == [0, 0]
    assert scores.tolist() == [lr + bal + 0, lr + bal + 10]


@pytest.mark.parametrize("kw", [dict(), dict(w_taint=0), dict(w_bal=0), dict(gpus=False), dict(taints=False)])
def test_oracle_modes_agree_with_extensions(kw):
    """The faithful restatement (per-pod regroup) and the incremental one agree
    with the extensions on, including pods already placed with GPU requests."""
    outs = []
    for faithful in (False, True):
        c = ExtCase(nn=30, npods=160, **kw)
        o = c.load(OracleScheduler(c.cfg, faithful=faithful))
        for i in range(0, 40, 2):
            o.add_pod(i % 30, c.batch, i)
        rest = PodBatch(c.batch.pods[40:], c.batch.ids, c.batch.ext[40:])
        outs.append(o.batch(rest, 5))
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    assert (outs[0][0] >= 0).sum() > 20
    if kw.get("gpus", True):  # GPUs run out: FitErrors on the extended resource
        assert (outs[0][0] == abi.KSG_OUT_NOFIT).sum() > 0


@pytest.mark.parametrize("name,nn,w_taint,w_bal", [
    ("config2", 700, 0, 0),    # filters only (the window path's extension set)
    ("config2", 700, 1, 1),    # + TaintToleration (the cross-shard max) + BalancedAllocation
    ("config1", 257, 3, 0),
    ("config5", 1500, 0, 2),
])
def test_threaded_restatement_with_extensions_matches_single_thread(name, nn, w_taint, w_bal):
    """orc_schedule_batch_mt_ext (the full-size checker for BASELINE config 5 with
    extended resources) against the single-thread incremental restatement:
    every decision, the generator state and the committed totals."""
    e = ExtCase(name, nn, 600, seed=5, w_taint=w_taint, w_bal=w_bal)
    a = e.load(OracleScheduler(e.cfg))
    b = e.load(OracleScheduler(e.cfg))
    placed = 0
    for part in (slice(0, 250), slice(250, 600)):
        sub = PodBatch(e.batch.pods[part], e.batch.ids, e.batch.ext[part])
        ga, sa = a.batch(sub, 99 + part.start)
        gb, sb = b.batch_mt(sub, 99 + part.start, 5)
        assert np.array_equal(ga, gb) and sa == sb
        placed += int((ga >= 0).sum())
    assert placed > 0
    for x, y in zip(a.read_requested(), b.read_requested()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.read_ext_used(), b.read_ext_used())
