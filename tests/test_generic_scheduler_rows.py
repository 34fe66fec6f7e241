"""TestGenericScheduler and the TestFindFit rows (pkg/scheduler/generic_scheduler_test.go:96-297)
through the HIP path, begin / commit and the batch, with the reference's own expected hosts.

The Go rows use test closures (generic_scheduler_test.go:29-79); each maps onto a
bitmask configuration of the same behaviour:
  falsePredicate            -> a LabelsPresence predicate on a label no node carries (every
                               node fails it: predicates.go:215-229)
  truePredicate             -> no predicate
  matchesPredicate          -> HostName with Spec.Host = the pod's name (pod.Name == node
                               becomes PodFitsHost, predicates.go:181-186)
  EqualPriority             -> the config's EqualPriority weight (generic_scheduler.go:180-195)
  numericPriority,          -> node-static scores through ksg_set_static_terms (they depend on
  reverseNumericPriority       the node name only): score = Atoi(name), max + min - Atoi(name)
The seed-0 row ("test 2") uses the one known bit of Go's rand.NewSource(0): its first Int()
is odd, so of the ties [machine2, machine1] (score desc, host desc) index 1 is machine1.
"""
import numpy as np
import pytest

from kubernetes_amd import abi, ingest
from kubernetes_amd.api import Node, ObjectMeta, Pod, PodSpec
from kubernetes_amd.engine import PodBatch
from kubernetes_amd.factory import PredicateDesc, PriorityDesc, SchedulerConfig
from tests.golden_util import load

G = load("scheduler_golden.json")
_NONE_LABEL = "golden-no-node-has-this-label"


def row_setup(c, predicates, prioritizers):
    """-> (SchedulerConfig, nodes, pod, static score fn(names) or None, n_priority_configs)."""
    preds = {}
    host = ""
    for p in predicates:
        if p == "false":
            preds["false"] = PredicateDesc("LabelsPresence", (_NONE_LABEL,), True)
        elif p in ("matches", "match"):
            preds[p] = PredicateDesc("HostName")
            host = c["pod_name"]
        else:
            assert p == "true", p
    prios, static = [], []
    for name, w in prioritizers:
        if name == "EqualPriority":
            prios.append(PriorityDesc("EqualPriority", int(w)))
        else:
            assert name in ("numericPriority", "reverseNumericPriority"), name
            static.append((name, int(w)))

    def static_score(names):
        num = np.array([int(n) for n in names], np.int64)
        out = np.zeros(len(names), np.int64)
        for name, w in static:
            out += w * (num if name == "numericPriority" else num.max() + num.min() - num)
        return out

    cfg = SchedulerConfig(preds, prios, [])
    nodes = [Node(metadata=ObjectMeta(name=n)) for n in c["nodes"]]
    pod = Pod(metadata=ObjectMeta(name=c["pod_name"]), spec=PodSpec(host=host))
    return cfg, nodes, pod, (static_score if static else None), len(prioritizers)


def _ingest(c, predicates, prioritizers):
    cfg, nodes, pod, static, n_conf = row_setup(c, predicates, prioritizers)
    it = ingest.Interner()
    for k in cfg.label_keys():
        it.key_id(k)
    view = ingest.ClusterView(nodes, [], it)
    kc = cfg.compile(it.key_id)
    kc.n_priority_configs = n_conf
    batch = ingest.ingest_pods(view, [pod], uids=[7])
    return kc, view, batch, static


@pytest.mark.parametrize("c", G["generic_scheduler"], ids=[c["name"] for c in G["generic_scheduler"]])
def test_row_mapping_compiles(c):
    """CPU: every row maps onto a config the ABI takes (the closures' stand-ins)."""
    kc, view, batch, static = _ingest(c, c["predicates"], c["prioritizers"])
    assert kc.n_priority_configs == len(c["prioritizers"])
    if "false" in c["predicates"]:
        assert kc.predicates & abi.PRED_LABELSPRESENCE and kc.n_presence == 1
    if "matches" in c["predicates"]:
        assert kc.predicates & abi.PRED_HOSTNAME
        assert int(batch.pods[0]["host"]) == view.names.index(c["pod_name"])
    if static is not None:
        sc = static(view.names)
        assert sc.shape == (len(c["nodes"]),)


def _device(kc, view, static):
    from kubernetes_amd.engine import DeviceScheduler
    dev = DeviceScheduler(kc, device=0)
    dev.set_cluster(view.arrays)
    if static is not None:
        dev.set_static_terms(None, static(view.names), True)
    return dev


@pytest.mark.gpu
@pytest.mark.parametrize("c", G["generic_scheduler"], ids=[c["name"] for c in G["generic_scheduler"]])
def test_generic_scheduler_rows_on_hip(c):
    """begin + commit (the caller's draw r, tie r % k) and the batch with the caller's draws
    (ksg_schedule_batch_draws) give the row's expected host for every draw, or a FitError."""
    kc, view, batch, static = _ingest(c, c["predicates"], c["prioritizers"])
    dev = _device(kc, view, static)
    draws = list(range(6)) + [2**62 + 1, 2**63 - 1]
    for r in draws:
        rc, _, k, _ = dev.begin(batch, 0)
        if c["expects_err"]:
            assert rc == abi.KSG_NOFIT and k == 0
            continue
        assert rc == abi.KSG_OK and k >= 1
        got = view.names[dev.commit(r % k)]
        assert got in c["expected_hosts"], (r, got)
        dev.remove_pod(7)  # (AssumePod undone: every draw sees the same cluster)
        out, used = dev.batch_draws(batch, np.array([r], np.uint64))
        assert used == 1 and view.names[int(out[0])] == got
        dev.remove_pod(7)
    if c["expects_err"]:
        out, used = dev.batch_draws(batch, np.array([5], np.uint64))
        assert int(out[0]) == abi.KSG_OUT_NOFIT and used == 0  # (no draw for a FitError)
    if "go_rand_seed0_host" in c:  # Go's rand.NewSource(0): the first Int() is odd
        rc, _, k, _ = dev.begin(batch, 0)
        assert rc == abi.KSG_OK and k == 2
        assert view.names[dev.commit(1 % k)] == c["go_rand_seed0_host"]
    dev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("c", G["find_fit"], ids=[c["name"] for c in G["find_fit"]])
def test_find_fit_rows_on_hip(c):
    """findNodesThatFit's FailedPredicateMap (generic_scheduler_test.go:96-138): the fail
    codes of begin name the row's failing predicate on exactly the row's nodes."""
    kc, view, batch, static = _ingest(c, c["predicates"], [["EqualPriority", 1]])
    dev = _device(kc, view, static)
    rc, _, k, fails = dev.begin(batch, 0, want_fail=True)
    code_of = {"false": abi.FAIL_LABELSPRESENCE, "match": abi.FAIL_HOSTNAME, "matches": abi.FAIL_HOSTNAME}
    want = {n: code_of[p[0]] for n, p in c["failed"].items()}
    got = {view.names[i]: int(f) for i, f in enumerate(fails) if f != abi.FAIL_NONE}
    assert got == want
    assert (rc == abi.KSG_NOFIT) == (len(want) == len(c["nodes"]))
    dev.close()
