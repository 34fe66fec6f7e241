"""Kubelet admission with the scheduler's predicates.

handleNotFittingPods (pkg/kubelet/kubelet.go:1745-1771) re-checks a node's own pods with
scheduler.PodMatchesNodeLabels (predicates.go:161-167) and, over the pods sorted by
creation time, scheduler.CheckPodsExceedingCapacity (predicates.go:104-124). Pinned by the
reference's TestHandleNodeSelector / TestHandleMemExceeded (kubelet_test.go:2929-3032,
tests/golden/kubelet_golden.json) through the object-level restatement (ref_model), the C
restatement (orc_admit_pods) and the HIP kernel (ksg_admit.hip, -m gpu); then many random
nodes' sets in one launch against the C restatement, bit for bit.
"""
import numpy as np
import pytest

from kubernetes_amd import abi
from kubernetes_amd.api import ObjectMeta, Pod, PodSpec, Quantity, make_node
from kubernetes_amd.kubelet import KubeletAdmission, MachineInfo, capacity_from_machine_info, pods_by_creation_time
from kubernetes_amd.api import Container, ResourceList, ResourceRequirements
from oracle import pyoracle
from oracle import ref_model as R
from tests.golden_util import load, mk_pod

G = load("kubelet_golden.json")


def _case(c):
    pods = []
    for d in c["pods"]:
        p = mk_pod(d)
        p.metadata.creation_timestamp = float(d["created"])
        pods.append(p)
    node = make_node("testnode", labels=c["node_labels"])
    cap = capacity_from_machine_info(MachineInfo(**c["machine"]))
    return node, cap, pods


def _ref_handle(node, cap, pods):
    """handleNotFittingPods' scheduler checks through the object-level restatement."""
    why = {}
    fitting = []
    for p in pods:
        if R.pod_matches_node_labels(p, node):
            fitting.append(p)
        else:
            why[p.key()] = "nodeSelectorMismatching"
    _, not_fitting = R.check_pods_exceeding_capacity(pods_by_creation_time(fitting), cap)
    for p in not_fitting:
        why[p.key()] = "capacityExceeded"
    return why


@pytest.mark.parametrize("c", G["cases"], ids=[c["test"] for c in G["cases"]])
def test_golden_ref_model(c):
    assert _ref_handle(*_case(c)) == c["rejected"]


@pytest.mark.parametrize("c", G["cases"], ids=[c["test"] for c in G["cases"]])
def test_golden_c_oracle(c):
    node, cap, pods = _case(c)
    pods = pods_by_creation_time(pods)
    ka = KubeletAdmission(build_only=True)
    arr, batch, pairs = ka.build([(node, cap, pods)])
    codes = pyoracle.admit_pods(arr, batch, pairs, 3)
    names = {abi.ADMIT_NODESELECTOR: "nodeSelectorMismatching", abi.ADMIT_CAPACITY: "capacityExceeded"}
    assert {p.key(): names[int(k)] for p, k in zip(pods, codes) if k} == c["rejected"]


@pytest.mark.gpu
@pytest.mark.parametrize("c", G["cases"], ids=[c["test"] for c in G["cases"]])
def test_golden_hip(c):
    ka = KubeletAdmission()
    try:
        node, cap, pods = _case(c)
        assert ka.handle_not_fitting_pods(pods, node, cap) == c["rejected"]
        fit, notfit = ka.check_capacity_exceeded(pods, cap)
        rf, rn = R.check_pods_exceeding_capacity(pods_by_creation_time(pods), cap)
        assert [p.key() for p in fit] == [p.key() for p in rf] and [p.key() for p in notfit] == [p.key() for p in rn]
        m, nm = ka.check_node_selector_matching(pods, node)
        assert [p.key() for p in m] == [p.key() for p in pods if R.pod_matches_node_labels(p, node)]
    finally:
        ka.close()


def _random_sets(seed, n_sets=300, max_pods=60):
    rng = np.random.default_rng(seed)
    sets = []
    for s in range(n_sets):
        labels = {"zone": f"z{rng.integers(4)}", "disk": str(rng.choice(["ssd", "hdd"]))}
        if rng.integers(10) == 0:
            labels["zone"] = "bad value!"
        node = make_node(f"n{s}", labels=labels)
        k = int(rng.integers(5))
        cap = ResourceList(cpu=Quantity.from_milli(0 if k == 0 else int(rng.integers(1, 8)) * 1000),
                           memory=Quantity.from_int(0 if k == 1 else int(rng.integers(1, 16)) << 28))
        if k == 4:  # near int64: the greedy sums wrap as Go's int64 does
            cap = ResourceList(cpu=Quantity.from_milli((1 << 62)), memory=Quantity.from_int((1 << 62)))
        pods = []
        for i in range(int(rng.integers(0, max_pods))):
            sel = None
            r = int(rng.integers(6))
            if r == 0:
                sel = {"zone": f"z{rng.integers(4)}"}
            elif r == 1:
                sel = {"disk": "ssd", "zone": f"z{rng.integers(4)}"}
            elif r == 2:
                sel = {"zone": "bad value!"}  # SelectorFromSet trap: matches everything
            cpu = int(rng.integers(0, 2500)) if k != 4 else (1 << 61) + int(rng.integers(1000))
            mem = int(rng.integers(0, 1 << 30)) if k != 4 else (1 << 61)
            pods.append(Pod(metadata=ObjectMeta(name=f"p{s}-{i}", namespace="ns", creation_timestamp=float(i)),
                            spec=PodSpec(node_selector=sel, containers=[Container(resources=ResourceRequirements(
                                ResourceList(cpu=Quantity.from_milli(cpu), memory=Quantity.from_int(mem))))])))
        sets.append((node, cap, pods))
    sets.append((make_node("empty"), ResourceList(), []))
    return sets


def test_random_sets_ref_model_vs_c_oracle():
    sets = _random_sets(1, n_sets=60, max_pods=25)
    ka = KubeletAdmission(build_only=True)
    arr, batch, pairs = ka.build(sets)
    codes = pyoracle.admit_pods(arr, batch, pairs, 3)
    at = 0
    names = {abi.ADMIT_NODESELECTOR: "nodeSelectorMismatching", abi.ADMIT_CAPACITY: "capacityExceeded"}
    for node, cap, pods in sets:
        got = {p.key(): names[int(k)] for p, k in zip(pods, codes[at:at + len(pods)]) if k}
        assert got == _ref_handle(node, cap, pods)
        at += len(pods)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [2, 3])
def test_random_sets_hip_vs_c_oracle(seed):
    sets = _random_sets(seed)
    ka = KubeletAdmission()
    try:
        arr, batch, pairs = ka.build(sets)
        for mode in (1, 2, 3):
            got = ka.engine.admit(arr, batch, pairs, mode)
            want = pyoracle.admit_pods(arr, batch, pairs, mode)
            if mode != 3:
                want = (want == abi.ADMIT_OK).astype(np.uint8)
            assert np.array_equal(got, want), mode
        assert (got == abi.ADMIT_CAPACITY).any() and (got == abi.ADMIT_NODESELECTOR).any()
    finally:
        ka.close()


@pytest.mark.gpu
def test_overlapping_admission_sets_are_refused():
    """Two admission sets sharing a pod would have two kernel lanes write its
    result: the call fails with KSG_ERR_ARG before any device work."""
    from kubernetes_amd.engine import KsgError

    sets = _random_sets(4)
    ka = KubeletAdmission()
    try:
        arr, batch, pairs = ka.build(sets)
        bad = arr.copy()
        j = next(k for k in range(1, len(bad)) if bad[k]["n_pods"] > 0)
        bad[j]["pod_off"] = bad[0]["pod_off"]  # set j now covers set 0's first pods
        bad[j]["n_pods"] = max(1, min(int(bad[j]["n_pods"]), int(bad[0]["n_pods"])))
        if int(bad[0]["n_pods"]) == 0:
            bad[0]["n_pods"] = 1
        with pytest.raises(KsgError, match="share pod"):
            ka.engine.admit(bad, batch, pairs, 3)
        got = ka.engine.admit(arr, batch, pairs, 3)  # the context is still usable
        assert np.array_equal(got, pyoracle.admit_pods(arr, batch, pairs, 3))
    finally:
        ka.close()
