"""The drop-in algorithm.Scheduler (kubernetes_amd.scheduler.GPUScheduler) on the GPU,
pod by pod through ksg_schedule_begin/commit, against the object-level restatement
(oracle/ref_model.GenericScheduler) with the same injected random source: same hosts,
same FitError predicate maps (fit masks), same number of random draws."""
import copy

import pytest

from kubernetes_amd.api import PodStatus
from kubernetes_amd.scheduler import (FakeMinionLister, FakePodLister, FakeServiceLister, FitError, GPUScheduler,
                                      SchedulingError,
                                      SplitMix64Rand)
from oracle import ref_model as R
from tests.test_oracle_crosscheck import _workload

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,nn,npods,tight,existing", [
    ("config2", 60, 120, False, 10),
    ("config2", 20, 80, True, 0),
    ("config4", 48, 100, True, 12),
    ("policy_labels", 30, 80, False, 6),
    ("policy_many_labels", 90, 120, False, 8),  # static terms past the config's slots (ksg_add_static_config)
    ("policy_many_labels", 500, 30, True, 0),
])
def test_schedule_matches_ref_model(name, nn, npods, tight, existing):
    w = _workload(name, nn, npods, tight, existing)
    lister_ref = R.PodLister(list(w.existing))
    preds, prios = R.from_config(w.config, w.nodes, lister_ref, R.ServiceLister(w.services))
    rnd_ref = SplitMix64Rand(77)
    ref = R.GenericScheduler(preds, prios, lister_ref, rnd_ref)

    lister_gpu = FakePodLister(list(w.existing))
    rnd_gpu = SplitMix64Rand(77)
    gpu = GPUScheduler(w.config, lister_gpu, FakeServiceLister(w.services), rnd_gpu)
    minions = FakeMinionLister(w.nodes)
    try:
        for p in w.pods:
            try:
                want = ref.schedule(p, w.nodes)
            except R.FitError as e:
                with pytest.raises(FitError) as ei:
                    gpu.schedule(p, minions)
                assert set(ei.value.failed_predicates) == set(e.failed_predicates)  # same failing nodes
                continue
            except KeyError:  # ServiceAffinity's peer is on a host that is not a node
                with pytest.raises(SchedulingError):
                    gpu.schedule(p, minions)
                continue
            got = gpu.schedule(p, minions)
            assert got == want
            q = copy.copy(p)
            q.status = PodStatus(host=got)
            lister_ref.pods.append(q)  # AssumePod reported back by the lister
            lister_gpu.pods.append(q)
        assert rnd_gpu.state == rnd_ref.state
    finally:
        gpu.close()


def test_no_minions():
    from kubernetes_amd import factory
    from kubernetes_amd.api import Pod
    from kubernetes_amd.scheduler import NoMinionsError

    g = GPUScheduler(factory.create_from_provider(), FakePodLister([]))
    with pytest.raises(NoMinionsError):
        g.schedule(Pod(), FakeMinionLister([]))
    g.close()


def test_unnamed_pods_relist_keeps_device_equal_to_lister():
    """Fake listers hold unnamed pods (key "/"), as the reference's test tables do. Every
    Schedule re-lists them (MapPodsToMachines, predicates.go:354-375): the device's
    requested totals must equal the lister's pods' sums after each call, however many
    unnamed pods share a key and whatever the scheduler committed in between."""
    import numpy as np

    from kubernetes_amd import factory
    from kubernetes_amd.api import Container, ObjectMeta, Pod, PodSpec, ResourceList, ResourceRequirements, make_node
    from kubernetes_amd.resource import Quantity

    def pod(cpu, host=""):
        return Pod(metadata=ObjectMeta(),
                   spec=PodSpec(containers=[Container(resources=ResourceRequirements(ResourceList(
                       cpu=Quantity.from_milli(cpu), memory=Quantity.from_int(cpu << 20))))]),
                   status=PodStatus(host=host))

    nodes = [make_node(f"m{i}", 10000, 10 << 30) for i in range(4)]
    lister = FakePodLister([pod(100, "m0"), pod(200, "m0"), pod(300, "m1"), pod(400, "gone")])
    g = GPUScheduler(factory.create_from_provider(), lister, FakeServiceLister([]), SplitMix64Rand(5))
    minions = FakeMinionLister(nodes)
    try:
        for step in range(6):
            host = g.schedule(pod(50 + step), minions)
            if step % 2:  # the scheduler's commit reported back (AssumePod), unnamed too
                lister.pods.append(pod(50 + step, host))
            g._sync(nodes)  # what the next Schedule call sees
            want = np.zeros(len(nodes), np.int64)
            for p in lister.pods:
                if p.status.host in {n.metadata.name for n in nodes}:
                    want[int(p.status.host[1:])] += p.spec.containers[0].resources.limits.cpu().milli_value()
            got_c, _ = g.engine.read_requested()
            assert np.array_equal(got_c, want), (step, got_c, want)
    finally:
        g.close()


@pytest.mark.parametrize("nn,npods", [(300, 120), (600, 30)])
def test_batch_with_static_terms_matches_ref_model(nn, npods):
    """ksg_schedule_batch (window path) under a Policy with more LabelsPresence /
    LabelPreference terms than the config's slots: the static terms evaluated on the
    device in two slot passes (ksg_add_static_config) against the object-level
    restatement, pod by pod."""
    w = _workload("policy_many_labels", nn, npods, False, 0)
    lister_ref = R.PodLister([])
    preds, prios = R.from_config(w.config, w.nodes, lister_ref, R.ServiceLister(w.services))
    rnd_ref = SplitMix64Rand(91)
    ref = R.GenericScheduler(preds, prios, lister_ref, rnd_ref)
    want = []
    for p in w.pods:
        try:
            h = ref.schedule(p, w.nodes)
        except (R.FitError, KeyError):
            want.append(None)
            continue
        want.append(h)
        q = copy.copy(p)
        q.status = PodStatus(host=h)
        lister_ref.pods.append(q)
    gpu = GPUScheduler(w.config, FakePodLister([]), FakeServiceLister(w.services))
    try:
        got, state = gpu.schedule_batch(w.pods, FakeMinionLister(w.nodes), 91)
        assert got == want
        assert state == rnd_ref.state
        assert gpu.engine.batch_totals()["windows"] > 0  # (the window path ran)
    finally:
        gpu.close()
