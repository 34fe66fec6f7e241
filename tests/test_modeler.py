"""SimpleModeler + the event-driven device mirror (kubernetes_amd.modeler).

* TestModeler's table (plugin/pkg/scheduler/modeler_test.go:52-75, tests/golden/modeler_golden.json).
* cache.Store event semantics.
* PodMirror bookkeeping fuzz: after every sync() the pods on the (recording) sink are
  exactly SimpleModeler.list_pods(), through adds / updates / deletes / Replace of the
  scheduled store, assumed pods pruned by the queue or the scheduled store, our own
  commits adopted by AssumePod or dropped after a rejected Bind, and reloads.
* A scheduleOne loop (scheduler.go:90-122: Schedule -> Bind (sometimes rejected) ->
  AssumePod, with lagging reflector events) in lockstep against the object-level
  restatement re-listing the same modeler on every pod: on CPU with the C oracle
  behind the mirror, on the GPU (-m gpu) through GPUScheduler.
"""
import copy
import json
import os
import random

import pytest

from kubernetes_amd.api import ObjectMeta, Pod, PodStatus
from kubernetes_amd.modeler import (ADD, DELETE, UPDATE, FakeModeler, ModelerPodLister, PodMirror, SimpleModeler,
                                    Store, StoreToPodLister, meta_namespace_key)
from kubernetes_amd.scheduler import SplitMix64Rand
from oracle import ref_model as R
from tests.test_oracle_crosscheck import _workload

HERE = os.path.dirname(os.path.abspath(__file__))


def _nn_pods(ids):
    return [Pod(metadata=ObjectMeta(namespace=ns, name=n)) for ns, n in ids]


def test_modeler_golden():
    with open(os.path.join(HERE, "golden", "modeler_golden.json")) as f:
        g = json.load(f)
    assert len(g["cases"]) == 3
    for c in g["cases"]:
        q, s = StoreToPodLister(), StoreToPodLister()
        for p in _nn_pods(c["queued"]):
            q.store.add(p)
        for p in _nn_pods(c["scheduled"]):
            s.store.add(p)
        m = SimpleModeler(q, s)
        for p in _nn_pods(c["assumed"]):
            m.assume_pod(p)
        got = sorted((p.namespace, p.name) for p in m.pod_lister().list())
        assert got == sorted(tuple(x) for x in c["expect"])


def test_store_events_and_keys():
    ev = []
    st = Store()
    st.add_listener(lambda op, k, old, new: ev.append((op, k)))
    a = Pod(metadata=ObjectMeta(namespace="ns", name="a"))
    b = Pod(metadata=ObjectMeta(name="b"))
    st.add(a)
    st.add(copy.deepcopy(a))
    st.add(b)
    st.delete(Pod(metadata=ObjectMeta(name="zz")))  # absent: no event
    st.replace([b, Pod(metadata=ObjectMeta(namespace="x", name="c"))])
    assert ev == [(ADD, "ns/a"), (UPDATE, "ns/a"), (ADD, "b"), (DELETE, "ns/a"), (UPDATE, "b"), (ADD, "x/c")]
    assert meta_namespace_key(b) == "b" and st.get(b)[1] and not st.get(a)[1]
    assert sorted(st.list_keys()) == ["b", "x/c"]
    seen = []
    FakeModeler(seen.append).assume_pod(a)
    FakeModeler().assume_pod(a)
    assert seen == [a]


class _RecordingSink:
    def __init__(self):
        self.live = {}

    def add_pod(self, host_id, batch, i=0):
        uid, pod = batch
        assert uid not in self.live
        self.live[uid] = (host_id, pod)

    def remove_pod(self, uid):
        del self.live[uid]


def _pod(rng, name, host=""):
    return Pod(metadata=ObjectMeta(namespace=rng.choice(["", "default", "other"]), name=name,
                                   labels={"app": rng.choice("abc")}), status=PodStatus(host=host))


def _mirror_state(sink):
    return sorted((meta_namespace_key(p), h, id(p)) for h, p in sink.live.values())


def _modeler_state(m, hosts):
    return sorted((meta_namespace_key(p), hosts(p), id(p)) for p in m.list_pods())


@pytest.mark.parametrize("seed", range(12))
def test_mirror_bookkeeping_fuzz(seed):
    rng = random.Random(seed)
    q, s = StoreToPodLister(), StoreToPodLister()
    m = SimpleModeler(q, s)
    sink = _RecordingSink()
    hosts = lambda p: hash(p.status.host) & 0xFFFF  # noqa: E731
    uids = iter(range(1, 10 ** 9))
    mir = PodMirror(m, sink, lambda p, uid: (hosts(p), (uid, p)), lambda: next(uids))
    names = [f"p{i}" for i in range(25)]
    for step in range(400):
        r = rng.random()
        name = rng.choice(names)
        if r < 0.25:
            s.store.add(_pod(rng, name, f"h{rng.randrange(5)}"))
        elif r < 0.35 and len(s.store):
            s.store.delete(rng.choice(s.store.list()))
        elif r < 0.45:
            q.store.add(_pod(rng, name))
        elif r < 0.52 and len(q.store):
            q.store.delete(rng.choice(q.store.list()))
        elif r < 0.80:  # our own commit; AssumePod follows unless the Bind is rejected
            p = _pod(rng, name, f"h{rng.randrange(5)}")
            mir.committed(p, next(uids), hosts(p))
            sink.live[mir.pending[meta_namespace_key(p)][0]] = (hosts(p), p)
            if rng.random() < 0.8:
                m.assume_pod(p if rng.random() < 0.9 else _pod(rng, name, "elsewhere"))
        elif r < 0.85:
            m.assume_pod(_pod(rng, name, f"h{rng.randrange(5)}"))
        elif r < 0.88:
            s.store.replace([_pod(rng, n, f"h{rng.randrange(5)}") for n in rng.sample(names, 6)])
        elif r < 0.90:
            sink.live.clear()  # cluster re-uploaded
            mir.reload()
        if rng.random() < 0.5:
            mir.sync()
            assert _mirror_state(sink) == _modeler_state(m, hosts), step
    mir.sync()
    assert _mirror_state(sink) == _modeler_state(m, hosts)
    assert mir.stats["adopted"] > 0 and mir.stats["dropped_commits"] > 0


# ---- scheduleOne loop against the re-listing restatement ---------------------------
class _OracleMirrorScheduler:
    """CPU stand-in for GPUScheduler's modeler path in this test: the same ingest and
    PodMirror, the C oracle as the sink (test infrastructure checking the mirror)."""

    def __init__(self, config, modeler, services, rnd):
        from kubernetes_amd.ingest import ClusterView, Interner, PodBatchBuilder
        from oracle.pyoracle import OracleScheduler

        self._CV, self._PBB = ClusterView, PodBatchBuilder
        self.config, self.services, self.random = config, services, rnd
        self.it = Interner()
        for k in config.label_keys():
            self.it.key_id(k)
        self.orc = OracleScheduler(config.compile(self.it.key_id))
        self.fail_names = config.fail_code_names()
        self.uid = 0
        self.nodes_sig = None
        self.mir = PodMirror(modeler, self.orc, self._ingest, self._new_uid)

    def _new_uid(self):
        self.uid += 1
        return self.uid

    def _ingest(self, pod, uid):
        b = self._PBB(self.view, self.config.affinity_labels())
        b.add(pod, uid)
        return self.view.host_id(pod.status.host), b.build()

    def schedule(self, pod, nodes):
        from kubernetes_amd.scheduler import FitError

        if tuple(id(n) for n in nodes) != self.nodes_sig:
            self.view = self._CV(nodes, self.services, self.it)
            self.orc.set_cluster(self.view.arrays)
            self.nodes_sig = tuple(id(n) for n in nodes)
            self.mir.reload()
        else:
            self.mir.sync()
        uid = self._new_uid()
        _, batch = self._ingest(pod, uid)
        rc, _, k, fails = self.orc.begin(batch, 0, want_fail=True)
        if rc != 0:
            raise FitError(pod, {self.view.names[n]: {self.fail_names[int(c)]} for n, c in enumerate(fails) if c})
        node = self.orc.commit(self.random.int() % k)
        self.mir.committed(pod, uid, node)
        return self.view.names[node]


def _schedule_loop(w, make_sched, seed, n_events=3):
    """scheduleOne over w.pods with a shared SimpleModeler; returns the decisions."""
    from kubernetes_amd.scheduler import FitError, SchedulingError

    rng = random.Random(seed)
    q, s = StoreToPodLister(), StoreToPodLister()
    for p in w.existing:
        s.store.add(p)
    m = SimpleModeler(q, s)
    queue = list(w.pods)
    for p in queue:
        q.store.add(p)
    nodes = list(w.nodes)
    rnd_ref, rnd_dev = SplitMix64Rand(seed), SplitMix64Rand(seed)
    dev = make_sched(m, w, rnd_dev)

    def new_ref():
        lister = m.pod_lister()  # re-lists on every call, as the reference does
        preds, prios = R.from_config(w.config, nodes, lister, R.ServiceLister(w.services))
        return R.GenericScheduler(preds, prios, lister, rnd_ref)

    ref = new_ref()
    in_flight = []  # assumed pods the scheduled-pod reflector has not delivered yet
    out = []
    steps = 0
    while queue and steps < 3 * len(w.pods):
        steps += 1
        pod = queue.pop(0)
        q.store.delete(pod)  # NextPod: Pop from the FIFO
        try:
            want = ref.schedule(pod, nodes)
        except R.FitError as e:
            with pytest.raises(FitError) as ei:
                dev.schedule(pod, nodes)
            assert set(ei.value.failed_predicates) == set(e.failed_predicates)
            out.append(None)
            continue
        except KeyError:
            with pytest.raises(SchedulingError):
                dev.schedule(pod, nodes)
            out.append("error")
            continue
        got = dev.schedule(pod, nodes)
        assert got == want, (steps, pod.metadata.name)
        out.append(got)
        if rng.random() < 0.12:  # Bind rejected: Error func requeues the pod
            if rng.random() < 0.5:
                queue.append(pod)
                q.store.add(pod)
        else:
            assumed = copy.copy(pod)
            assumed.spec = copy.copy(pod.spec)
            assumed.spec.host = got
            assumed.status = PodStatus(host=got)
            m.assume_pod(assumed)
            in_flight.append(assumed)
        for _ in range(rng.randrange(n_events + 1)):  # reflector events, delivered late
            r = rng.random()
            if r < 0.6 and in_flight:
                a = in_flight.pop(rng.randrange(min(3, len(in_flight))))
                s.store.add(copy.copy(a))
            elif r < 0.75 and len(s.store):
                s.store.delete(rng.choice(s.store.list()))  # a pod finished / was deleted
            elif r < 0.85 and in_flight:  # re-created unassigned under the same name
                a = in_flight.pop()
                fresh = copy.copy(a)
                fresh.spec = copy.copy(a.spec)
                fresh.spec.host = ""
                fresh.status = PodStatus()
                queue.append(fresh)
                q.store.add(fresh)
        if steps == len(w.pods) // 2 and len(nodes) > 4:  # node poller: one node gone
            nodes = nodes[:1] + nodes[2:]
            ref = new_ref()
    assert rnd_dev.state == rnd_ref.state
    return out, dev


LOOP_CASES = [("config2", 40, 90, False, 8), ("config2", 16, 70, True, 0), ("config4", 40, 80, True, 6),
              ("policy_labels", 24, 70, False, 5)]


@pytest.mark.parametrize("name,nn,npods,tight,existing", LOOP_CASES)
def test_schedule_loop_oracle_mirror(name, nn, npods, tight, existing):
    w = _workload(name, nn, npods, tight, existing)
    out, dev = _schedule_loop(w, lambda m, w, rnd: _OracleMirrorScheduler(w.config, m, w.services, rnd), seed=11)
    assert any(o not in (None, "error") for o in out)
    assert dev.mir.stats["adopted"] > 0 and dev.mir.stats["dropped_commits"] > 0
    dev.orc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,nn,npods,tight,existing", LOOP_CASES)
def test_schedule_loop_gpu_modeler(name, nn, npods, tight, existing):
    from kubernetes_amd.scheduler import FakeServiceLister, GPUScheduler

    class _Nodes:
        def __init__(self, nodes):
            self.nodes = nodes

    w = _workload(name, nn, npods, tight, existing)
    made = []

    def make(m, w, rnd):
        g = GPUScheduler(w.config, m.pod_lister(), FakeServiceLister(w.services), rnd)
        assert isinstance(m.pod_lister(), ModelerPodLister) and g._events is not None

        class _Adapter:  # schedule(pod, nodes) -> GPUScheduler.schedule(pod, MinionLister)
            def schedule(self, pod, nodes):
                lst = _Nodes(nodes)
                lst.list = lambda: lst.nodes
                return g.schedule(pod, lst)

        made.append(g)
        return _Adapter()

    try:
        out, _ = _schedule_loop(w, make, seed=11)
        st = made[0]._events.stats
        assert any(o not in (None, "error") for o in out)
        assert st["adopted"] > 0 and st["dropped_commits"] > 0 and st["reloads"] == 2
    finally:
        for g in made:
            g.close()


def test_store_events_follow_mutation_order_across_threads():
    """Listeners run under the store lock: replaying the event stream reproduces the
    store's final state even with several writer threads on the same keys."""
    import threading

    st = Store()
    replay = {}
    st.add_listener(lambda op, k, old, new: replay.pop(k) if op == DELETE else replay.__setitem__(k, new))

    def writer(seed):
        rng = random.Random(seed)
        for _ in range(3000):
            p = Pod(metadata=ObjectMeta(name=f"p{rng.randrange(8)}"), status=PodStatus(host=str(seed)))
            (st.delete if rng.random() < 0.3 else st.add)(p)

    ts = [threading.Thread(target=writer, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert {k: id(v) for k, v in replay.items()} == {k: id(st.get_by_key(k)[0]) for k in st.list_keys()}


def test_reload_races_a_reflector_thread():
    """A reflector thread adding pods while reload() snapshots the stores: each pod is
    on the device exactly once afterwards (either in the snapshot or queued after it)."""
    import threading

    q, s = StoreToPodLister(), StoreToPodLister()
    m = SimpleModeler(q, s)
    sink = _RecordingSink()
    hosts = lambda p: hash(p.status.host) & 0xFFFF  # noqa: E731
    uids = iter(range(1, 10 ** 9))
    mir = PodMirror(m, sink, lambda p, uid: (hosts(p), (uid, p)), lambda: next(uids))
    rng = random.Random(3)
    for i in range(50):
        s.store.add(_pod(rng, f"p{i}", "h1"))
    mir.sync()
    stop = threading.Event()

    def reflector():
        j = 0
        while not stop.is_set() and j < 3000:
            s.store.add(_pod(random.Random(j), f"r{j % 400}", f"h{j % 3}"))
            j += 1

    t = threading.Thread(target=reflector)
    t.start()
    try:
        for _ in range(30):
            sink.live.clear()
            mir.reload()
            mir.sync()
    finally:
        stop.set()
        t.join()
    mir.sync()
    assert _mirror_state(sink) == _modeler_state(m, hosts)
    assert len(sink.live) == len(m.list_pods())
