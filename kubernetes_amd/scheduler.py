"""The drop-in `algorithm.Scheduler` backed by the HIP Filter/Score pass.

Reference interface (pkg/scheduler):
  type Scheduler interface { Schedule(api.Pod, MinionLister) (string, error) }   scheduler.go:25-27
  NewGenericScheduler(predicates, prioritizers, pods PodLister, random)           generic_scheduler.go:197-204
  FitError{Pod, FailedPredicates}                                                  generic_scheduler.go:30-44
  MinionLister / PodLister / ServiceLister and their fakes                         listers.go:27-93

`GPUScheduler.schedule(pod, minion_lister)` keeps the reference's contract:
  * no nodes -> NoMinionsError("no minions available to schedule pods");
  * nothing fits (or the priority list is empty) -> FitError with a
    FailedPredicateMap (one failing predicate name per node);
  * otherwise exactly one `random.int()` draw and the ix-th host, ix = r % ties,
    in (score desc, name desc) order.
The pods the scheduler sees are exactly what `pod_lister.list()` returns at each
call (as MapPodsToMachines re-lists them, predicates.go:354-375). With a plain
lister the device state is reconciled against it by namespace/name before each
pod; with SimpleModeler's lister (kubernetes_amd.modeler) it is kept equal to
the modeler's stores by their change events (PodMirror), so a Schedule call costs
O(events + assumed pods) on the host instead of O(all pods).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

from . import abi
from .api import Node, Pod, Service
from .engine import DeviceScheduler, PodBatch
from .factory import SchedulerConfig
from .ingest import ClusterView, Interner, PodBatchBuilder
from .labels import everything, selector_from_set
from .modeler import ModelerPodLister, PodMirror


class FitError(Exception):
    """*FitError (generic_scheduler.go:30-44)."""

    def __init__(self, pod: Pod, failed_predicates: Dict[str, set]):
        self.pod = pod
        self.failed_predicates = failed_predicates
        out = f"failed to find fit for pod: {pod.metadata.namespace}/{pod.metadata.name}"
        for node in sorted(failed_predicates):
            out += f"Node {node}: {','.join(sorted(failed_predicates[node]))}"
        super().__init__(out)


class NoMinionsError(Exception):
    def __init__(self):
        super().__init__("no minions available to schedule pods")


class SchedulingError(Exception):
    """Non-fit errors from a predicate (e.g. ServiceAffinity's peer lookup)."""


# ---- listers (listers.go:27-93) ----------------------------------------------
class FakeMinionLister:
    def __init__(self, nodes: Sequence[Node]):
        self.nodes = list(nodes)

    def list(self) -> List[Node]:
        return list(self.nodes)


class FakePodLister:
    def __init__(self, pods: Sequence[Pod]):
        self.pods = list(pods)

    def list(self, selector=None) -> List[Pod]:
        sel = selector or everything()
        return [p for p in self.pods if sel.matches(p.metadata.labels)]


class FakeServiceLister:
    def __init__(self, services: Sequence[Service]):
        self.services = list(services)

    def list(self) -> List[Service]:
        return list(self.services)

    def get_pod_services(self, pod: Pod) -> List[Service]:
        out = [s for s in self.services
               if s.metadata.namespace == pod.metadata.namespace
               and selector_from_set(s.spec.selector).matches(pod.metadata.labels)]
        if not out:
            raise LookupError(f"Could not find service for pod {pod.metadata.name} in namespace "
                              f"{pod.metadata.namespace} with labels: {pod.metadata.labels}")
        return out


class SplitMix64Rand:
    """Injected deterministic source: Int() = splitmix64 >> 1.
    Go's `*rand.Rand` stream cannot be reproduced without the Go stdlib; the
    caller's own source can be passed instead (anything with .int())."""

    MASK = (1 << 64) - 1

    def __init__(self, seed: int = 0):
        self.state = seed & self.MASK

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & self.MASK
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.MASK
        return z ^ (z >> 31)

    def int(self) -> int:
        return self.next() >> 1


class GPUScheduler:
    """algorithm.Scheduler on the MI355X (NewGenericScheduler's drop-in)."""

    def __init__(self, config: SchedulerConfig, pod_lister, service_lister=None, random=None,
                 device: int = 0):
        self.config = config
        self.pod_lister = pod_lister
        self.service_lister = service_lister or FakeServiceLister([])
        self.random = random if random is not None else SplitMix64Rand(0)
        self.interner = Interner()
        for k in config.label_keys():
            self.interner.key_id(k)
        self.aff_labels = config.affinity_labels()
        self.engine = DeviceScheduler(config.compile(self.interner.key_id), device=device)
        self.fail_names = config.fail_code_names()
        self.view: Optional[ClusterView] = None
        self._node_sig = None
        self._svc_sig = None
        self._mirror: Dict[str, tuple] = {}  # listed pod's distinct key -> (uid, host_id, id(pod))
        self._assumed: List[tuple] = []  # (pod key, uid, host_id) committed since the last re-list
        self._next_uid = 1
        # the modeler's PodLister (factory.go: f.PodLister = modeler.PodLister()):
        # mirror its stores by events instead of re-listing every pod per Schedule
        self._events: Optional[PodMirror] = None
        if isinstance(pod_lister, ModelerPodLister):
            self._events = PodMirror(pod_lister.modeler, self.engine, self._ingest_one, self._uid,
                                     host_of=lambda p: self.view.host_id(p.status.host))

    def close(self):
        self.engine.close()

    # ---- state reconciliation ----------------------------------------------
    def _uid(self) -> int:
        u = self._next_uid
        self._next_uid += 1
        return u

    def _ingest_one(self, pod: Pod, uid: int):
        b = PodBatchBuilder(self.view, self.aff_labels)
        b.add(pod, uid)
        return self.view.host_id(pod.status.host), b.build()

    def _sync(self, nodes: Sequence[Node]):
        services = self.service_lister.list()
        # list equality: identity first per element, so an unchanged list is ~10 us at
        # 5k nodes (an equal-valued replacement object counts as unchanged)
        nsig = list(nodes)
        ssig = list(services)
        if nsig != self._node_sig or ssig != self._svc_sig or self.view is None:
            self.view = ClusterView(nodes, services, self.interner)
            self.engine.set_cluster(self.view.arrays)
            # LabelsPresence / LabelPreference past the config's slots: slot passes on the device
            for extra in self.config.static_passes(self.interner.key_id):
                self.engine.add_static_config(extra)
            self._node_sig, self._svc_sig = nsig, ssig
            self._mirror = {}
            self._assumed = []
            if self._events is not None:
                self._events.reload()
                return
        if self._events is not None:
            self._events.sync()
            return
        pods = self.pod_lister.list(everything())
        want = {}
        for p in pods:  # unnamed / duplicate keys (fake listers) stay distinct pods
            k = p.key()
            if k in want:
                j = 1
                while f"{k}#{j}" in want:
                    j += 1
                k = f"{k}#{j}"
            want[k] = p
        # pods this scheduler committed since the last call: kept iff the lister now
        # reports them (under their key, or a #j variant of it) on the same host
        assumed, self._assumed = self._assumed, []
        for akey, uid, host in assumed:
            k, j, match = akey, 0, None
            while k in want:
                if k not in self._mirror and self.view.host_id(want[k].status.host) == host:
                    match = k
                    break
                j += 1
                k = f"{akey}#{j}"
            if match is None:
                self.engine.remove_pod(uid)
            else:
                self._mirror[match] = (uid, host, id(want[match]))
        for key in [k for k, (uid, host, pid) in self._mirror.items()
                    if k not in want or id(want[k]) != pid or self.view.host_id(want[k].status.host) != host]:
            self.engine.remove_pod(self._mirror.pop(key)[0])
        add = [(k, p) for k, p in want.items() if k not in self._mirror]
        if add:
            b = PodBatchBuilder(self.view, self.aff_labels)
            uids = []
            for _, p in add:
                uid = self._uid()
                uids.append(uid)
                b.add(p, uid)
            batch = b.build()
            for i, (k, p) in enumerate(add):
                h = self.view.host_id(p.status.host)
                self.engine.add_pod(h, batch, i)
                self._mirror[k] = (uids[i], h, id(p))

    # ---- Schedule -------------------------------------------------------------
    def schedule(self, pod: Pod, minion_lister) -> str:
        nodes = minion_lister.list()
        if len(nodes) == 0:
            raise NoMinionsError()
        self._sync(nodes)
        uid = self._uid()
        b = PodBatchBuilder(self.view, self.aff_labels)
        b.add(pod, uid)
        batch = b.build()
        try:
            rc, _, k, fails = self.engine.begin(batch, 0, want_fail=True)
        except Exception as e:  # ServiceAffinity peer on an unknown node, etc.
            if getattr(e, "code", None) == abi.KSG_ERR_NOPEER:
                raise SchedulingError(str(e)) from e
            raise
        if rc == abi.KSG_NONODES:
            raise NoMinionsError()
        if rc == abi.KSG_NOFIT:
            failed = {}
            for n, code in enumerate(fails):
                if code:
                    failed[self.view.names[n]] = {self.fail_names[int(code)]}
            raise FitError(pod, failed)
        r = self.random.int()
        node = self.engine.commit(r % k)
        # the device now assumes the pod on `node` (AssumePod); the next _sync keeps it
        # iff the pod lister reports it there too.
        host = self.view.names[node]
        if self._events is not None:  # adopted when AssumePod reports it, else dropped
            self._events.committed(pod, uid, node)
        else:
            self._assumed.append((pod.key(), uid, node))
        return host

    # ---- batch path (persistent kernel) -------------------------------------
    def schedule_batch(self, pods: Sequence[Pod], minion_lister, rng_state: int):
        """Schedule pods in order without host round-trips; each success is assumed
        (committed) before the next pod. -> (hosts or None per pod, rng_state)."""
        nodes = minion_lister.list()
        if len(nodes) == 0:
            return [None] * len(pods), rng_state
        self._sync(nodes)
        b = PodBatchBuilder(self.view, self.aff_labels)
        uids = []
        for p in pods:
            uids.append(self._uid())
            b.add(p, uids[-1])
        out, rng_state = self.engine.batch(b.build(), rng_state)
        hosts = []
        for i, p in enumerate(pods):
            if out[i] >= 0:
                hosts.append(self.view.names[out[i]])
                if self._events is not None:
                    self._events.committed(p, uids[i], int(out[i]))
                else:
                    self._assumed.append((p.key(), uids[i], int(out[i])))
            else:
                hosts.append(None)
        return hosts, rng_state


def new_gpu_scheduler(config: SchedulerConfig, pod_lister, service_lister=None, random=None,
                      device: int = 0) -> GPUScheduler:
    """Counterpart of NewGenericScheduler at factory.go:149."""
    return GPUScheduler(config, pod_lister, service_lister, random, device)
