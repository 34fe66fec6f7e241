"""SimpleModeler and the event-driven device mirror.

Reference:
  cache.Store (keyed, Add/Update/Delete/Get/List/Replace)       pkg/client/cache/store.go:27-250
  MetaNamespaceKeyFunc                                          pkg/client/cache/store.go:53-66
  StoreToPodLister.List / Exists                                pkg/client/cache/listers.go:37-62
  SystemModeler / FakeModeler / SimpleModeler                   plugin/pkg/scheduler/modeler.go:31-155
    AssumePod                                                   modeler.go:76-78
    listPods: drop assumed pods that now exist in the queued or
    scheduled store, then scheduled ++ assumed                  modeler.go:89-139
  scheduleOne: Schedule -> Bind -> AssumePod(Status.Host=dest)  plugin/pkg/scheduler/scheduler.go:90-122

The reference re-lists every pod on every Schedule call (MapPodsToMachines,
predicates.go:354-375, through the modeler's PodLister). On the GPU the node
state is resident in HBM, so `PodMirror` keeps it equal to
`SimpleModeler.list_pods()` from the stores' change events instead: a
scheduled-pod event is one ksg_add_pod / ksg_remove_pod, the listPods pruning
walks only the (short) assumed list, and the pod the scheduler itself just
committed on the device is adopted when AssumePod reports it (so it is not
counted twice), or removed again if it never is (a rejected Bind).
Events are queued under a lock by whatever thread feeds the stores (the
reflector goroutines' role) and applied between pods by the scheduling
thread, as SURVEY.md 8(b) "Threading" requires.
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Callable, Dict, List, Optional, Tuple

from .api import Pod
from .labels import everything

ADD, UPDATE, DELETE = "add", "update", "delete"


def meta_namespace_key(obj) -> str:
    """cache.MetaNamespaceKeyFunc (store.go:53-66): "ns/name", or "name" with no namespace."""
    m = obj.metadata
    return f"{m.namespace}/{m.name}" if m.namespace else m.name


class Store:
    """cache.Store (store.go): a keyed, thread-safe object cache. Listeners get
    (op, key, old, new) for each change, called under the store's lock so that
    the event order is the mutation order (listeners must only enqueue)."""

    def __init__(self, key_func: Callable = meta_namespace_key):
        self._lock = threading.RLock()
        self._items: Dict[str, object] = {}
        self._key = key_func
        self._listeners: List[Callable] = []

    def add_listener(self, fn: Callable) -> None:
        self._listeners.append(fn)

    def _emit(self, op, key, old, new):
        for fn in self._listeners:
            fn(op, key, old, new)

    def add(self, obj) -> None:  # store.go:79-92 (Add on an existing key replaces it)
        k = self._key(obj)
        with self._lock:
            old = self._items.get(k)
            self._items[k] = obj
            self._emit(ADD if old is None else UPDATE, k, old, obj)

    def update(self, obj) -> None:  # store.go:148-160
        self.add(obj)

    def delete(self, obj) -> None:  # store.go:162-174
        k = self._key(obj)
        with self._lock:
            old = self._items.pop(k, None)
            if old is not None:
                self._emit(DELETE, k, old, None)

    def get(self, obj) -> Tuple[Optional[object], bool]:  # store.go:212-220
        return self.get_by_key(self._key(obj))

    def get_by_key(self, key: str) -> Tuple[Optional[object], bool]:  # store.go:222-230
        with self._lock:
            it = self._items.get(key)
        return it, it is not None

    def list(self) -> list:  # store.go:176-186
        with self._lock:
            return list(self._items.values())

    def list_keys(self) -> List[str]:
        with self._lock:
            return list(self._items)

    def replace(self, objs) -> None:  # store.go:232-250
        new = {self._key(o): o for o in objs}
        with self._lock:
            old = self._items
            self._items = dict(new)
            for k, o in old.items():
                if k not in new:
                    self._emit(DELETE, k, o, None)
            for k, o in new.items():
                self._emit(ADD if k not in old else UPDATE, k, old.get(k), o)

    def __len__(self):
        with self._lock:
            return len(self._items)


class StoreToPodLister:
    """listers.go:37-62: List(selector) over the store, Exists by namespace/name."""

    def __init__(self, store: Optional[Store] = None):
        self.store = store if store is not None else Store()

    def list(self, selector=None) -> List[Pod]:
        sel = selector if selector is not None else everything()
        return [p for p in self.store.list() if sel.matches(p.metadata.labels)]

    def exists(self, pod: Pod) -> bool:
        return self.store.get(pod)[1]


class FakeModeler:
    """modeler.go:44-53."""

    def __init__(self, assume_pod_func: Optional[Callable] = None):
        self.assume_pod_func = assume_pod_func

    def assume_pod(self, pod: Pod) -> None:
        if self.assume_pod_func is not None:
            self.assume_pod_func(pod)


class SimpleModeler:
    """modeler.go:55-155: the pods the scheduler knows are scheduled, plus the ones
    it assumed it scheduled that have not shown up in either store yet."""

    def __init__(self, queued_pods: StoreToPodLister, scheduled_pods: StoreToPodLister):
        self.queued_pods = queued_pods
        self.scheduled_pods = scheduled_pods
        self.assumed_pods = StoreToPodLister(Store(meta_namespace_key))

    def assume_pod(self, pod: Pod) -> None:  # modeler.go:76-78
        self.assumed_pods.store.add(pod)

    def prune_assumed(self) -> None:
        """modeler.go:95-117: stop assuming a pod once it exists in the queue or the
        scheduled store (checked by key; every assumed pod, not only the selected)."""
        for pod in self.assumed_pods.store.list():
            if self.queued_pods.exists(pod) or self.scheduled_pods.exists(pod):
                self.assumed_pods.store.delete(pod)

    def list_pods(self, selector=None) -> List[Pod]:  # modeler.go:89-139
        self.prune_assumed()
        scheduled = self.scheduled_pods.list(selector)
        assumed = self.assumed_pods.list(selector)
        return scheduled + assumed

    def pod_lister(self) -> "ModelerPodLister":  # modeler.go:141-155
        return ModelerPodLister(self)


class ModelerPodLister:
    """simpleModelerPods (modeler.go:147-155): List = listPods. The GPU scheduler
    recognises it and mirrors the modeler's stores by events instead of re-listing."""

    def __init__(self, modeler: SimpleModeler):
        self.modeler = modeler

    def list(self, selector=None) -> List[Pod]:
        return self.modeler.list_pods(selector)


class PodMirror:
    """Keeps a device context's pod set equal to `modeler.list_pods()`.

    `sink` has the engine's add_pod(host_id, batch, i) / remove_pod(uid);
    `ingest(pod, uid)` turns one pod into (host_id, PodBatch) for the current
    ClusterView. Call `sync()` between pods, `reload()` after the cluster (nodes or
    services) was re-uploaded, and `committed(pod, uid, host_id)` right after the
    scheduler committed `pod` on the device itself.
    """

    SCHED, ASSUMED = 0, 1

    def __init__(self, modeler: SimpleModeler, sink, ingest: Callable, new_uid: Callable[[], int],
                 host_of: Optional[Callable] = None):
        self.modeler = modeler
        self.sink = sink
        self.ingest = ingest
        self.new_uid = new_uid
        # pod -> host id without a full ingest (the adoption check only needs the host)
        self.host_of = host_of if host_of is not None else (lambda p: ingest(p, 0)[0])
        self._q: deque = deque()
        self._qlock = threading.Lock()
        # (source, key) -> uid on the device
        self.on_device: Dict[Tuple[int, str], int] = {}
        self.pending: Dict[str, Tuple[int, int]] = {}  # key -> (uid, host_id) of our own commits
        modeler.scheduled_pods.store.add_listener(self._listener(self.SCHED))
        modeler.assumed_pods.store.add_listener(self._listener(self.ASSUMED))
        self.stats = {"adds": 0, "removes": 0, "adopted": 0, "dropped_commits": 0, "reloads": 0}

    def _listener(self, src: int):
        def fn(op, key, old, new):
            with self._qlock:
                self._q.append((src, op, key, new))
        return fn

    def _add(self, src: int, key: str, pod: Pod):
        self._remove(src, key)  # an ADD for a key already on the device replaces it
        uid = self.new_uid()
        host_id, batch = self.ingest(pod, uid)
        self.sink.add_pod(host_id, batch, 0)
        self.on_device[(src, key)] = uid
        self.stats["adds"] += 1

    def _remove(self, src: int, key: str):
        uid = self.on_device.pop((src, key), None)
        if uid is not None:
            self.sink.remove_pod(uid)
            self.stats["removes"] += 1

    def _drain(self):
        while True:
            with self._qlock:
                if not self._q:
                    return
                src, op, key, pod = self._q.popleft()
            if src == self.ASSUMED and op == ADD and key in self.pending:
                uid, host_id = self.pending.pop(key)
                if self.host_of(pod) == host_id:  # AssumePod of the pod we just committed there: adopt it
                    self.on_device[(src, key)] = uid
                    self.stats["adopted"] += 1
                    continue
                self.sink.remove_pod(uid)
                self.stats["dropped_commits"] += 1
            if op in (UPDATE, DELETE):
                self._remove(src, key)
            if op in (ADD, UPDATE):
                self._add(src, key, pod)

    def _drop_pending(self):
        for uid, _ in self.pending.values():
            self.sink.remove_pod(uid)
            self.stats["dropped_commits"] += 1
        self.pending.clear()

    def sync(self) -> None:
        """Apply queued store events, then listPods' pruning (whose deletes are
        events too). Afterwards the device holds exactly modeler.list_pods()."""
        self._drain()
        self._drop_pending()  # committed but never assumed (Bind rejected)
        self.modeler.prune_assumed()
        self._drain()

    def reload(self) -> None:
        """The device context was re-created from a new ClusterView (node or service
        change): discard the queue and load the modeler's current pod set.

        The queue is cleared and both stores are snapshotted while holding the stores'
        locks (their listeners enqueue under them), so an event is either already in
        the snapshot or queued after it, never both."""
        self.pending.clear()
        self.on_device.clear()
        self.modeler.prune_assumed()
        sched, assumed = self.modeler.scheduled_pods.store, self.modeler.assumed_pods.store
        with sched._lock, assumed._lock:
            with self._qlock:
                self._q.clear()
            snap = [(self.SCHED, k, sched.get_by_key(k)) for k in sched.list_keys()]
            snap += [(self.ASSUMED, k, assumed.get_by_key(k)) for k in assumed.list_keys()]
        for src, key, (p, ok) in snap:
            if ok:
                self._add(src, key, p)
        self.stats["reloads"] += 1

    def committed(self, pod: Pod, uid: int, host_id: int) -> None:
        key = meta_namespace_key(pod)
        if key in self.pending:  # scheduled again before AssumePod: the first never took effect
            self.sink.remove_pod(self.pending.pop(key)[0])
            self.stats["dropped_commits"] += 1
        self.pending[key] = (uid, host_id)
