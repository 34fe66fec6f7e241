"""ctypes binding of oracle/_build/liboracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker. Same method surface as
kubernetes_amd.engine.DeviceScheduler so a test can run both on one input.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from kubernetes_amd import abi
from kubernetes_amd.engine import ClusterArrays, PodBatch

HERE = os.path.dirname(os.path.abspath(__file__))
# KSG_ORACLE_LIB: a sanitizer build of the same restatement (tests/test_sanitizers.py)
LIB = os.environ.get("KSG_ORACLE_LIB") or os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    vp = C.c_void_p
    P = C.POINTER
    sigs = {
        "orc_create": (vp, [P(abi.KsgConfig), C.c_int]),
        "orc_destroy": (None, [vp]),
        "orc_set_cluster": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint32, vp, C.c_uint32, C.c_uint32]),
        "orc_add_pod": (C.c_int, [vp, C.c_uint32, vp, vp]),
        "orc_remove_pod": (C.c_int, [vp, C.c_uint64]),
        "orc_evaluate": (C.c_int, [vp, vp, vp, vp, vp]),
        "orc_domain_counts": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, vp]),
        "orc_evaluate_counts": (C.c_int, [vp, vp, vp, vp, vp, vp]),
        "orc_taint_max": (C.c_int, [vp, vp, vp, vp, C.c_uint32, C.c_uint32, P(C.c_int32)]),
        "orc_evaluate_ext_tmax": (C.c_int, [vp, vp, vp, vp, C.c_int32, vp, vp]),
        "orc_schedule_begin": (C.c_int, [vp, vp, vp, C.c_size_t, P(C.c_int64), P(C.c_uint32), vp]),
        "orc_schedule_commit": (C.c_int, [vp, C.c_uint32, P(C.c_int32)]),
        "orc_schedule_batch": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint32, P(C.c_uint64), vp]),
        "orc_read_requested": (None, [vp, vp, vp]),
        "orc_read_ext_used": (None, [vp, vp]),
        "orc_admit_pods": (None, [vp, C.c_uint32, vp, C.c_uint32, vp, vp, C.c_int, vp]),
        "orc_schedule_batch_mt": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint32, P(C.c_uint64), vp, C.c_int]),
        "orc_schedule_batch_mt_ext": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.c_uint32, P(C.c_uint64), vp, C.c_int]),
        "orc_set_extensions": (None, [vp, P(abi.KsgExtConfig)]),
        "orc_set_node_ext": (None, [vp, vp, vp, vp, vp]),
        "orc_add_pod_ext": (C.c_int, [vp, C.c_uint32, vp, vp, vp]),
        "orc_schedule_batch_ext": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.c_uint32, P(C.c_uint64), vp]),
        "orc_schedule_begin_ext": (C.c_int, [vp, vp, vp, vp, C.c_size_t, P(C.c_int64), P(C.c_uint32), vp]),
        "orc_evaluate_ext": (C.c_int, [vp, vp, vp, vp, vp, vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a if len(a) else np.zeros(1, np.uint32)


class OracleScheduler:
    """CPU restatement; faithful=True reproduces the reference's cost structure."""

    def __init__(self, cfg: abi.KsgConfig, faithful: bool = False):
        self._lib = load()
        self.cfg = cfg
        self._o = C.c_void_p(self._lib.orc_create(C.byref(cfg), 1 if faithful else 0))
        self.n_nodes = 0
        self.n_scalar = 0

    def close(self):
        if self._o:
            self._lib.orc_destroy(self._o)
            self._o = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_cluster(self, cl: ClusterArrays):
        nodes = np.ascontiguousarray(cl.nodes, dtype=abi.NODE_DTYPE)
        np_ = _u32(cl.node_pairs)
        pk = _u32(cl.pair_keys)
        self._lib.orc_set_cluster(self._o, abi.ptr(nodes), len(nodes), abi.ptr(np_), len(cl.node_pairs),
                                  abi.ptr(pk), len(pk), int(cl.n_services))
        self.n_nodes = len(nodes)

    def set_extensions(self, ext: abi.KsgExtConfig):
        self._lib.orc_set_extensions(self._o, C.byref(ext))
        self.n_scalar = int(ext.n_scalar)

    def read_ext_used(self):
        u = np.zeros(max(self.n_scalar * self.n_nodes, 1), np.int64)
        self._lib.orc_read_ext_used(self._o, abi.ptr(u))
        return u[: self.n_scalar * self.n_nodes].reshape(self.n_scalar, self.n_nodes)

    def set_node_ext(self, scalar_cap, taint_off, taint_n, taint_ids):
        cap = np.ascontiguousarray(scalar_cap, np.int64).reshape(-1)
        cap = cap if len(cap) else np.zeros(1, np.int64)
        toff, tn, ti = _u32(taint_off), _u32(taint_n), _u32(taint_ids)  # (held across the call)
        self._lib.orc_set_node_ext(self._o, abi.ptr(cap), abi.ptr(toff), abi.ptr(tn), abi.ptr(ti))

    def _ext(self, batch: PodBatch, i: int):
        return None if batch.ext is None else np.ascontiguousarray(batch.ext[i : i + 1], dtype=abi.POD_EXT_DTYPE)

    def add_pod(self, host_id: int, batch: PodBatch, i: int = 0):
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        e, ids = self._ext(batch, i), _u32(batch.ids)  # (held: the pointers must outlive the call)
        self._lib.orc_add_pod_ext(self._o, int(host_id), abi.ptr(pod), abi.ptr(e), abi.ptr(ids))

    def remove_pod(self, uid: int):
        rc = self._lib.orc_remove_pod(self._o, int(uid))
        if rc != 0:
            raise KeyError(uid)

    def begin(self, batch: PodBatch, i: int = 0, want_fail: bool = False):
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        ids = _u32(batch.ids)
        m = C.c_int64(0)
        k = C.c_uint32(0)
        fails = np.zeros(max(self.n_nodes, 1), np.uint8) if want_fail else None
        rc = self._lib.orc_schedule_begin_ext(self._o, abi.ptr(pod), abi.ptr(self._ext(batch, i)), abi.ptr(ids),
                                              len(batch.ids), C.byref(m), C.byref(k), abi.ptr(fails))
        if rc not in (abi.KSG_OK, abi.KSG_NOFIT, abi.KSG_NONODES):
            raise RuntimeError(f"oracle begin rc={rc}")
        return rc, m.value, k.value, (fails[: self.n_nodes] if fails is not None else None)

    def commit(self, tie_index: int) -> int:
        out = C.c_int32(-1)
        rc = self._lib.orc_schedule_commit(self._o, int(tie_index), C.byref(out))
        if rc != 0:
            raise RuntimeError(f"oracle commit rc={rc}")
        return out.value

    def batch(self, batch: PodBatch, rng_state: int):
        n = len(batch)
        pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
        out = np.empty(max(n, 1), np.int32)
        st = C.c_uint64(rng_state)
        ext = None if batch.ext is None else np.ascontiguousarray(batch.ext, dtype=abi.POD_EXT_DTYPE)
        self._lib.orc_schedule_batch_ext(self._o, abi.ptr(pods), abi.ptr(ext), n, abi.ptr(_u32(batch.ids)),
                                         len(batch.ids), C.byref(st), abi.ptr(out))
        return out[:n], st.value

    def batch_mt(self, batch: PodBatch, rng_state: int, nthreads: int):
        """Incremental mode with each pod's node loop split over `nthreads` threads
        (node-rank shards); same decisions as batch(), extension records included."""
        n = len(batch)
        pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
        out = np.empty(max(n, 1), np.int32)
        st = C.c_uint64(rng_state)
        ext = None if batch.ext is None else np.ascontiguousarray(batch.ext, dtype=abi.POD_EXT_DTYPE)
        self._lib.orc_schedule_batch_mt_ext(self._o, abi.ptr(pods), abi.ptr(ext), n, abi.ptr(_u32(batch.ids)),
                                            len(batch.ids), C.byref(st), abi.ptr(out), int(nthreads))
        return out[:n], st.value

    def evaluate(self, batch: PodBatch, i: int = 0):
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        fails = np.zeros(max(self.n_nodes, 1), np.uint8)
        scores = np.zeros(max(self.n_nodes, 1), np.int64)
        rc = self._lib.orc_evaluate_ext(self._o, abi.ptr(pod), abi.ptr(self._ext(batch, i)),
                                        abi.ptr(_u32(batch.ids)), abi.ptr(fails), abi.ptr(scores))
        return rc, fails[: self.n_nodes], scores[: self.n_nodes]

    def domain_counts(self, batch: PodBatch, i: int, lo: int, hi: int, n_anti: int, n_pairs: int):
        """ServiceAntiAffinity partial domain counts of pod i over the filtered
        nodes of shard [lo, hi) (orc_domain_counts): int32[n_anti, n_pairs]."""
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        out = np.zeros((max(n_anti, 1), max(n_pairs, 1)), np.int32)
        rc = self._lib.orc_domain_counts(self._o, abi.ptr(pod), abi.ptr(_u32(batch.ids)), lo, hi, abi.ptr(out))
        return rc, out

    def evaluate_counts(self, batch: PodBatch, i: int, dcount: np.ndarray):
        """evaluate() scoring ServiceAntiAffinity with the supplied domain counts."""
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        fails = np.zeros(max(self.n_nodes, 1), np.uint8)
        scores = np.zeros(max(self.n_nodes, 1), np.int64)
        dc = np.ascontiguousarray(dcount, np.int32)
        rc = self._lib.orc_evaluate_counts(self._o, abi.ptr(pod), abi.ptr(_u32(batch.ids)), abi.ptr(dc),
                                           abi.ptr(fails), abi.ptr(scores))
        return rc, fails[: self.n_nodes], scores[: self.n_nodes]

    def taint_max(self, batch: PodBatch, i: int, lo: int, hi: int) -> int:
        """TaintTolerationPriority's max soft-taint count over the filtered nodes of
        shard [lo, hi) (orc_taint_max; the sharded step's partial)."""
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        out = C.c_int32(0)
        e, ids = self._ext(batch, i), _u32(batch.ids)  # (held: the pointers must outlive the call)
        rc = self._lib.orc_taint_max(self._o, abi.ptr(pod), abi.ptr(e), abi.ptr(ids), lo, hi, C.byref(out))
        assert rc == abi.KSG_OK or rc == abi.KSG_ERR_NOPEER, rc
        return int(out.value)

    def evaluate_tmax(self, batch: PodBatch, i: int, tmax: int):
        """evaluate() with TaintTolerationPriority's max supplied (the all-reduced one)."""
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        fails = np.zeros(max(self.n_nodes, 1), np.uint8)
        scores = np.zeros(max(self.n_nodes, 1), np.int64)
        e, ids = self._ext(batch, i), _u32(batch.ids)  # (held: the pointers must outlive the call)
        rc = self._lib.orc_evaluate_ext_tmax(self._o, abi.ptr(pod), abi.ptr(e), abi.ptr(ids), int(tmax), abi.ptr(fails),
                                             abi.ptr(scores))
        return rc, fails[: self.n_nodes], scores[: self.n_nodes]

    def shard(self):
        return 0, self.n_nodes

    def read_requested(self):
        c = np.zeros(max(self.n_nodes, 1), np.int64)
        m = np.zeros(max(self.n_nodes, 1), np.int64)
        self._lib.orc_read_requested(self._o, abi.ptr(c), abi.ptr(m))
        return c[: self.n_nodes], m[: self.n_nodes]


def admit_pods(sets, batch: PodBatch, pairs, mode: int = 3):
    """C restatement of the kubelet's admission checks (orc_admit_pods):
    mode 1 capacity, 2 nodeSelector, 3 both in the kubelet's order -> codes."""
    lib = load()
    sets = np.ascontiguousarray(sets, dtype=abi.ADMISSION_SET_DTYPE)
    pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
    out = np.zeros(max(len(pods), 1), np.uint8)
    lib.orc_admit_pods(abi.ptr(sets), len(sets), abi.ptr(pods), len(pods), abi.ptr(_u32(batch.ids)),
                       abi.ptr(_u32(pairs)), int(mode), abi.ptr(out))
    return out[: len(pods)]
