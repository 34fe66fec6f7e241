"""Thin object wrapper over one libkschedgpu.so context.

`DeviceScheduler` owns a `ksg_ctx` (device memory, HIP stream, optional RCCL
communicator) and speaks in the interned numpy arrays of kubernetes_amd.ingest.
Every method maps 1:1 onto a C-ABI entry point of include/kschedgpu.h; any
non-OK return that is not a scheduling outcome raises KsgError. There is no
host-side evaluation here — the HIP kernels are the only implementation.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

from typing import Optional

import numpy as np

from . import abi


class KsgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ksg error {code}: {msg}")
        self.code = code


@dataclass
class ClusterArrays:
    """Interned node set: rank-ordered nodes, their label pair ids, pair->key."""

    nodes: np.ndarray  # NODE_DTYPE[N]
    node_pairs: np.ndarray  # uint32
    pair_keys: np.ndarray  # uint32[n_pairs] (entry 0 unused)
    n_services: int
    names: list = field(default_factory=list)  # node names in rank order (optional)

    @property
    def n_nodes(self) -> int:
        return int(self.nodes.shape[0])


@dataclass
class PodBatch:
    """Interned pods (POD_DTYPE) with their shared id list."""

    pods: np.ndarray
    ids: np.ndarray  # uint32
    # extensions (include/kschedgpu.h ksg_pod_ext, POD_EXT_DTYPE[n]; None: none)
    ext: Optional[np.ndarray] = None

    def __len__(self):
        return int(self.pods.shape[0])

    def one(self, i: int) -> "PodBatch":
        return PodBatch(self.pods[i : i + 1].copy(), self.ids,
                        None if self.ext is None else self.ext[i : i + 1].copy())



def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


class DeviceScheduler:
    """One scheduling context on one GPU (or one shard of a node-sharded set)."""

    def __init__(self, cfg: abi.KsgConfig, device: int = 0, rank: int = 0, world: int = 1,
                 nccl_id: bytes | None = None, allgather=None):
        """world > 1: exchange over RCCL (`nccl_id` from rank 0's nccl_unique_id()),
        or over the caller's transport `allgather(send: bytes) -> bytes` (the
        rank-major concatenation of every rank's `send`; ksg_set_allgather).
        world == 1 with an `nccl_id`: the exchange path over a 1-rank RCCL
        communicator (RCCL exercised on one GPU)."""
        self._lib = abi.load_library()
        self._ctx = C.c_void_p()
        self._xfn = None
        if world == 1 and nccl_id is None:
            rc = self._lib.ksg_create(C.byref(cfg), device, C.byref(self._ctx))
        else:
            if (nccl_id is None) == (allgather is None):
                raise ValueError("a sharded context needs exactly one of nccl_id / allgather")
            idbuf = C.create_string_buffer(nccl_id, 128) if nccl_id is not None else None
            rc = self._lib.ksg_create_sharded(C.byref(cfg), device, rank, world, idbuf, C.byref(self._ctx))
        if rc != abi.KSG_OK:
            raise KsgError(rc, "ksg_create failed (see stderr)")
        self.cfg = cfg
        self.n_nodes = 0
        self.n_scalar = 0
        self.world = world
        self.rank = rank
        if world > 1 and allgather is not None:
            self._install_allgather(allgather)

    def _install_allgather(self, allgather):
        world = self.world

        def cb(_user, send, recv, nbytes):
            try:
                got = allgather(C.string_at(send, nbytes))
                if len(got) != world * nbytes:
                    return -1
                C.memmove(recv, got, world * nbytes)
                return 0
            except Exception:  # an exception must not unwind through C
                import traceback

                traceback.print_exc()
                return -1

        self._xfn = abi.ALLGATHER_FN(cb)  # kept alive with the context
        rc = self._lib.ksg_set_allgather(self._ctx, self._xfn, None)
        if rc != abi.KSG_OK:
            self._err(rc)

    @staticmethod
    def nccl_unique_id() -> bytes:
        lib = abi.load_library()
        buf = C.create_string_buffer(128)
        rc = lib.ksg_nccl_unique_id(buf)
        if rc != abi.KSG_OK:
            raise KsgError(rc, "ncclGetUniqueId failed")
        return buf.raw

    def close(self):
        if self._ctx:
            self._lib.ksg_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, rc: int):
        msg = self._lib.ksg_last_error(self._ctx)
        raise KsgError(rc, msg.decode() if msg else "")

    # ---- cluster / pod state ---------------------------------------------
    def set_cluster(self, cl: ClusterArrays):
        nodes = np.ascontiguousarray(cl.nodes, dtype=abi.NODE_DTYPE)
        np_ = _u32(cl.node_pairs if len(cl.node_pairs) else np.zeros(1, np.uint32))
        pk = _u32(cl.pair_keys if len(cl.pair_keys) else np.zeros(1, np.uint32))
        rc = self._lib.ksg_set_cluster(self._ctx, abi.ptr(nodes), len(nodes), abi.ptr(np_), len(cl.node_pairs),
                                       abi.ptr(pk), len(pk), int(cl.n_services))
        if rc != abi.KSG_OK:
            self._err(rc)
        self.n_nodes = len(nodes)

    # ---- extensions (include/kschedgpu.h; parity unpinned) ---------------------
    def set_extensions(self, ext: abi.KsgExtConfig):
        rc = self._lib.ksg_set_extensions(self._ctx, C.byref(ext))
        if rc != abi.KSG_OK:
            self._err(rc)
        self.n_scalar = int(ext.n_scalar)

    def set_node_ext(self, scalar_cap: np.ndarray, taint_off: np.ndarray, taint_n: np.ndarray,
                     taint_ids: np.ndarray):
        """scalar_cap int64[n_scalar, N]; node n's taints taint_ids[taint_off[n]:+taint_n[n]]."""
        cap = np.ascontiguousarray(scalar_cap, np.int64).reshape(-1)
        cap = cap if len(cap) else np.zeros(1, np.int64)
        ti = _u32(taint_ids if len(taint_ids) else np.zeros(1, np.uint32))
        toff, tn = _u32(taint_off), _u32(taint_n)  # (held: a converted copy must outlive the call)
        rc = self._lib.ksg_set_node_ext(self._ctx, self.n_nodes, abi.ptr(cap), abi.ptr(toff), abi.ptr(tn), abi.ptr(ti),
                                        len(taint_ids))
        if rc != abi.KSG_OK:
            self._err(rc)

    def add_pod(self, host_id: int, batch: PodBatch, i: int = 0):
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        ids = _u32(batch.ids if len(batch.ids) else np.zeros(1, np.uint32))
        if batch.ext is not None:
            ext = np.ascontiguousarray(batch.ext[i : i + 1], dtype=abi.POD_EXT_DTYPE)
            rc = self._lib.ksg_add_pod_ext(self._ctx, int(host_id), abi.ptr(pod), abi.ptr(ext), abi.ptr(ids))
        else:
            rc = self._lib.ksg_add_pod(self._ctx, int(host_id), abi.ptr(pod), abi.ptr(ids))
        if rc != abi.KSG_OK:
            self._err(rc)

    def remove_pod(self, uid: int):
        rc = self._lib.ksg_remove_pod(self._ctx, int(uid))
        if rc != abi.KSG_OK:
            self._err(rc)

    # ---- scheduling ---------------------------------------------------------
    def begin(self, batch: PodBatch, i: int = 0, want_fail: bool = False):
        """-> (rc, max_score, tie_count, fail_codes|None); rc in {OK, NOFIT, NONODES}."""
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        ids = _u32(batch.ids if len(batch.ids) else np.zeros(1, np.uint32))
        m = C.c_int64(0)
        k = C.c_uint32(0)
        lo, hi = self.shard()
        fails = np.zeros(max(hi - lo, 1), np.uint8) if want_fail else None
        if batch.ext is not None:
            ext = np.ascontiguousarray(batch.ext[i : i + 1], dtype=abi.POD_EXT_DTYPE)
            rc = self._lib.ksg_schedule_begin_ext(self._ctx, abi.ptr(pod), abi.ptr(ext), abi.ptr(ids), C.byref(m),
                                                  C.byref(k), abi.ptr(fails))
        else:
            rc = self._lib.ksg_schedule_begin(self._ctx, abi.ptr(pod), abi.ptr(ids), C.byref(m), C.byref(k),
                                              abi.ptr(fails))
        if rc not in (abi.KSG_OK, abi.KSG_NOFIT, abi.KSG_NONODES):
            self._err(rc)
        return rc, m.value, k.value, (fails[: hi - lo] if fails is not None else None)

    def commit(self, tie_index: int) -> int:
        out = C.c_int32(-1)
        rc = self._lib.ksg_schedule_commit(self._ctx, int(tie_index), C.byref(out))
        if rc != abi.KSG_OK:
            self._err(rc)
        return out.value

    def batch(self, batch: PodBatch, rng_state: int):
        """Schedule every pod of the batch in order on the device. -> (out, rng_state)."""
        n = len(batch)
        pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
        ids = _u32(batch.ids if len(batch.ids) else np.zeros(1, np.uint32))
        out = np.empty(max(n, 1), np.int32)
        st = C.c_uint64(rng_state)
        if batch.ext is not None:
            ext = np.ascontiguousarray(batch.ext, dtype=abi.POD_EXT_DTYPE)
            rc = self._lib.ksg_schedule_batch_ext(self._ctx, abi.ptr(pods), abi.ptr(ext), n, abi.ptr(ids),
                                                  len(batch.ids), C.byref(st), abi.ptr(out))
        else:
            rc = self._lib.ksg_schedule_batch(self._ctx, abi.ptr(pods), n, abi.ptr(ids), len(batch.ids),
                                              C.byref(st), abi.ptr(out))
        if rc != abi.KSG_OK:
            self._err(rc)
        return out[:n], st.value

    def batch_draws(self, batch: PodBatch, draws):
        """ksg_schedule_batch_draws: the batch with the caller's rand.Int() values
        (draws[k] for the k-th pod that finds a node). -> (out, draws used)."""
        n = len(batch)
        pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
        ids = _u32(batch.ids if len(batch.ids) else np.zeros(1, np.uint32))
        out = np.empty(max(n, 1), np.int32)
        dr = np.ascontiguousarray(draws if len(draws) else np.zeros(1), dtype=np.uint64)
        used = C.c_uint32(0)
        rc = self._lib.ksg_schedule_batch_draws(self._ctx, abi.ptr(pods), n, abi.ptr(ids), len(batch.ids), abi.ptr(dr),
                                                len(draws), C.byref(used), abi.ptr(out))
        if rc != abi.KSG_OK:
            self._err(rc)
        return out[:n], int(used.value)

    def batch_unwind(self, batch: PodBatch, out, k: int, rng_state=None):
        """ksg_batch_unwind: pod k's Bind was rejected (scheduler.go:107-112). Undoes the
        commits of pods k..n-1 of the last batch; -> (draws pods 0..k consumed, the
        rng_state stepped back over pods k+1..n-1's draws, or None)."""
        n = len(batch)
        pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
        o = np.ascontiguousarray(out, dtype=np.int32)
        kept = C.c_uint32(0)
        st = C.c_uint64(0 if rng_state is None else int(rng_state))
        rc = self._lib.ksg_batch_unwind(self._ctx, abi.ptr(pods), abi.ptr(o), n, int(k),
                                        None if rng_state is None else C.byref(st), C.byref(kept))
        if rc != abi.KSG_OK:
            self._err(rc)
        return int(kept.value), (None if rng_state is None else st.value)

    def evaluate(self, batch: PodBatch, i: int = 0):
        """Per-node (fail code, combined score) of the shard, no commit."""
        pod = np.ascontiguousarray(batch.pods[i : i + 1])
        ids = _u32(batch.ids if len(batch.ids) else np.zeros(1, np.uint32))
        lo, hi = self.shard()
        fails = np.zeros(max(hi - lo, 1), np.uint8)
        scores = np.zeros(max(hi - lo, 1), np.int64)
        if batch.ext is not None:
            ext = np.ascontiguousarray(batch.ext[i : i + 1], dtype=abi.POD_EXT_DTYPE)
            rc = self._lib.ksg_evaluate_ext(self._ctx, abi.ptr(pod), abi.ptr(ext), abi.ptr(ids), abi.ptr(fails),
                                            abi.ptr(scores))
        else:
            rc = self._lib.ksg_evaluate(self._ctx, abi.ptr(pod), abi.ptr(ids), abi.ptr(fails), abi.ptr(scores))
        if rc not in (abi.KSG_OK, abi.KSG_NONODES):
            self._err(rc)
        return rc, fails[: hi - lo], scores[: hi - lo]

    def set_window(self, window: int):
        """Pods per speculative window (0 = exact one-pod-at-a-time kernel)."""
        rc = self._lib.ksg_set_window(self._ctx, int(window))
        if rc != abi.KSG_OK:
            self._err(rc)

    def last_batch_stats(self) -> dict:
        st = np.zeros(4, np.uint32)
        self._lib.ksg_last_batch_stats(self._ctx, abi.ptr(st))
        return {"windows": int(st[0]), "stops_service": int(st[1]), "stops_exhausted": int(st[2]),
                "stops_cache": int(st[3])}

    def last_batch_windows(self) -> int:
        return self.last_batch_stats()["windows"]

    def last_batch_kernel_ms(self) -> dict:
        """Window path: device ms of the snapshot kernel, of the resolver, windows."""
        o = np.zeros(3, np.float64)
        self._lib.ksg_last_batch_kernel_ms(self._ctx, abi.ptr(o))
        return {"eval_ms": float(o[0]), "resolve_ms": float(o[1]), "launches": int(o[2])}

    HOST_PHASES = ("validate", "upload", "setup", "enqueue", "mirror_replay", "round_wait", "final_wait",
                   "bookkeeping")

    def last_batch_host_us(self) -> dict:
        """Host microseconds of the last batch by phase (ksg_last_batch_host_us)."""
        o = np.zeros(8, np.float64)
        self._lib.ksg_last_batch_host_us(self._ctx, abi.ptr(o))
        return {k: float(v) for k, v in zip(self.HOST_PHASES, o)}

    def batch_totals(self) -> dict:
        """The per-batch diagnostics summed over every batch so far (ksg_batch_totals)."""
        o = np.zeros(24, np.float64)
        self._lib.ksg_batch_totals(self._ctx, abi.ptr(o))
        return {"batches": int(o[0]), "device_ms": float(o[1]), "eval_ms": float(o[2]),
                "resolve_ms": float(o[3]), "launches": int(o[4]), "windows": int(o[5]),
                "stops_service": int(o[6]), "stops_exhausted": int(o[7]), "stops_cache": int(o[8]),
                "host_us": {k: float(v) for k, v in zip(self.HOST_PHASES, o[9:17])},
                "wcap_sum": float(o[17]), "t0_ms": float(o[18])}

    def set_static_terms(self, fit_words, score, weighted: bool):
        """ksg_set_static_terms: static node terms past the config's slots (after
        set_cluster; fit_words uint64[ceil(N/64)] or None, score int64[N] or None)."""
        fw = None if fit_words is None else np.ascontiguousarray(fit_words, np.uint64)
        sc = None if score is None else np.ascontiguousarray(score, np.int64)
        rc = self._lib.ksg_set_static_terms(self._ctx, None if fw is None else abi.ptr(fw),
                                            None if sc is None else abi.ptr(sc), 1 if weighted else 0)
        if rc != abi.KSG_OK:
            self._err(rc)

    def add_static_config(self, extra: abi.KsgConfig):
        """ksg_add_static_config: one slot pass of LabelsPresence / LabelPreference terms
        past the config's slots, evaluated on the device from the node labels."""
        rc = self._lib.ksg_add_static_config(self._ctx, C.byref(extra))
        if rc != abi.KSG_OK:
            self._err(rc)

    def serve_stats(self) -> dict:
        """The resident begin/commit server (ksg_serve_stats)."""
        o = np.zeros(4, np.uint64)
        self._lib.ksg_serve_stats(self._ctx, abi.ptr(o))
        return {"launches": int(o[0]), "requests": int(o[1]), "running": bool(o[2]), "eligible": bool(o[3]),
                "grid": int(o[3]) == 2}

    def debug_counters(self) -> np.ndarray:
        """KSG_DEBUG=8 contexts: the window resolver's per-stage cycle counters
        (cycles / 64, summed over every window so far)."""
        o = np.zeros(abi.KSG_DEBUG_COUNTER_WORDS, np.int32)
        rc = self._lib.ksg_debug_counters(self._ctx, abi.ptr(o), len(o))
        if rc != abi.KSG_OK:
            self._err(rc)
        return o

    def last_batch_ms(self) -> float:
        ms = C.c_double(0)
        self._lib.ksg_last_batch_ms(self._ctx, C.byref(ms))
        return ms.value

    def shard(self):
        lo = C.c_uint32(0)
        hi = C.c_uint32(0)
        self._lib.ksg_shard(self._ctx, C.byref(lo), C.byref(hi))
        return lo.value, hi.value

    def admit(self, sets: np.ndarray, batch: PodBatch, pairs, mode: int = 3) -> np.ndarray:
        """Kubelet admission over many nodes' sets (ksg_admit.hip). mode 1:
        ksg_check_pods_exceeding_capacity (1 = fitting), 2: ksg_pod_matches_node_labels
        (1 = matches), 3: ksg_admit_pods (KSG_ADMIT_* codes)."""
        sets = np.ascontiguousarray(sets, dtype=abi.ADMISSION_SET_DTYPE)
        pods = np.ascontiguousarray(batch.pods, dtype=abi.POD_DTYPE)
        ids = _u32(batch.ids if len(batch.ids) else np.zeros(1, np.uint32))
        prs = _u32(pairs if len(pairs) else np.zeros(1, np.uint32))
        out = np.zeros(max(len(pods), 1), np.uint8)
        if mode == 1:
            rc = self._lib.ksg_check_pods_exceeding_capacity(self._ctx, abi.ptr(sets), len(sets), abi.ptr(pods),
                                                             len(pods), abi.ptr(out))
        elif mode == 2:
            rc = self._lib.ksg_pod_matches_node_labels(self._ctx, abi.ptr(sets), len(sets), abi.ptr(pods), len(pods),
                                                       abi.ptr(ids), len(batch.ids), abi.ptr(prs), len(pairs),
                                                       abi.ptr(out))
        else:
            rc = self._lib.ksg_admit_pods(self._ctx, abi.ptr(sets), len(sets), abi.ptr(pods), len(pods), abi.ptr(ids),
                                          len(batch.ids), abi.ptr(prs), len(pairs), abi.ptr(out))
        if rc != abi.KSG_OK:
            self._err(rc)
        return out[: len(pods)]

    def read_ext_used(self) -> np.ndarray:
        """Committed extended-resource usage, int64[n_scalar, n_nodes] (ksg_read_ext_used)."""
        u = np.zeros(max(self.n_scalar * self.n_nodes, 1), np.int64)
        rc = self._lib.ksg_read_ext_used(self._ctx, abi.ptr(u))
        if rc != abi.KSG_OK:
            self._err(rc)
        return u[: self.n_scalar * self.n_nodes].reshape(self.n_scalar, self.n_nodes)

    def read_requested(self):
        c = np.zeros(max(self.n_nodes, 1), np.int64)
        m = np.zeros(max(self.n_nodes, 1), np.int64)
        rc = self._lib.ksg_read_requested(self._ctx, abi.ptr(c), abi.ptr(m))
        if rc != abi.KSG_OK:
            self._err(rc)
        return c[: self.n_nodes], m[: self.n_nodes]


def gloo_allgather(group=None):
    """allgather callable for DeviceScheduler over a torch.distributed process
    group (host transport; e.g. gloo ranks sharing one GPU in tests)."""
    import torch
    import torch.distributed as dist

    def ag(send: bytes) -> bytes:
        t = torch.frombuffer(bytearray(send), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(outs, t, group=group)
        return b"".join(o.numpy().tobytes() for o in outs)

    return ag


# ---- node sharding (host side of the multi-GPU exchange; include/kschedgpu.h) ----
REC_HDR_BYTES = C.sizeof(abi.KsgShardRecord)


def shard_range(n_nodes: int, rank: int, world: int):
    """ksg_shard_range: node range [lo, hi) of `rank`'s shard."""
    lib = abi.load_library()
    lo, hi = C.c_uint32(0), C.c_uint32(0)
    rc = lib.ksg_shard_range(int(n_nodes), int(rank), int(world), C.byref(lo), C.byref(hi))
    if rc != abi.KSG_OK:
        raise KsgError(rc, "ksg_shard_range")
    return lo.value, hi.value


def merge_records(records: np.ndarray, n_nodes: int, empty_priorities: bool = False,
                  rng_state: int | None = None, tie_index: int = 0):
    """ksg_merge_records over a uint8[world, rec_bytes] array of shard records.
    -> (rc, node, max_score, tie_count, rng_state)."""
    lib = abi.load_library()
    rec = np.ascontiguousarray(records, dtype=np.uint8)
    world, rec_bytes = rec.shape
    node = C.c_int32(-1)
    m = C.c_int64(0)
    k = C.c_uint64(0)
    st = C.c_uint64(rng_state or 0)
    rc = lib.ksg_merge_records(abi.ptr(rec), rec_bytes, world, int(n_nodes), 1 if empty_priorities else 0,
                               C.byref(st) if rng_state is not None else None, int(tie_index), C.byref(node),
                               C.byref(m), C.byref(k))
    if rc not in (abi.KSG_OK, abi.KSG_NOFIT, abi.KSG_ERR_NOPEER):
        raise KsgError(rc, "ksg_merge_records")
    return rc, node.value, m.value, k.value, (st.value if rng_state is not None else None)


def make_shard_record(fails: np.ndarray, scores: np.ndarray, lo: int, word_lo: int, nwords_max: int,
                      error: bool = False) -> np.ndarray:
    """Pack one shard's record (header + tie bitmap) from its per-node fail codes and scores
    (the layout ksg_scan_kernel writes; used by callers that evaluate shards themselves)."""
    out = np.zeros(REC_HDR_BYTES + 8 * nwords_max, np.uint8)
    hdr = abi.KsgShardRecord.from_buffer(out)
    fit = fails == 0
    hdr.error = 1 if error else 0
    if fit.any() and not error:
        m = int(scores[fit].max())
        ties = np.nonzero(fit & (scores == m))[0] + lo
        hdr.max_score = m
        hdr.tie_count = len(ties)
        words = out[REC_HDR_BYTES:].view(np.uint64)
        rel = ties - word_lo * 64
        np.bitwise_or.at(words, rel // 64, (np.uint64(1) << (rel % 64).astype(np.uint64)))
    else:
        hdr.max_score = -(1 << 63)
        hdr.tie_count = 0
    return out
