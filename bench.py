#!/usr/bin/env python3
"""bench.py — pods scheduled/sec of the MI355X Filter/Score pass (BASELINE.json metric).

A "step" is one batch of `--batch` pods scheduled in order through the hot path
(filter every node, score, argmax + reference tie-break, commit) by
ksg_schedule_batch: windows of pods are scored against a snapshot on all CUs
and resolved in order, exactly, by one workgroup. Up to 65,536 nodes on one rank
(configs 1-3) that is one launch per window, ksg_win_fused_kernel (block 0
resolves while the other blocks score the window); past that, sharded, or with
the extensions, three: ksg_win_score_kernel, ksg_win_t0_kernel (per-pod T0
images) and ksg_win_plain_kernel; with ServiceAntiAffinity the count / score
passes and ksg_win_resolve2_kernel / ksg_win_resolve_kernel;
node state is resident in HBM before the timed region (the C ABI copies the
batch descriptors in, ~B*88 bytes, inside the step).

  N=1 : BASELINE config 2 — 5,000 nodes / 10,000 pods, DefaultProvider
        (PodFitsPorts, PodFitsResources, NoDiskConflict, MatchNodeSelector,
        HostName + LeastRequested(1), ServiceSpreading(1), Equal(0)).
  N>1 : BASELINE config 3 — 15,000 nodes node-sharded across N GPUs: each GPU
        scores its shard for a window of pods, the shards' per-word results are
        all-gathered with RCCL over xGMI once per window, and every GPU resolves
        the window identically over its replica of the node state (strong
        scaling: the total node count is fixed).

Roofline: bound "hbm"; achieved = algorithmic bytes per launch / kernel time,
with SURVEY.md 8(d)'s 60 B/node/pod for this predicate+priority set
(resources 32 + ports 8 + PD 8 + labels 8 + spread count 4) x nodes x pods per
launch; kernel time from HIP events on the library's stream. The resolver is a
latency-bound dependency chain, so the line also carries `latency`: resolver
cycles per pod at the 2.4 GHz engine clock and, from an untimed KSG_DEBUG=8
rerun, the chain's per-stage cycles. cpu_baseline: the
C restatement in faithful mode (the reference's per-pod MapPodsToMachines
regroup + per-node rescans + sort; single thread like the reference's one
scheduling goroutine) timed on this host over a bounded prefix of the same
workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from tools.srcsha import kernel_src_sha  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip-level parameters
CLOCK_MHZ = 2400.0  # MI355X max engine clock (MI355X_MICROARCH.md); the resolver's stamps count it
BYTES_PER_NODE = {"config1": 32, "config2": 60, "config3": 60, "config4": 64, "config5": 84}


def traffic_entry(tj, key, src_sha, stale):
    """profiles/traffic.json's PMC entry for key, only when it was measured on the build of
    these sources (its kernel_src_sha, tools/srcsha.py); an entry from another build is
    appended to stale (reported as roofline.traffic_source.stale) and not used."""
    ent = tj.get(key)
    if ent and ent.get("kernel_src_sha") != src_sha:
        stale.append({"entry": key, "source": ent.get("source"), "round": ent.get("round")})
        return None
    return ent


def _dist_env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(
        os.environ.get("LOCAL_RANK", "0"))


def _torch_sync():
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


# KSG_DEBUG=8 counter layout of the register-slot resolver (ksg_window.hip):
# lane -> (role, stage); counters are cycles / 64 summed over windows
_STAGES2 = {
    0: ("committer", "ring_wait"), 1: ("committer", "head"), 2: ("committer", "wait_checkers_and_xcheck"),
    3: ("committer", "select"), 4: ("committer", "slot_and_node_post"), 5: ("committer", "commit"),
    6: ("handoff", "xcheck_to_committer"), 31: ("handoff", "node_to_xchecker"),
    10: ("committer", "ring_wait_first4"), 11: ("committer", "ring_wait_rest"),
    16: ("checker0", "wait"), 17: ("checker0", "apply"), 18: ("checker0", "check"),
    19: ("checker1", "wait"), 20: ("checker1", "apply"), 21: ("checker1", "check"),
    24: ("producers_sum_over_waves", "ring_wait"), 25: ("producers_sum_over_waves", "loads"),
    26: ("producers_sum_over_waves", "draw_wait"), 27: ("producers_sum_over_waves", "stage"),
    28: ("xchecker", "wait_node"), 29: ("xchecker", "check"), 30: ("xchecker", "bookkeeping_and_lists"),
    # (ServiceAntiAffinity re-ranks: their count x 64 per pod and their cycles)
    9: ("committer", "rerank_x64"), 12: ("committer", "rerank_cycles"),
    22: ("checker0", "check_record"), 23: ("checker0", "check_slot"),  # (check = these + the row sums and post)
}


# the plain resolver (every configuration without ServiceAntiAffinity, ksg_plain.hip)
_STAGES_PLAIN = {
    0: ("committer", "ring_wait"), 1: ("committer", "head"),
    2: ("committer", "wait_checkers_and_xcheck"), 3: ("committer", "select_and_node_post"),
    4: ("committer", "slot"), 5: ("committer", "commit"),
    6: ("handoff", "xcheck_to_committer"), 31: ("handoff", "node_to_xchecker"),
    10: ("committer", "ring_wait_first4"), 11: ("committer", "ring_wait_rest"),
    12: ("committer", "verdict_reads"), 13: ("committer", "head_reads"),  # (select / head = the rest)
    16: ("checker0", "wait"), 17: ("checker0", "apply"), 18: ("checker0", "check"),
    19: ("checker1", "wait"), 20: ("checker1", "apply"), 21: ("checker1", "check"),
    22: ("checker0", "check_loads"), 23: ("checker0", "check_resources_lr"),  # (check = the rest)
    14: ("checker0", "ext_fit"), 15: ("checker0", "ext_score"), 9: ("checker0", "ext_verdict"),  # (extension scores)
    24: ("producers_sum_over_waves", "ring_wait"), 25: ("producers_sum_over_waves", "loads"),
    26: ("producers_sum_over_waves", "draw_wait"), 27: ("producers_sum_over_waves", "stage"),
    28: ("xchecker", "wait_node"), 32: ("xchecker", "check"),
    33: ("xchecker", "ext_score"), 29: ("xchecker", "post_and_replay"), 34: ("xchecker", "ring_wait"),
    39: ("flagger", "wait"), 40: ("flagger", "flags"),
    # (counts x 64 per pod: commits whose node's verdict the committer took from phase A's
    # single-commit drop bitmap, and those the x-checker checked)
    41: ("xchecker", "x_by_committer_x64"), 42: ("xchecker", "x_checked_x64"),
    43: ("committer", "entry_not_staged_x64"),  # (pods whose ring entry the head round found unstaged)
    44: ("committer", "entry_wait"),  # (cycles waiting for those entries, per pod of the run)
}


def _phase_a_bytes(cfg, pods, ids, ns, nw, w):
    """Algorithmic bytes of one phase-A launch (ksg_win_score_kernel) scoring w
    pods on a shard of ns nodes / nw words, counting each distinct row once per
    launch (the window's pods share rows in L2; FETCH_SIZE sees a row once): the
    node state (cap and requested totals 32 B, the static score 4 B) and the
    LabelsPresence word once; one 8-byte word per word of every DISTINCT
    predicate row the window's pods name (nodeSelector pairs, PD and host-port
    keys, ServiceAffinity pairs); the service-count row (4 B per node) of every
    distinct service among them (when ServiceSpreading or ServiceAntiAffinity is
    on); the per-(pod, word) best score + tie bitmap written (12 B) and the pods'
    192-byte records. Averaged over the batch's consecutive windows of w pods."""
    w = max(1, int(round(w)))
    na = int(cfg.n_aff_labels)
    cnt_on = int(cfg.w_service_spreading) != 0 or any(int(cfg.w_anti[a]) != 0 for a in range(int(cfg.n_anti)))
    n = len(pods)
    rows, svcs = [], []
    for w0 in range(0, max(n - w + 1, 1), w):
        sel, keys, aff, sv = set(), set(), set(), set()
        for p in pods[w0:w0 + w]:
            sel.update(ids[int(p["sel_off"]):int(p["sel_off"]) + int(p["n_sel"])].tolist())
            keys.update(ids[int(p["pds_off"]):int(p["pds_off"]) + int(p["n_pds"])].tolist())
            keys.update(ids[int(p["ports_off"]):int(p["ports_off"]) + int(p["n_ports"])].tolist())
            for j in range(na):
                if int(p["aff_pair"][j]) >= 0:
                    aff.add(int(p["aff_pair"][j]))
            if int(p["service"]) >= 0:
                sv.add(int(p["service"]))
        rows.append(len(sel | aff) + len(keys))  # (pairmap rows: selector and affinity pairs; keymap rows)
        svcs.append(len(sv))
    u_rows = float(np.mean(rows)) if rows else 0.0
    u_svc = float(np.mean(svcs)) if svcs else 0.0
    return (36.0 * ns + 8.0 * nw + u_rows * nw * 8.0 + (u_svc * ns * 4.0 if cnt_on else 0.0)
            + w * nw * 12.0 + w * 192.0)


def _stage_breakdown(cfg, view, args, step_batch, anti, ext=None):
    """Per-stage resolver cycles per pod from a KSG_DEBUG=8 context over the
    bench's first steps (untimed; the stamps cost a few percent)."""
    from kubernetes_amd import workload
    from kubernetes_amd.engine import DeviceScheduler

    old = os.environ.get("KSG_DEBUG")
    os.environ["KSG_DEBUG"] = str(int(old or "0") | 8)  # read when the context builds its device state
    s2 = None
    try:
        s2 = DeviceScheduler(cfg, device=0)
        if args.window is not None:
            s2.set_window(args.window)
        if ext is not None:
            s2.set_extensions(ext[0])
        s2.set_cluster(view.arrays)
        if ext is not None:
            s2.set_node_ext(*ext[1])
        rng = workload.TIEBREAK_SEED
        pods = 0
        for s in range(min(3, args.warmup + args.steps)):
            b = step_batch(s)
            _, rng = s2.batch(b, rng)
            pods += len(b.pods)
        c = s2.debug_counters().astype(np.int64) * 64
    finally:
        if s2 is not None:
            s2.close()
        if old is None:
            del os.environ["KSG_DEBUG"]
        else:
            os.environ["KSG_DEBUG"] = old
    if anti:
        return {"pods": pods, "raw_cycles_per_pod": [round(float(v) / pods, 1) for v in c],
                "note": "LDS-slot resolver (ServiceAntiAffinity): raw counters, layout in ksg_window.hip"}
    out = {"pods": pods, "unit": "cycles/pod",
           "drops_per_pod": float(c[7]) / 64 / pods, "unpredicted_per_pod": float(c[8]) / 64 / pods}
    plain = not any(int(cfg.w_anti[a]) != 0 for a in range(int(cfg.n_anti)))
    for lane, (role, st) in (_STAGES_PLAIN if plain else _STAGES2).items():
        out.setdefault(role, {})[st] = round(float(c[lane]) / pods, 1)
    nwin = float(c[54]) / 64
    if plain and nwin > 0:  # the fused launch's window start (10-ns ticks, s_memrealtime), per window
        out["window_start_us"] = {"windows": int(nwin),
                                  "to_first_group_scored": round(float(c[52]) / 64 / nwin / 100, 2),
                                  "to_first_entry_staged": round(float(c[53]) / 64 / nwin / 100, 2)}
        ntask = float(c[61]) / 64
        if ntask > 0:  # the first scoring task's timeline from block 0's start (us, per window)
            out["window_start_us"]["first_task"] = {
                k_: round(float(c[i]) / 64 / ntask / 100, 2)
                for i, k_ in ((56, "block_start"), (57, "task_start"), (58, "scored"), (59, "drained"),
                              (60, "counted"))}
    return out


def _phase_a_standalone(cfg, view, args, step_batch, ext=None, world=1):
    """The fused window launch (one plain rank) scores each window inside the resolver's
    launch, so phase A has no events of its own there. Its standalone time comes from an
    untimed context with KSG_FUSED=0 over the bench's first steps: phase A, the T0-image
    kernel and the resolver launched apart, the scoring kernel's own HIP events."""
    from kubernetes_amd import workload
    from kubernetes_amd.engine import DeviceScheduler

    old = os.environ.get("KSG_FUSED")
    os.environ["KSG_FUSED"] = "0"
    s2 = None
    try:
        s2 = DeviceScheduler(cfg, device=0)
        if args.window is not None:
            s2.set_window(args.window)
        if ext is not None:
            s2.set_extensions(ext[0])
        s2.set_cluster(view.arrays)
        if ext is not None:
            s2.set_node_ext(*ext[1])
        rng = workload.TIEBREAK_SEED
        for s in range(args.warmup):  # (the same warm-up as the timed run, then its first steps)
            _, rng = s2.batch(step_batch(s), rng)
        t0 = s2.batch_totals()
        for s in range(args.warmup, args.warmup + min(4, args.steps)):
            _, rng = s2.batch(step_batch(s), rng)
        t1 = s2.batch_totals()
        t = {k_: t1[k_] - t0[k_] for k_ in ("launches", "eval_ms", "t0_ms", "wcap_sum", "resolve_ms")}
    finally:
        if s2 is not None:
            s2.close()
        if old is None:
            del os.environ["KSG_FUSED"]
        else:
            os.environ["KSG_FUSED"] = old
    if t["launches"] <= 0 or t["eval_ms"] <= 0:
        return None
    return {"eval_ms_avg": t["eval_ms"] / t["launches"], "t0_ms_avg": t["t0_ms"] / t["launches"],
            "wcap_mean": t["wcap_sum"] / t["launches"] if t["wcap_sum"] > 0 else None,
            "resolve_ms_avg": t["resolve_ms"] / t["launches"], "launches": t["launches"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1000, help="pods per step")
    ap.add_argument("--workload", default=None, help="config1..config5 (default: config2 at N=1, config3 at N>1)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--window", type=int, default=None,
                    help="pods per speculative window (0 = exact one-pod-at-a-time kernel)")
    ap.add_argument("--transport", choices=("rccl", "gloo"), default="rccl",
                    help="N>1 exchange: RCCL over xGMI (default), or host-staged over the gloo group "
                         "(rehearsal of the sharded path with several ranks on one GPU)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (profiles/), keyed by workload")
    ap.add_argument("--extensions", action="store_true",
                    help="add the extensions beyond this reference vintage (taints / tolerations, GPU and FPGA "
                         "counts, TaintToleration + BalancedResourceAllocation; parity unpinned; the window path, "
                         "--window 0 for the exact kernels), reported as a separate workload (SURVEY.md section 0, "
                         "item 2)")
    ap.add_argument("--ext-filters-only", action="store_true",
                    help="with --extensions: the filters only (taints, extended resources), TaintToleration and "
                         "BalancedResourceAllocation weights 0")
    ap.add_argument("--ext-taints-only", action="store_true",
                    help="with --extensions --ext-filters-only: no extended resources either (taints and "
                         "tolerations only: with ServiceAntiAffinity, config 4, the window path takes them)")
    ap.add_argument("--prefix-pods", type=int, default=0,
                    help="place this many of the workload's first pods (untimed, 5,000-pod batches) before the "
                         "warm-up, so the timed steps run on the late-run state (fuller nodes, FitErrors); the "
                         "cpu_baseline legs start from the same state (the prefix's placements added as pods)")
    ap.add_argument("--no-stages", action="store_true",
                    help="skip the resolver's per-stage cycle breakdown (a second, untimed run with KSG_DEBUG=8)")
    args = ap.parse_args()

    # HIP events around every 8th window launch (the library's default is every 4th): each event
    # record between two dependent launches adds ~4.5 us to the gap between them (kernel trace:
    # 0 us between launches without one), so the sampled kernel times cost the timed region
    # ~0.7 % instead of ~1.5 %; KSG_KERNEL_EVENTS in the environment overrides
    os.environ.setdefault("KSG_KERNEL_EVENTS", "8")
    world, rank, local_rank = _dist_env()
    if world != args.gpus and world > 1:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus={args.gpus}")
    wl = args.workload or ("config2" if world == 1 else "config3")
    pre = max(0, args.prefix_pods)
    n_pods = pre + (args.warmup + args.steps) * args.batch

    from kubernetes_amd import ingest, workload
    from kubernetes_amd.engine import DeviceScheduler, PodBatch

    t0 = time.time()
    w = workload.build(wl, n_nodes=args.nodes, n_pods=n_pods)
    it = ingest.Interner()
    for k in w.config.label_keys():
        it.key_id(k)
    view = ingest.ClusterView(w.nodes, w.services, it)
    batch = ingest.ingest_pods(view, w.pods, aff_labels=w.config.affinity_labels())
    cfg = w.config.compile(it.key_id)
    n_nodes = view.arrays.n_nodes
    ext = None  # (--extensions) the context's ExtConfig and node arrays
    if args.extensions:
        from kubernetes_amd.extensions import ExtInterner

        fo = args.ext_filters_only
        ecfg, node_taints, node_scalar, tols, scal = workload.extension_data(n_nodes, n_pods, w_taint=0 if fo else 1,
                                                                             w_bal=0 if fo else 1,
                                                                             gpus=not (fo and args.ext_taints_only))
        inter = ExtInterner(ecfg)
        node_arrays = inter.node_arrays(node_taints, node_scalar)
        rec, ids_x = inter.pod_records(batch.ids, tols, scal)
        batch = PodBatch(batch.pods, ids_x, rec)
        ext = (ecfg.compile(max(len(inter.taints), 1)), node_arrays)

    def load_cluster(s):
        """set_cluster (+ the extensions, which must be enabled before it)."""
        if ext is not None:
            s.set_extensions(ext[0])
        s.set_cluster(view.arrays)
        if ext is not None:
            s.set_node_ext(*ext[1])
        return s
    if rank == 0:
        print(f"[bench] {wl}: {n_nodes} nodes, {n_pods} pods, ingest {time.time() - t0:.1f}s", file=sys.stderr,
              flush=True)

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        dist = dist_mod
        if torch.cuda.is_available() and torch.cuda.device_count() > local_rank:
            torch.cuda.set_device(local_rank)  # torch's syncs (barrier()) on this rank's GPU, not GPU 0
        dist.init_process_group("gloo")
        if args.transport == "rccl":
            idb = DeviceScheduler.nccl_unique_id() if rank == 0 else bytes(128)
            obj = [idb]
            dist.broadcast_object_list(obj, src=0)
            sched = DeviceScheduler(cfg, device=local_rank, rank=rank, world=world, nccl_id=obj[0])
        else:
            from kubernetes_amd.engine import gloo_allgather

            ndev = max(torch.cuda.device_count(), 1)
            sched = DeviceScheduler(cfg, device=local_rank % ndev, rank=rank, world=world,
                                    allgather=gloo_allgather())
    else:
        sched = DeviceScheduler(cfg, device=0)
    if args.window is not None:
        sched.set_window(args.window)
    load_cluster(sched)

    def pod_slice(lo, hi):
        return PodBatch(batch.pods[lo:hi], batch.ids, None if batch.ext is None else batch.ext[lo:hi])

    def step_batch(s):
        return pod_slice(pre + s * args.batch, pre + (s + 1) * args.batch)

    rng = workload.TIEBREAK_SEED
    out_pre = []  # (--prefix-pods) the untimed prefix's placements
    for lo in range(0, pre, 5000):
        o, rng = sched.batch(pod_slice(lo, min(pre, lo + 5000)), rng)
        out_pre.append(o)
    out_pre = np.concatenate(out_pre) if out_pre else np.zeros(0, np.int32)
    rng_pre = rng
    outs = []
    for s in range(args.warmup):
        o, rng = sched.batch(step_batch(s), rng)
        outs.append(o)

    def barrier():
        if dist is not None:
            dist.barrier()
        _torch_sync()

    # the library's per-batch diagnostics (device ms, kernel ms from the HIP
    # events, window stats, host phases) accumulate in the context: read once
    # on each side of the timed steps (ksg_batch_totals), not after every step
    tot0 = sched.batch_totals()
    barrier()
    t_start = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        o, rng = sched.batch(step_batch(s), rng)
        outs.append(o)
    barrier()
    elapsed = time.perf_counter() - t_start
    tot1 = sched.batch_totals()
    assert tot1["batches"] - tot0["batches"] == args.steps
    kern_ms = [(tot1["device_ms"] - tot0["device_ms"]) / args.steps]
    host_us = {k_: tot1["host_us"][k_] - tot0["host_us"][k_] for k_ in tot1["host_us"]}
    kk = {k_: tot1[k_] - tot0[k_] for k_ in ("eval_ms", "resolve_ms", "launches", "t0_ms")}
    wstats = {k_: tot1[k_] - tot0[k_] for k_ in ("windows", "stops_service", "stops_exhausted", "stops_cache")}
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    out = np.concatenate(outs)
    timed = out[args.warmup * args.batch:]
    pods_timed = args.steps * args.batch
    value = pods_timed / elapsed

    if rank != 0:
        sched.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel ----------------------------------------
    # window path (default): the resolver dominates (rocprof: >90% of device
    # time); one launch resolves a window of pods, so algorithmic bytes per
    # launch = pods_per_launch x nodes x B/node and the launch duration comes
    # from the HIP events the library records around each resolver launch.
    # exact path (--window 0) / sharded: the one batch kernel per step.
    bpn = BYTES_PER_NODE.get(wl, 60)
    # the in-order resolver this config runs: the LDS-slot one for ServiceAntiAffinity
    # without the re-rank (several anti priorities, > 31 label values, sharded,
    # KSG_DEBUG & 2048 / 4096), else the register-slot one (ksg_window.hip,
    # ksg_set_cluster's rr_dz)
    dbg = int(os.environ.get("KSG_DEBUG", "0") or 0)
    anti = any(int(cfg.w_anti[a]) != 0 for a in range(int(cfg.n_anti)))
    plain = not anti  # no ServiceAntiAffinity: the plain resolver (ksg_plain.hip)
    if anti:
        pk = np.asarray(view.arrays.pair_keys, np.uint32) & np.uint32(0x7FFFFFFF)
        n_dom = int((pk[1:] == np.uint32(cfg.anti_key[0])).sum()) if len(pk) > 1 else 0
        rerank = (int(cfg.n_anti) == 1 and world == 1 and n_dom + 1 <= 32 and view.arrays.n_services <= 4096
                  and not (dbg & 2048))
        anti = not (rerank and not (dbg & 4096))  # True: the LDS-slot resolver runs
    wcap = args.window if args.window else int(os.environ.get("KSG_WINDOW", "128"))
    nwords = (n_nodes + 63) // 64
    if kk["launches"] > 0:
        launches = kk["launches"]
        pods_per_launch = pods_timed / launches
        # (KSG_KERNEL_EVENTS=0 drops the per-kernel events: no kernel times, an A/B switch)
        kavg_s = kk["resolve_ms"] / launches / 1e3 or float("nan")
        kavg_sampled_s = kavg_s
        # the in-order resolver: the plain one without ServiceAntiAffinity (ksg_plain.hip),
        # else the LDS-slot one or the register-slot re-rank (ksg_window.hip)
        # the fused window launch (one plain rank, no extensions): phase A runs inside the
        # resolver's launch, one kernel per window (ksg_win_fused_kernel)
        fused = kk["eval_ms"] == 0 and plain and world == 1
        kname = ("ksg_win_fused_kernel" if fused else "ksg_win_plain_kernel" if plain else
                 "ksg_win_resolve_kernel" if anti else "ksg_win_resolve2_kernel")
        if fused:
            # one kernel per window and nothing else on the stream but the batch's two small copies:
            # the batches' own HIP events (ksg_last_batch_ms, every launch of the timed steps) over
            # the launches give the kernel's mean duration without the sampling noise of every 8th
            # launch (a round mixes ~250-us windows, a short last one and ~4-us no-op launches;
            # round-6 record: within 1-2 % of the kernel trace's timed launches, the sampled mean
            # 8-15 % off)
            kavg_s = (tot1["device_ms"] - tot0["device_ms"]) / launches / 1e3
        # phase A scores this rank's shard (N/world nodes) for the window's W pods
        # (the capacity the library used: it shrinks W where windows stop early); its
        # events bracket the scoring kernel(s) only (the T0-image kernel and, with
        # world > 1, the per-window all-gather are timed apart: win_t0_ms_avg).
        ev_s = kk["eval_ms"] / launches / 1e3 or float("nan")
        w_used = tot1["wcap_sum"] - tot0["wcap_sum"]
        w_mean = w_used / launches if w_used > 0 else float(wcap)
        # (fused: phase A's standalone time from an untimed KSG_FUSED=0 side run)
        side = _phase_a_standalone(cfg, view, args, step_batch, ext) if fused else None
        if side:
            ev_s = side["eval_ms_avg"] / 1e3
            w_mean = side["wcap_mean"] or w_mean
        ev_bytes = _phase_a_bytes(cfg, batch.pods[:4096], np.asarray(batch.ids), n_nodes / world, nwords / world,
                                   w_mean)
        # (HIP events around every timed_launch_stride-th launch of a round, the
        # sampled mean scaled to all launches; KSG_KERNEL_EVENTS=N sets the stride)
        extra = {"launches": launches, "pods_per_launch": pods_per_launch,
                 "timed_launch_stride": int(os.environ.get("KSG_KERNEL_EVENTS", "8") or 0),
                 "win_eval_ms_avg": kk["eval_ms"] / launches,
                 "win_t0_ms_avg": kk["t0_ms"] / launches,
                 "win_eval_model_bytes_per_launch": ev_bytes,
                 "win_eval_pods_per_launch": w_mean,
                 "win_eval_model_GBps": ev_bytes / ev_s / 1e9,
                 "win_eval_node_pod_evals_per_s": (n_nodes / world) * wcap / ev_s,
                 "fused_window_launch": bool(fused)}
        if fused:
            extra["kernel_ms_avg_basis"] = "batch HIP events (ksg_last_batch_ms) / launches"
            extra["kernel_ms_avg_sampled_events"] = kavg_sampled_s * 1e3
        if fused:
            extra["win_eval_source"] = ("untimed KSG_FUSED=0 side run over the first steps: phase A's own "
                                        "events; in the timed run it scores inside ksg_win_fused_kernel")
            extra["unfused_side_run"] = side
    else:
        pods_per_launch = args.batch
        kavg_s = float(np.mean(kern_ms)) / 1e3 if kern_ms else float("nan")
        kname = "ksg_batch_kernel" if world == 1 else "ksg_scan_kernel+ksg_decide_kernel+rccl"
        extra = {"launches": args.steps, "pods_per_launch": pods_per_launch}
    alg_bytes = bpn * n_nodes * pods_per_launch
    achieved = alg_bytes / kavg_s
    traffic = None
    tj = {}
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        pass
    src_sha = kernel_src_sha()
    stale = []

    def counters(key):
        return traffic_entry(tj, key, src_sha, stale)

    ent = counters(f"{wl}:{n_nodes}:{kname}")
    if ent:
        traffic = ent["hbm_bytes_per_launch"]
    traffic_source = {"kernel_src_sha": src_sha, "resolver": ent and {"source": ent["source"], "round": ent["round"]},
                      "stale": stale}
    roofline = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel": kname,
                "kernel_ms_avg": kavg_s * 1e3, "bytes_per_node_pod": bpn, "alg_bytes_per_launch": alg_bytes}
    roofline.update(extra)
    roofline["traffic_source"] = traffic_source
    filter_score = None
    if kk["launches"] > 0:
        ent = counters(f"{wl}:{n_nodes}:ksg_win_score_kernel")  # phase A's counter-measured bytes (profiles/)
        traffic_source["filter_score"] = ent and {"source": ent["source"], "round": ent["round"]}
        if ent:
            roofline["win_eval_traffic"] = ent["hbm_bytes_per_launch"]
            roofline["win_eval_traffic_GBps"] = ent["hbm_bytes_per_launch"] / ev_s / 1e9
        # the filter/score kernel itself (phase A: every node of the shard x the window's pods,
        # findNodesThatFit + prioritizeNodes, generic_scheduler.go:100-165) against the HBM peak:
        # its counter-measured bytes (FETCH x2 + WRITE, profiles/traffic.json) when this workload
        # has a PMC pass, else its byte model, over its mean launch time from the HIP events
        fs_bytes = ent["hbm_bytes_per_launch"] if ent else ev_bytes
        filter_score = {"kernel": "ksg_win_score_kernel" + (" (standalone, KSG_FUSED=0 side run)" if fused else ""),
                        "bound": "hbm", "unit": "GB/s",
                        "basis": "pmc_traffic" if ent else "byte_model",
                        "bytes_per_launch": fs_bytes, "ms_avg": ev_s * 1e3,
                        "achieved": fs_bytes / ev_s / 1e9, "peak": HBM_PEAK / 1e9,
                        "frac": fs_bytes / ev_s / HBM_PEAK,
                        "pods_per_launch": w_mean, "nodes": n_nodes / world}
        roofline["filter_score_frac"] = filter_score["frac"]

    # ---- latency view: the resolver is one in-order dependency chain per window
    # (one workgroup), so its bound is the chain's cycles per pod,
    # not bytes. Stage breakdown: a second, untimed run of the first steps on a
    # context with the resolver's s_memtime stamps on (KSG_DEBUG=8).
    latency = None
    if kk["launches"] > 0:
        us_pod = kk["resolve_ms"] * 1e3 / pods_timed
        latency = {"bound": "latency", "resolver_us_per_pod": us_pod, "clock_mhz": CLOCK_MHZ,
                   "resolver_cycles_per_pod": us_pod * CLOCK_MHZ,
                   "window_eval_us_per_pod": kk["eval_ms"] * 1e3 / pods_timed}
        if world == 1 and not args.no_stages:
            latency["stages"] = _stage_breakdown(cfg, view, args, step_batch, anti, ext)

    # ---- CPU baseline: faithful restatement, single thread, bounded prefix ------
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        from oracle.pyoracle import OracleScheduler

        n_run = n_pods - pre  # (the pods after the prefix: warm-up + timed)

        def cpu_ctx(faithful):
            """An oracle at the state the GPU's warm-up started from: the prefix's placements
            added as pods on their nodes (ksg_add_pod's form), in placement order."""
            o_ = load_cluster(OracleScheduler(cfg, faithful=faithful))
            for i in np.flatnonzero(out_pre >= 0):
                o_.add_pod(int(out_pre[i]), batch, int(i))
            return o_

        orc = cpu_ctx(True)
        r = rng_pre
        done = 0
        t_c = time.perf_counter()
        chunk = 50
        cpu_out = []
        while done < n_run and time.perf_counter() - t_c < args.cpu_seconds:
            o, r = orc.batch(pod_slice(pre + done, pre + min(n_run, done + chunk)), r)
            cpu_out.append(o)
            done += len(o)
        cpu_s = time.perf_counter() - t_c
        cpu_out = np.concatenate(cpu_out)
        agree = bool(np.array_equal(cpu_out, out[:done]))
        # the stronger CPU design point beside it: the same restatement in incremental
        # mode (closed forms over SoA, no per-pod re-list), one thread, a bounded prefix
        inc = cpu_ctx(False)
        r = rng_pre
        done_i = 0
        t_i = time.perf_counter()
        while done_i < n_run and time.perf_counter() - t_i < min(args.cpu_seconds, 5.0):
            o, r = inc.batch(pod_slice(pre + done_i, pre + min(n_run, done_i + 200)), r)
            done_i += len(o)
        inc_s = time.perf_counter() - t_i
        inc.close()
        # ... and node-sharded over this process's CPU share (OMP_NUM_THREADS: 16 on the
        # GPU box, whose os.cpu_count() is the whole machine's), SURVEY.md 8(d) "CPU timing" ii
        nthr = max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
        mt = cpu_ctx(False)
        r = rng_pre
        done_m = 0
        mt_out = [np.zeros(0, np.int32)]
        t_m = time.perf_counter()
        # the whole run's pods (warm-up + timed) when they fit the budget: this leg is also the
        # decision check of every pod the GPU placed, extension records included
        while done_m < n_run and time.perf_counter() - t_m < max(args.cpu_seconds, 30.0):
            o, r = mt.batch_mt(pod_slice(pre + done_m, pre + min(n_run, done_m + 500)), r, nthr)
            mt_out.append(o)
            done_m += len(o)
        mt_s = max(time.perf_counter() - t_m, 1e-9)
        mt_all = done_m == n_run and r == rng  # (and the generator state after the last timed step)
        mt.close()
        mt_agree = bool(np.array_equal(np.concatenate(mt_out), out[:done_m]))
        start = (f"from the state after the first {pre} pods (the GPU's placements added)" if pre
                 else "from an empty cluster")
        cpu = {"value": done / cpu_s, "unit": "pods/s", "cores": 1, "kind": "port",
               "sample": f"first {done} pods of the same {wl} workload on {n_nodes} nodes {start} "
                         f"({cpu_s:.1f}s, faithful mode: per-pod MapPodsToMachines regroup, per-node predicate "
                         f"rescans, HostPriorityList sort); decisions identical to GPU: {agree}",
               "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
               "incremental": {"value": done_i / inc_s, "unit": "pods/s", "cores": 1,
                               "sample": f"first {done_i} pods {start}, incremental mode (SoA closed forms, "
                                         f"no per-pod re-list), {inc_s:.1f}s"},
               "incremental_nproc": {"value": done_m / mt_s, "unit": "pods/s", "cores": nthr,
                                     "sample": f"first {done_m} of the run's {n_run} pods (warm-up + timed) {start}, "
                                               f"incremental mode, each pod's node loop split over {nthr} threads "
                                               f"(node-rank shards, two spin barriers per pod; ServiceAntiAffinity "
                                               f"configs run 1 thread), {mt_s:.1f}s; decisions identical to GPU: "
                                               f"{mt_agree}",
                                     "decisions_identical": mt_agree, "pods_checked": done_m,
                                     "whole_run_checked": bool(mt_all and mt_agree)}}

    xname = "RCCL" if args.transport == "rccl" else "host-staged gloo"
    line = {
        "metric": "pods scheduled/sec",
        "value": value,
        "unit": "pods/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "device_ms_per_step": float(np.mean(kern_ms)) if kern_ms else None,
        "host_us_per_step": {k_: round(v_ / args.steps, 1) for k_, v_ in host_us.items()},
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded splitmix64 scheduler_perf-style cluster; SURVEY.md 8(d))",
        "config": {"workload": f"{wl}: {n_nodes} nodes, {n_pods} pods, "
                               + ("DefaultProvider" if wl in ("config2", "config3", "config5") else wl)
                               + ((" + extension filters (taints/tolerations; scoring extensions off; parity "
                                   "unpinned)" if args.ext_filters_only and args.ext_taints_only else
                                   " + extension filters (taints/tolerations, GPU/FPGA counts; scoring "
                                   "extensions off; parity unpinned, window path)" if args.ext_filters_only else
                                   " + extensions (taints/tolerations, GPU/FPGA counts, TaintToleration, "
                                   "BalancedResourceAllocation; parity unpinned)") if ext else ""),
                   "nodes": n_nodes, "pods_per_step": args.batch,
                   "prefix_pods": pre, "placed_in_prefix": int((out_pre >= 0).sum()),
                   "timed_pods": [pre + args.warmup * args.batch, n_pods],
                   "placed_in_timed": int((timed >= 0).sum()), "fit_errors_in_timed": int((timed == -1).sum()),
                   "snapshots_in_timed": wstats,
                   "exchange": None if world == 1 else args.transport,
                   "parallelism": ("speculative windows: all-CU snapshot scoring + in-order exact resolver"
                                   if kk["launches"] else "single workgroup persistent kernel") if world == 1
                   else (f"node-sharded x{world}: shard scoring, {xname} all-gather per window, replicated resolver"
                         if kk["launches"] else f"node-sharded x{world}, {xname} all-gather per pod")},
        "roofline": roofline,
        "filter_score": filter_score,
        "latency": latency,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    sched.close()
    if dist is not None:
        dist.destroy_process_group()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for l in f:
                if l.startswith("model name"):
                    return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
