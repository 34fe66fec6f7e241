#!/usr/bin/env python3
"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/profile_gpu.sh) into
profiles/traffic.json: HBM-side bytes per launch of each window-path kernel.

Units and corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts half
the bytes of a wide read (128-B requests tallied at 64 B), so it is doubled. The
doubling is calibrated here for every access width the kernels use
(tools/fetch_calib.hip, profiles/r3_fetch_calib.json): contiguous 4-, 8- and
16-B-per-lane reads, 8-B gathers one per 64-B or 128-B line, agent-scope (sc1)
8-B loads -- FETCH_SIZE x 1024 is exactly half the bytes of the 128-B lines
touched in each case.

Each entry carries the round tag (KSG_ROUND, e.g. "r5") and the kernel sources' sha
(tools/srcsha.py) of the tree it was measured on; bench.py takes an entry only when that
sha is the current one.

usage: tools/traffic_from_pmc.py <prof_dir> <workload> <n_nodes> [profiles/traffic.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tools.srcsha import kernel_src_sha  # noqa: E402

KERNELS = {"ksg_win_plain_kernel": "ksg_win_plain_kernel", "ksg_win_fused_kernel": "ksg_win_fused_kernel",
           "ksg_win_t0_kernel": "ksg_win_t0_kernel",
           "ksg_win_resolve_kernel": "ksg_win_resolve_kernel", "ksg_win_resolve2_kernel": "ksg_win_resolve2_kernel",
           "ksg_win_resolve3_kernel": "ksg_win_resolve3_kernel", "ksg_win_score_kernel": "ksg_win_score_kernel",
           "ksg_batch_kernel": "ksg_batch_kernel"}


def per_launch(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            for key in KERNELS:
                if row["Kernel_Name"].split("(")[0].split("<")[0].split()[-1] == key:
                    acc[key].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items() if v}


def main():
    prof, wl, n_nodes = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "traffic.json")
    fetch = per_launch(os.path.join(prof, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_launch(os.path.join(prof, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    try:
        with open(out) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        tj = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * fetch.get(k, 0.0)  # gfx950 FETCH_SIZE correction (x2)
        wb = write.get(k, 0.0)
        tj[f"{wl}:{n_nodes}:{k}"] = {"hbm_bytes_per_launch": fb + wb, "fetch_bytes_per_launch": fb,
                                     "write_bytes_per_launch": wb, "source": os.path.basename(prof.rstrip("/")),
                                     "round": os.environ.get("KSG_ROUND", ""), "kernel_src_sha": kernel_src_sha(),
                                     "note": "FETCH_SIZE KiB x1024 x2 (gfx950, calibrated: profiles/r3_fetch_calib.json) + WRITE_SIZE KiB x1024, mean per launch"}
        print(k, tj[f"{wl}:{n_nodes}:{k}"])
    with open(out, "w") as f:
        json.dump(tj, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
