"""Fill a recorded bench line's counter-measured fields from profiles/traffic.json after the run.

A record run measures the bench lines before its PMC passes exist (tools/gpu_record.sh: bench
steps, then prof steps), so those lines carry `roofline.traffic: null`. This recomputes, exactly as
bench.py does, `roofline.traffic`, `roofline.win_eval_traffic(_GBps)`, `filter_score` (its basis
becomes the counter bytes) and `roofline.traffic_source` from the entries measured on the same
kernel sources (kernel_src_sha must equal the line's own), and marks the line
`traffic_filled_after_run`. Nothing else in the line changes.

usage: python tools/fill_traffic.py <bench.json> [out.json] [profiles/traffic.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import HBM_PEAK, traffic_entry  # noqa: E402


def fill(d, tj):
    r = d["roofline"]
    ts = r.get("traffic_source") or {}
    sha = ts.get("kernel_src_sha")
    wl = d["config"]["workload"].split(":")[0]
    nn = d["config"]["nodes"]
    stale = []
    ent = traffic_entry(tj, f"{wl}:{nn}:{r['kernel']}", sha, stale)
    if ent:
        r["traffic"] = ent["hbm_bytes_per_launch"]
        ts["resolver"] = {"source": ent["source"], "round": ent["round"]}
    fs = d.get("filter_score")
    fent = traffic_entry(tj, f"{wl}:{nn}:ksg_win_score_kernel", sha, stale)
    if fent and fs:
        ev_s = fs["ms_avg"] / 1e3
        r["win_eval_traffic"] = fent["hbm_bytes_per_launch"]
        r["win_eval_traffic_GBps"] = fent["hbm_bytes_per_launch"] / ev_s / 1e9
        fs.update({"basis": "pmc_traffic", "bytes_per_launch": fent["hbm_bytes_per_launch"],
                   "achieved": fent["hbm_bytes_per_launch"] / ev_s / 1e9,
                   "frac": fent["hbm_bytes_per_launch"] / ev_s / HBM_PEAK})
        r["filter_score_frac"] = fs["frac"]
        ts["filter_score"] = {"source": fent["source"], "round": fent["round"]}
    ts["stale"] = stale
    r["traffic_source"] = ts
    d["traffic_filled_after_run"] = "profiles/traffic.json entries of the same kernel sources (tools/fill_traffic.py)"
    return d


def main():
    src = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else src
    tjp = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "traffic.json")
    d = json.loads(open(src).read().strip().splitlines()[-1])
    with open(tjp) as f:
        tj = json.load(f)
    d = fill(d, tj)
    with open(out, "w") as f:
        f.write(json.dumps(d) + "\n")
    print(out, d["roofline"].get("traffic"), (d.get("filter_score") or {}).get("basis"))


if __name__ == "__main__":
    main()
