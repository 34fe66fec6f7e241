"""Fold one record run (tools/gpu_record.sh <tag> prof / bench / sq, tools/gpu_dropin.sh) from
gpurun_out/ into profiles/: the PMC passes into profiles/traffic.json (round and source sha
tags, tools/traffic_from_pmc.py), the bench lines, kernel-trace stats, SQ fractions
(tools/sq_summary.py) and drop-in records under profiles/<round>_*; prints the table rows.
usage: python tools/collect_record.py <tag> [round=r6]"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
WLS = ("config1", "config2", "config3", "config4", "config5")


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main(tag, rnd="r6"):
    env = dict(os.environ, KSG_ROUND=rnd)
    for wl in WLS:
        d = os.path.join(OUT, f"prof_{tag}_{wl}")
        if not os.path.isdir(d):
            continue
        nn = last_json(os.path.join(d, "bench_kt.json"))["config"]["nodes"]
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_from_pmc.py"), d, wl, str(nn),
                        os.path.join(PROF, "traffic.json")], check=True, env=env, stdout=subprocess.DEVNULL)
        ks = sorted(glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True))
        if ks:
            shutil.copy(ks[0], os.path.join(PROF, f"{rnd}_{wl}_kernel_stats.csv"))
    rows = []
    for wl, src in [(w, f"{tag}_bench_{w}.json") for w in WLS] + [("config2_extensions", f"{tag}x_bench_config2.json")]:
        p = os.path.join(OUT, src)
        if not os.path.exists(p):
            continue
        d = last_json(p)
        with open(os.path.join(PROF, f"{rnd}_bench_{wl}_1gpu.json"), "w") as f:
            f.write(json.dumps(d) + "\n")
        lat = d.get("latency") or {}
        cb = d.get("cpu_baseline") or {}
        rows.append((wl, round(d["value"]), round(lat.get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"], 2),
                     round(d.get("device_ms_per_step") or 0, 2), round(d["roofline"]["frac"], 4), d["roofline"].get("traffic"),
                     round((d.get("filter_score") or {}).get("frac") or 0, 4), round(cb.get("value") or 0),
                     round((cb.get("incremental") or {}).get("value") or 0),
                     round((cb.get("incremental_nproc") or {}).get("value") or 0)))
    for wl in ("config2", "config5"):
        c = os.path.join(OUT, f"sq_{tag}_{wl}", "run_counter_collection.csv")
        if os.path.exists(c):
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), c,
                            os.path.join(PROF, f"{rnd}_sq_{wl}.json"),
                            f"rocprofv3 --pmc (8 SQ counters), bench.py --workload {wl} --steps 3 --warmup 1, record run {tag}"],
                           check=True, stdout=subprocess.DEVNULL)
    dj = os.path.join(OUT, f"{tag}_dropin.jsonl")
    if os.path.exists(dj):
        shutil.copy(dj, os.path.join(PROF, f"{rnd}_dropin.jsonl"))
        for line in open(dj):
            d = json.loads(line)
            print("dropin", d["nodes"], "policy", d.get("policy", 0), "ext", d.get("ext", 0), "p50", d["us_p50"],
                  "p99", d["us_p99"], round(d["pods_per_s"]))
    for r in rows:
        print(*r)


if __name__ == "__main__":
    main(*sys.argv[1:])
