"""Fold one rocprofv3 SQ counter pass (tools/gpu_record.sh sq) into per-kernel fractions.

Each dispatch's counters are summed per kernel; the fractions are of SQ_WAVE_CYCLES (the
wave-resident quad-cycles; ACTIVE_INST_ANY + WAIT_ANY + WAIT_INST_ANY ~ WAVE_CYCLES, disjoint,
MI355X_MICROARCH.md PMC table):
  valu   SQ_ACTIVE_INST_VALU / WAVE_CYCLES   a wave issuing vector ALU work
  salu   SQ_ACTIVE_INST_SCA  / WAVE_CYCLES   ... scalar ALU work
  issue  SQ_ACTIVE_INST_ANY  / WAVE_CYCLES   ... any instruction
  wait   SQ_WAIT_ANY         / WAVE_CYCLES   parked on s_waitcnt / barrier / s_sleep
  stall  SQ_WAIT_INST_ANY    / WAVE_CYCLES   ready, but its instruction could not issue
and busy = SQ_BUSY_CYCLES per dispatch (quad-cycles, summed over the SEs).
usage: python tools/sq_summary.py <run_counter_collection.csv> <out.json> [label]"""
import csv
import json
import sys
from collections import defaultdict


def summarize(path):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        if not name.startswith(("ksg_", "void ksg_")):
            continue
        name = name.replace("void ", "")
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    out = {}
    for k, c in per.items():
        n = len(disp[k])
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        out[k] = {
            "dispatches": n,
            "waves_per_dispatch": c.get("SQ_WAVES", 0.0) / n,
            "wave_cycles_per_dispatch": c.get("SQ_WAVE_CYCLES", 0.0) / n,
            "busy_cycles_per_dispatch": c.get("SQ_BUSY_CYCLES", 0.0) / n,
            "valu": c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
            "salu": c.get("SQ_ACTIVE_INST_SCA", 0.0) / wc,
            "issue": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "wait": c.get("SQ_WAIT_ANY", 0.0) / wc,
            "stall": c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
        }
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    doc = {"source": sys.argv[3] if len(sys.argv) > 3 else sys.argv[1], "units": "fractions of SQ_WAVE_CYCLES",
           "kernels": res}
    json.dump(doc, open(sys.argv[2], "w"), indent=1)
    for k, v in res.items():
        print(k, {a: round(b, 3) if isinstance(b, float) else b for a, b in v.items()})
