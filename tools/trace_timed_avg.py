"""Mean duration of one kernel over the last K launches of a rocprofv3 kernel trace.

The `--stats` summary averages every launch (warm-up steps included); bench.py's
`roofline.kernel_ms_avg` covers only the timed region's `roofline.launches`
launches. This takes the same last-K slice of the trace so the two can be compared.

usage: tools/trace_timed_avg.py <run_kernel_trace.csv> <kernel substring> <K>
"""
import csv
import sys


def main():
    path, name, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    last = dur[-k:]
    print(f"{name}: {len(dur)} launches, mean {sum(dur) / len(dur):.1f} us; "
          f"last {len(last)} mean {sum(last) / len(last):.1f} us")


if __name__ == "__main__":
    main()
