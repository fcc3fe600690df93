"""Reduce a rocprofv3 --stats kernel CSV to one kernel's average duration, labelled with the build it was measured
on (for bench.py's roofline: profiles/<tag>_rocprof_<kernel tag>.json).
    python tools/rocprof_kernel_avg.py <run_kernel_stats.csv> <kernel substring> <build id>"""
import csv
import json
import sys


def main():
    path, sub, bid = sys.argv[1], sys.argv[2], sys.argv[3]
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Name"]]
    calls = sum(int(r["Calls"]) for r in rows)
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    print(json.dumps({"kernel_substring": sub, "build_id": bid, "calls": calls, "avg_us": round(total_ns / calls / 1e3, 3),
                      "source": path}, indent=1))


if __name__ == "__main__":
    main()
