"""Summarise a rocprofv3 kernel-trace CSV by (kernel, grid size): calls, mean/total duration.
Run on the GPU box next to the trace (the raw trace is too large to bring back)."""
import collections
import csv
import sys

rows = csv.DictReader(open(sys.argv[1]))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r["Kernel_Name"]
    name = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
    if "<" in r["Kernel_Name"]:
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:70]
    grid = f'{r.get("Grid_Size_X", r.get("Grid_Size", "?"))}x{r.get("Grid_Size_Y", "")}'
    key = (name, grid, r.get("Workgroup_Size_X", ""))
    d = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    agg[key][0] += 1
    agg[key][1] += d
tot = sum(v[1] for v in agg.values())
out = sorted(agg.items(), key=lambda kv: -kv[1][1])
with open(sys.argv[2], "w") as f:
    f.write(f"total_ms {tot / 1e6:.2f}\n")
    for (name, grid, wg), (n, t) in out[:60]:
        f.write(f"{t / 1e6:9.2f} ms {100 * t / tot:5.1f}% n={n:7d} avg={t / n / 1e3:8.2f}us grid={grid} wg={wg} {name}\n")
