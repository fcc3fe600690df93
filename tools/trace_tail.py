"""Print the last N kernels of a rocprofv3 kernel-trace CSV in launch order (duration, grid, gap to the previous)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
prev = None
tot = 0.0
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:80]
    grid = f'{r.get("Grid_Size_X", "?")}x{r.get("Grid_Size_Y", "")}x{r.get("Grid_Size_Z", "")}'
    gap = (s - prev) / 1e3 if prev else 0.0
    tot += (e - s) / 1e3
    print(f"{(e - s) / 1e3:8.2f} us  gap {gap:7.2f}  grid={grid:16s} {name}")
    prev = e
print(f"busy {tot:.1f} us, span {(int(rows[-1]['End_Timestamp']) - int(rows[-n]['Start_Timestamp'])) / 1e3:.1f} us")
