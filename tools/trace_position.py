"""Per-position kernel durations inside a frame, from a rocprofv3 kernel-trace CSV.

A frame starts at every dispatch of the marker kernel (default: the talker gate-up GEMV, grid 196608 x wg 256);
for each target (kernel-name prefix, grid X, workgroup X) print the mean duration of its k-th dispatch after the
marker. Cold-vs-resident weights show up as a slow first code-predictor step followed by faster later steps.
usage: python3 tools/trace_position.py <kernel_trace.csv> [out.txt]"""
import collections
import csv
import sys

MARK = ("gemv_wt", "196608", "256")
TARGETS = [("gemv_wt", "196608", "512", "cp gate-up"), ("gemv_wt", "32768", "512", "cp down"),
           ("gemv_wt", "131072", "512", "cp qkv / lm_head"), ("attn_oproj_k", "131072", "512", "cp attn_oproj"),
           ("sample_k", "2048", "256", "sample")]


def key(r):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    return n, r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Workgroup_Size_X", "")


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    pos = collections.defaultdict(lambda: collections.defaultdict(list))
    cnt = None
    for r in rows:
        n, g, w = key(r)
        if n.startswith(MARK[0]) and g == MARK[1] and w == MARK[2]:
            cnt = collections.Counter()
            continue
        if cnt is None:
            continue
        for t in TARGETS:
            if n.startswith(t[0]) and g == t[1] and w == t[2]:
                k = cnt[t[3]]
                cnt[t[3]] += 1
                pos[t[3]][k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    for t in TARGETS:
        d = pos[t[3]]
        if not d:
            continue
        out.write(f"{t[3]}: mean us by dispatch index after the talker gate-up (n per index)\n")
        line = []
        for k in sorted(d):
            v = d[k]
            if len(v) < 20:
                continue
            line.append(f"{k}:{sum(v) / len(v):.2f}")
        for i in range(0, len(line), 10):
            out.write("  " + " ".join(line[i:i + 10]) + "\n")


if __name__ == "__main__":
    main()
