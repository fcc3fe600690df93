"""One decode frame's kernel sequence from a rocprofv3 --kernel-trace CSV of tools/frame_trace.py: the frames are
the repeats of the sequence that starts at each qt_cp_prefill launch (cp_step_k<1, 1>); prints, for the median
frame of the last generate, every kernel with its duration and the gap to the previous kernel's end, and totals.
    python tools/frame_trace_reduce.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict


def short(n):
    for k in ("cp_step_k<1, 1>", "cp_step_k<1, 0>", "talker_tail_k", "attn_decode_k", "gemv_wt", "sample_k",
              "frame_embed_k", "rmsnorm", "advance_rows", "gemm"):
        if k in n:
            return k
    return n.split("(")[0].replace("void ", "")[-40:]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "cp_step_k<1, 1>" in r[2]]
    frames = [rows[a:b] for a, b in zip(starts, starts[1:])]
    frames = frames[-20:-2]  # the last generate's steady frames
    tot = sorted(((f[-1][1] - f[0][0]) for f in frames))
    med = frames[[f[-1][1] - f[0][0] for f in frames].index(tot[len(tot) // 2])]
    t0 = med[0][0]
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    prev_end = None
    print(f"median frame: {(med[-1][1] - t0) / 1e3:.1f} us over {len(med)} kernels (of {len(frames)} frames: "
          f"{tot[0] / 1e3:.1f} .. {tot[-1] / 1e3:.1f})")
    for s, e, n in med:
        k = short(n)
        gap = 0.0 if prev_end is None else (s - prev_end) / 1e3
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
        agg[k][2] += gap
        prev_end = e
    busy = sum(v[1] for v in agg.values())
    gaps = sum(v[2] for v in agg.values())
    print(f"kernel time {busy:.1f} us, gaps {gaps:.1f} us")
    for k, (c, d, g) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {k:40s} x{c:3d}  {d:8.1f} us  ({d / c:6.2f} each)  gaps before {g:7.1f} us")


if __name__ == "__main__":
    main()
