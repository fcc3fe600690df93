"""Reduce rocprofv3 --pmc CSV directories (one pass each) to per-dispatch averages of every counter for kernels whose
name contains a substring.

    python tools/pmc_kernel_reduce.py <kernel-substring> <meta-file> <pass-dir> [<pass-dir> ...]

meta-file: "<build id> <algorithmic bytes per launch> ..." (written by the launch script).  FETCH_SIZE is doubled
(gfx950 counts half the bytes of wide coalesced reads, MI355X_MICROARCH.md HBM section); WRITE_SIZE is exact;
both are KiB.  The L2 -> CU request count (TCP_TCC_READ_REQ_sum, 64-B requests on gfx950 -- uncalibrated for other
widths) is reported as bytes too, next to the algorithmic bytes, to show re-reads inside the chip."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    sub, meta = sys.argv[1], open(sys.argv[2]).read().split()
    bid, algo = meta[0], int(meta[1])
    vals = defaultdict(list)
    for d in sys.argv[3:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if sub in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"kernel_substring": sub, "build_id": bid, "algorithmic_bytes_per_launch": algo,
           "dispatches": {k: len(v) for k, v in vals.items()}, "counters_avg_per_dispatch": avg}
    if "FETCH_SIZE" in avg:
        out["hbm_read_bytes"] = int(2 * avg["FETCH_SIZE"] * 1024)
    if "WRITE_SIZE" in avg:
        out["hbm_write_bytes"] = int(avg["WRITE_SIZE"] * 1024)
    if "hbm_read_bytes" in out and "hbm_write_bytes" in out:
        out["hbm_bytes_per_launch"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
        out["traffic_over_algorithmic"] = round(out["hbm_bytes_per_launch"] / algo, 4)
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        out["l2_hit_rate"] = round(avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]), 4)
    if "TCP_TCC_READ_REQ_sum" in avg:
        out["l2_to_cu_read_bytes_64B_req"] = int(64 * avg["TCP_TCC_READ_REQ_sum"])
        out["l2_to_cu_over_algorithmic"] = round(64 * avg["TCP_TCC_READ_REQ_sum"] / algo, 2)
    out["correction"] = ("hbm = 2 x FETCH_SIZE(KiB) x 1024 + WRITE_SIZE(KiB) x 1024 (gfx950 FETCH_SIZE half-count); "
                         "L2->CU = 64 B x TCP_TCC_READ_REQ")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
