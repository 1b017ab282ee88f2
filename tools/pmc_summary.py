"""Summarise rocprofv3 CSV output of tools/pmc2.sh: per-kernel mean duration
and mean counter values per dispatch (HBM bytes with the gfx950 FETCH_SIZE
x2 correction of MI355X_MICROARCH.md "HBM")."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def short(name):
    for k in ("cm_ibin_kernel", "cm_transpose_kernel", "cm_iapply_kernel", "cm_qbin_kernel",
              "cm_qlook_kernel", "cm_qkeep_kernel", "cm_bin_count", "cm_bin_scan", "cm_bin_scatter", "cm_bin_apply", "nw_tile_kernel",
              "nw_gather", "nw_bucket", "nw_split", "nw_rank", "cursor_kernel", "tile_packed_kernel", "tile_kernel", "splitter_kernel", "partition_kernel",
              "unmatched_kernel", "gather_kernel", "union", "slice_kernel", "crc_kernel",
              "darling_kernel", "cm_insert", "cm_count", "cm_scan", "cm_scatter",
              "snappy_lit_kernel", "snappy_kernel", "nw_tile_kernel", "nw_cand", "nw_seg",
              "dense_kernel"):
        if k in name:
            return k
    return None


def main(out):
    res = {"kernels": {}, "counters": {}}
    dur = defaultdict(list)
    for r in rows(os.path.join(out, "p1", "**", "*kernel_trace.csv")):
        k = short(r.get("Kernel_Name", ""))
        if k:
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, v in dur.items():
        res["kernels"][k] = {"dispatches": len(v), "mean_us": sum(v) / len(v) / 1e3}
    cnt = defaultdict(lambda: defaultdict(list))
    for r in rows(os.path.join(out, "p*", "**", "*counter_collection.csv")):
        k = short(r.get("Kernel_Name", ""))
        if k:
            cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in cnt.items():
        res["counters"][k] = {c: sum(v) / len(v) for c, v in d.items()}
    for k, d in res["counters"].items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_corrected"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
