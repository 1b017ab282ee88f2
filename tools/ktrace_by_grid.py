#!/usr/bin/env python3
"""Per-(kernel, grid size) launch statistics from a rocprofv3 kernel trace.

`rocprofv3 --stats` averages every launch of a kernel together; a bench run
launches the same kernel at several sizes (the headline batch, the cfg5
shards, the launch-floor plan), so its average is not the headline
launch's. This groups `*_kernel_trace.csv` by kernel name and grid size.

usage: ktrace_by_grid.py TRACE.csv [NAME_SUBSTRING ...]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    pats = sys.argv[2:]
    groups = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        if pats and not any(p in name for p in pats):
            continue
        grid = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
        wg = int(row["Workgroup_Size_X"]) * int(row["Workgroup_Size_Y"]) * int(row["Workgroup_Size_Z"])
        dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        groups[(name, grid, wg)].append(dur)
    print(f"{'kernel':<72} {'grid':>10} {'wg':>4} {'calls':>5} {'avg_us':>9} {'min_us':>9} {'max_us':>9}")
    for (name, grid, wg), v in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        short = name if len(name) <= 72 else name[:69] + "..."
        print(f"{short:<72} {grid:>10} {wg:>4} {len(v):>5} {sum(v) / len(v) / 1e3:>9.1f} "
              f"{min(v) / 1e3:>9.1f} {max(v) / 1e3:>9.1f}")


if __name__ == "__main__":
    main()
