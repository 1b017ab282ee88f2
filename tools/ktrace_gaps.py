#!/usr/bin/env python3
"""MEASUREMENT AID: the timeline of the last N launches of a rocprofv3 kernel
trace -- each kernel's duration and the gap to the next one's start (a
negative gap = the next kernel started before this one ended).

usage: ktrace_gaps.py TRACE.csv [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "psg::" in r["Kernel_Name"]][-n:]
    dur = {}
    gaps = {}
    for a, b in zip(rows, rows[1:]):
        ka = a["Kernel_Name"].split("(")[0].split("::")[-1][:28]
        d = (int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        dur.setdefault(ka, []).append(d)
        gaps.setdefault(ka, []).append(g)
        print(f"{ka:28s} {d:9.2f} us   gap to next {g:8.2f} us")
    for k in dur:
        print(f"mean {k:28s} {sum(dur[k]) / len(dur[k]):9.2f} us   gap {sum(gaps[k]) / len(gaps[k]):8.2f} us")


if __name__ == "__main__":
    main()
