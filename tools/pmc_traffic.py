"""Turn a tools/pmc2.sh summary (tools/pmc_summary.py output) into
profiles/pmc_summary.json, which bench.py reads as roofline.traffic: HBM
bytes per aggregate launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB (the
gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md "HBM", re-checked in
profiles/r01_fetch_calibration.txt).  usage:
  python3 tools/pmc_traffic.py <summary.json> <bytes_per_launch> [kernel] [out]"""
import json
import sys


def main(src, bpl, kernel="tile_kernel", out="profiles/pmc_summary.json", workload="cfg2",
         tracked=None):
    """tracked: the committed copy of `src` under profiles/ (the line's
    traffic_source names it; gpurun_out/ is scratch)."""
    allc = json.load(open(src))["counters"]
    if tracked:
        import shutil
        shutil.copyfile(src, tracked)
        src = tracked
    d = allc[kernel]
    hbm = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    res = {"kernel": kernel, "workload": workload, "bytes_per_launch": int(bpl),
           "hbm_bytes_per_launch": hbm,
           "read_bytes": 2 * d["FETCH_SIZE"] * 1024, "write_bytes": d["WRITE_SIZE"] * 1024,
           "ratio_to_algorithmic": hbm / int(bpl),
           "counters": d, "source": src}
    p = allc.get("partition_kernel")
    if p and "FETCH_SIZE" in p:
        res["partition_hbm_bytes_per_launch"] = (2 * p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024
        res["step_ratio_to_algorithmic"] = (hbm + res["partition_hbm_bytes_per_launch"]) / int(bpl)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
