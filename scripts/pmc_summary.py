#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE collected in separate runs) into
HBM bytes per launch of the collide-stream kernel, corrected as MI355X_MICROARCH.md §HBM says:
FETCH_SIZE (KiB) reports half the bytes of a wide coalesced streaming read on gfx950 -> x2;
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores.

usage: pmc_summary.py KEY FETCH_DIR WRITE_DIR OUT_JSON [--kernel fused_kernel]
"""
import csv
import glob
import json
import os
import sys


def counter_mean(d, counter, kernel):
    vals = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if counter in row.get("Counter_Name", "") and kernel in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    vals = vals[2:] if len(vals) > 4 else vals  # drop the first launches (cold caches)
    return sum(vals) / len(vals), len(vals)


def main():
    key, fdir, wdir, out = sys.argv[1:5]
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "fused_kernel"
    fetch_kib, nf = counter_mean(fdir, "FETCH_SIZE", kernel)
    write_kib, nw = counter_mean(wdir, "WRITE_SIZE", kernel)
    hbm = (2.0 * fetch_kib + write_kib) * 1024.0
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[key] = {"hbm_bytes_per_launch": hbm, "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
              "fetch_bytes_corrected": 2.0 * fetch_kib * 1024.0, "write_bytes": write_kib * 1024.0,
              "launches": [nf, nw], "kernel": kernel,
              "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); FETCH_SIZE x2 (gfx950)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d[key]))


if __name__ == "__main__":
    main()
