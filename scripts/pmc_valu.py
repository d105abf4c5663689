#!/usr/bin/env python3
"""Summarise rocprofv3 SQ passes of the deep-sweep kernel into VALU figures per launch:
FP64/FP32 FLOPs (SQ_INSTS_VALU_FLOPS_* counts per wave instruction; x64 lanes), VALU
instructions, and the share of wave cycles that issue VALU (SQ_ACTIVE_INST_VALU /
SQ_WAVE_CYCLES, both in quad-cycles).  Writes profiles/pmc_valu.json (read by bench.py).

usage: pmc_valu.py KEY FLOPS_CSV [SQ_CSV] [--kernel sweepk_kernel]
"""
import csv
import json
import os
import sys
from collections import defaultdict

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_valu.json")


def means(path, kernel):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v[2:]) / len(v[2:]) if len(v) > 4 else sum(v) / len(v) for k, v in acc.items()}


def main():
    key, flops_csv = sys.argv[1:3]
    sq_csv = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else None
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "sweepk_kernel"
    m = means(flops_csv, kernel)
    if sq_csv:
        m.update({k: v for k, v in means(sq_csv, kernel).items() if k not in m})
    fp = "SQ_INSTS_VALU_FLOPS_FP64" if "SQ_INSTS_VALU_FLOPS_FP64" in m else "SQ_INSTS_VALU_FLOPS_FP32"
    e = {"flops_per_launch": m[fp] * 64, "flops_counter": fp, "valu_insts_per_launch": m.get("SQ_INSTS_VALU"),
         "waves_per_launch": m.get("SQ_WAVES"),
         "valu_issue_share": (m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]) if "SQ_WAVE_CYCLES" in m else None,
         "source": "rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_* (x64 lanes), SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES"}
    d = json.load(open(OUT)) if os.path.exists(OUT) else {}
    d[key] = e
    json.dump(d, open(OUT, "w"), indent=1)
    print(json.dumps(e))


if __name__ == "__main__":
    main()
