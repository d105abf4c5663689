#!/usr/bin/env python3
"""Is a cycle bound by the host's submission?  Reads a rocprofv3 directory written with
--kernel-trace --hip-runtime-trace and prints, for the last N dispatches of the named kernels, the
time from the end of the launching HIP call to the kernel's start (lag: small = the kernel waited
for the host), and the period of consecutive launch calls on the host against the period of the
kernels on the GPU (equal periods with small lags = host bound).

usage: scripts/submit_lag.py TRACE_DIR [--kernel sweepk_kernel] [--last 50]
"""
import argparse
import csv
import glob
import os
import statistics as st


def rows(d, suffix):
    fs = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not fs:
        raise SystemExit(f"no *{suffix} under {d}")
    with open(fs[0]) as f:
        return list(csv.DictReader(f))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--kernel", action="append", default=None)
    p.add_argument("--last", type=int, default=50)
    a = p.parse_args()
    names = a.kernel or ["sweepk_kernel", "band_level_kernel", "rcclGenericKernel"]
    ks = rows(a.trace, "kernel_trace.csv")
    api = {r["Correlation_Id"]: r for r in rows(a.trace, "hip_api_trace.csv")}
    for name in names:
        sel = [k for k in ks if name in k["Kernel_Name"]]
        sel.sort(key=lambda k: int(k["Start_Timestamp"]))
        sel = sel[-a.last:]
        lag, hp, gp, calls = [], [], [], []
        prev = None
        for k in sel:
            r = api.get(k["Correlation_Id"])
            if r is None:
                continue
            ks0, ae = int(k["Start_Timestamp"]), int(r["End_Timestamp"])
            lag.append((ks0 - ae) / 1e3)
            calls.append(r["Function"])
            if prev is not None:
                hp.append((int(r["Start_Timestamp"]) - prev[0]) / 1e3)
                gp.append((ks0 - prev[1]) / 1e3)
            prev = (int(r["Start_Timestamp"]), ks0)
        if not lag:
            print(f"{name}: no dispatches with a HIP call")
            continue
        print(f"{name}: {len(lag)} dispatches ({calls[-1]}); launch call end -> kernel start: median "
              f"{st.median(lag):.1f} us, min {min(lag):.1f}, max {max(lag):.1f}")
        if hp:
            print(f"  period between launches: host {st.median(hp):.1f} us, GPU {st.median(gp):.1f} us (medians)")
    # the host thread's busiest calls over the window of the last dispatches
    if ks:
        t0 = int(sorted(ks, key=lambda k: int(k["Start_Timestamp"]))[-min(len(ks), 20 * a.last)]["Start_Timestamp"])
        tot = {}
        for r in api.values():
            if int(r["Start_Timestamp"]) >= t0:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                n, s = tot.get(r["Function"], (0, 0.0))
                tot[r["Function"]] = (n + 1, s + d)
        t1 = max(int(k["End_Timestamp"]) for k in ks)
        print(f"host time in HIP calls over the window of {(t1 - t0) / 1e3:.0f} us:")
        for f, (n, s) in sorted(tot.items(), key=lambda x: -x[1][1])[:12]:
            print(f"  {f:40s} {n:6d} calls {s:10.1f} us  {s / n:7.2f} us/call")


if __name__ == "__main__":
    main()
