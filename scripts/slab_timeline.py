"""Per-cycle kernel timeline of a slab run from a rocprofv3 kernel-trace CSV directory.

Prints per kernel kind (interior sweep, boundary sweep, pack, RCCL, other) the mean duration over
the last 100 cycles and the mean gap between consecutive interior sweeps (the cycle time)."""
import csv, glob, re, statistics, sys


def grid_threads(r):
    for k in ("Grid_Size", "Grid_Size_X", "Grid_SizeX"):
        if k in r and r[k]:
            return int(r[k])
    return 0


def kind(name, r=None):
    if "sweepk_kernel" in name:  # sweepk_kernel<T, VS, MODE, K, SLAB[, WPE]>: SLAB = the boundary sweeps,
        # or (round 5, the edge flag) a ghost-column interior: told apart by the grid (>= 64 workgroups)
        if r is not None and grid_threads(r) >= 64 * 256:
            return "sweep"
        return "sweep_slab" if re.search(r",\s*true\s*(,\s*\d+\s*)?>", name) else "sweep"
    if "pack" in name:
        return "pack"
    if "nccl" in name.lower():
        return "rccl"
    return name.split("(")[0][-40:]


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"], r)) for r in rows)
    ints = [e for e in ev if e[2] == "sweep"]
    if len(ints) < 50:  # lone slab: every sweep is a SLAB=false launch
        ints = [e for e in ev if e[2].startswith("sweep")]
    # the timed steps are the last ones: take the last 100 interior sweeps
    ints = ints[-100:]
    t0, t1 = ints[0][0], ints[-1][1]
    win = [e for e in ev if t0 <= e[0] <= t1]
    by = {}
    for s, e, k in win:
        by.setdefault(k, []).append((e - s) / 1e3)
    period = statistics.mean((b[0] - a[0]) / 1e3 for a, b in zip(ints, ints[1:]))
    print(f"cycle (interior start to start) {period:.2f} us over {len(ints)} cycles")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:30s} n={len(v):5d} mean {statistics.mean(v):8.2f} us  per cycle {sum(v) / len(ints):8.2f} us")
    # critical path hints: idle gap on the compute stream between interior sweeps
    gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(ints, ints[1:])]
    print(f"  gap between interior sweeps: mean {statistics.mean(gaps):.2f} us, median {statistics.median(gaps):.2f} us, "
          f"max {max(gaps):.2f} us")




def host_lag(d):
    """With a --hip-trace: for each interior sweep, when its launch call returned on the host
    relative to the end of the previous interior sweep (positive: the GPU waited for the host)."""
    kt = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    hs = glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)
    if not hs:
        return
    api = {r["Correlation_Id"]: r for r in csv.DictReader(open(hs[0]))}
    ints = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Correlation_Id"]) for r in kt
                  if kind(r["Kernel_Name"], r) == "sweep")[-100:]
    lags, starts = [], []
    for a, b in zip(ints, ints[1:]):
        h = api.get(b[2])
        if h is None:
            continue
        lags.append((int(h["End_Timestamp"]) - a[1]) / 1e3)
        starts.append((b[0] - max(a[1], int(h["End_Timestamp"]))) / 1e3)
    if lags:
        lags.sort()
        print(f"  launch call returned vs previous interior end: median {lags[len(lags) // 2]:.2f} us "
              f"(>0 in {sum(l > 0 for l in lags)} of {len(lags)})")
        starts.sort()
        print(f"  interior start after max(prev end, launch call): median {starts[len(starts) // 2]:.2f} us")
    per = {}
    t0, t1 = ints[0][0], ints[-1][1]
    for r in api.values():
        s = int(r["Start_Timestamp"])
        if t0 <= s <= t1:
            per.setdefault(r["Function"], []).append((int(r["End_Timestamp"]) - s) / 1e3)
    print("  host API time per cycle:", ", ".join(f"{k} {sum(v) / len(ints):.1f}" for k, v in
                                               sorted(per.items(), key=lambda kv: -sum(kv[1]))[:8]))


if __name__ == "__main__":
    main(sys.argv[1])
    host_lag(sys.argv[1])
