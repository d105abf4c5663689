"""Per-cycle timeline of the IB band cycle from a rocprofv3 trace directory: kernels of the last
cycles (start/end relative to the cycle's deep sweep, queue) and the host API time per cycle."""
import csv, glob, re, statistics, sys


def short(n):
    n = n.split("(")[0]
    if "sweepk_kernel" in n and re.search(r",\s*true\s*(,\s*\d+\s*)?>", n):
        return "sweep_slab"  # the boundary sweeps of an RCCL slab
    for k in ("sweepk_kernel", "fused_kernel", "band_level_kernel", "ib_point_kernel", "ib_ghost_kernel", "copyBuffer", "nccl",
              "Copy"):
        if k in n:
            return k
    return n[-30:]


def main(d):
    kt = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in kt)
    deep = [e for e in ev if e[2] == "sweepk_kernel"]
    per = [(b[0] - a[0]) / 1e3 for a, b in zip(deep[-60:], deep[-59:])]
    print(f"cycle (deep start to start): median {statistics.median(per):.1f} us")
    win = [e for e in ev if deep[-51][0] <= e[0] < deep[-1][0]]
    kinds = {}
    for s_, e_, k_, q_ in win:
        kinds.setdefault(k_, []).append((e_ - s_) / 1e3)
    print("  median duration per kind over the last 50 cycles: " +
          ", ".join(f"{k_} {statistics.median(v):.1f} us (x{len(v) / 50:.1f})" for k_, v in sorted(kinds.items())))
    t0 = deep[-4][0]
    for s, e, k, q in ev:
        if deep[-4][0] - 20000 <= s <= deep[-2][0]:
            print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {k}")
    hs = glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)
    if hs:
        api = list(csv.DictReader(open(hs[0])))
        a0, a1 = deep[-51][0], deep[-1][0]
        tot = {}
        for r in api:
            s = int(r["Start_Timestamp"])
            if a0 <= s <= a1:
                tot[r["Function"]] = tot.get(r["Function"], 0) + (int(r["End_Timestamp"]) - s) / 1e3
        print("  host API us per cycle:", ", ".join(f"{k} {v / 50:.1f}" for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:8]))


if __name__ == "__main__":
    main(sys.argv[1])
