#!/usr/bin/env python3
"""A/B the collide-stream kernel variants (one-step fused_kernel and the two-iteration sweep,
IBLB_SWEEP*) in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Each variant gets its own context (IBLB_FUSED_VARIANT
and IBLB_PLANE_PAD are read at iblb_create); results must be bit-identical across variants.

usage: tune_fused.py [--nx 4096 --ny 4096 --precision f64 --steps 100 --rounds 5]
                     [--variants 0,1,2,...] [--pads p1,p2]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--ny", type=int, default=4096)
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--pads", default="")
    ap.add_argument("--gaps", default="", help="IBLB_BUF_GAP values, crossed with --pads")
    ap.add_argument("--envs", default="", help="';'-separated environment sets, e.g. "
                    "'IBLB_FUSED_VARIANT=5;IBLB_FUSED_VARIANT=5 IBLB_LAYOUT=1 IBLB_COL_PAD=64' (overrides the rest)")
    a = ap.parse_args()
    import cuda_iblb_11_amd as P
    from cuda_iblb_11_amd import workloads as W
    rho, u = W.perturbed_state(a.nx, a.ny, W.SEED)
    combos = [(int(v), None, None) for v in a.variants.split(",")]
    if a.pads:
        gaps = [int(g) for g in a.gaps.split(",")] if a.gaps else [None]
        combos = [(int(v), int(p), g) for v in a.variants.split(",") for p in a.pads.split(",") for g in gaps]
    sets = []
    for v, pad, gap in combos:
        e = {"IBLB_FUSED_VARIANT": str(v)}
        if pad is not None:
            e["IBLB_PLANE_PAD"] = str(pad)
        if gap is not None:
            e["IBLB_BUF_GAP"] = str(gap)
        sets.append(((v, pad, gap), e))
    if a.envs:
        sets = []
        for grp in a.envs.split(";"):
            e = dict(kv.split("=") for kv in grp.split())
            sets.append((grp, e))
    names = sorted({k for _, e in sets for k in e} | {"IBLB_FUSED_VARIANT", "IBLB_PLANE_PAD", "IBLB_BUF_GAP",
                                                     "IBLB_SWEEP", "IBLB_SWEEP_W", "IBLB_SWEEP_VS", "IBLB_SWEEP_VARIANT",
                                                     "IBLB_SWEEP_DEPTH",
                                                     "IBLB_DEEP_W", "IBLB_DEEP_VS", "IBLB_DEEP_VARIANT", "IBLB_DEEP_BALANCE"})
    ctxs = []
    for key, e in sets:
        for name in names:
            os.environ.pop(name, None)
        os.environ.update(e)
        lat = P.Lattice(a.nx, a.ny, W.TAU, W.TAU2, precision=a.precision, body_force=W.BODY_FORCE)
        lat.set_state(rho, u)
        lat.step(10)
        lat.set_profiling(True)
        ctxs.append((key, lat))
    for name in names:
        os.environ.pop(name, None)
    res = {k: [] for k, _ in ctxs}
    for r in range(a.rounds):
        for k, lat in ctxs:
            lat.timing(reset=True)
            lat.step(a.steps)
            t = lat.timing(reset=True)
            # time per iteration: one-step launches count once, two-iteration sweeps twice
            res[k].append((t["fused_ms"] + t["sweep_ms"] + t["sweepk_ms"]) /
                          (t["fused_launches"] + 2 * t["sweep_launches"] + t["sweepk_depth"] * t["sweepk_launches"]))
        print(f"round {r} done", flush=True)
    bpc = 18 * (8 if a.precision == "f64" else 4)
    cells = a.nx * a.ny
    ref_rho, ref_u = ctxs[0][1].macro()
    for k, lat in ctxs:
        ms = np.array(res[k])
        r_, u_ = lat.macro()
        same = bool(np.array_equal(r_, ref_rho) and np.array_equal(u_, ref_u))
        row = {"config": k, "median_ms_per_iter": float(np.median(ms)), "min_ms": float(ms.min()),
               "mlups": cells / (np.median(ms) * 1e-3) / 1e6,
               "tbps_equiv_one_step": bpc * cells / (np.median(ms) * 1e-3) / 1e12, "bitwise_equal_to_first": same}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
