"""Regenerate nominals_envelope.json from the reference's own nominal outputs.

Reads /root/reference/CUDA_IBLB_11/Data/Nominals (data files shipped with the reference:
fluid snapshots `<it>-vector_nom.dat` with columns x y u_x u_y |u| rho, and the cumulative
flux `flux_nom.dat`).  They come from an older version of the code (300x200, LENGTH=100,
SimLog_nom.txt), so only summary statistics are kept: an envelope, not bit-level vectors.
Run in the build container (the reference is not present on the GPU box).
"""
import json
import os

import numpy as np

SRC = "/root/reference/CUDA_IBLB_11/Data/Nominals"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nominals_envelope.json")


def main():
    out = {"source": "CUDA_IBLB_11/Data/Nominals (older 300x200 version, SimLog_nom.txt)", "vector": {}}
    for it in (1000, 50000, 99000):
        a = np.loadtxt(os.path.join(SRC, f"{it}-vector_nom.dat"))
        out["vector"][str(it)] = {
            "cells": int(a.shape[0]),
            "nx": int(a[:, 0].max()) + 1, "ny": int(a[:, 1].max()) + 1,
            "rho_mean": float(a[:, 5].mean()), "rho_min": float(a[:, 5].min()), "rho_max": float(a[:, 5].max()),
            "u_max": float(a[:, 4].max()), "ux_mean": float(a[:, 2].mean()),
        }
    fl = np.loadtxt(os.path.join(SRC, "flux_nom.dat"))
    out["flux"] = {"t_ms": fl[:, 0].tolist(), "Q": fl[:, 1].tolist()}
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
