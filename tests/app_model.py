"""TEST INFRASTRUCTURE: the reference driver's outputs (main.cu:263-1065) restated on top of the
CPU oracle, to check the drop-in driver `cuda_iblb_11_amd/bin/IBLB` file for file.

`expected_run(args)` derives the parameters exactly as main.cu:284-321 (float / unsigned
arithmetic included), runs the oracle with the restated cilia kinematics for ITERATIONS
iterations and returns the text of every file the reference writes, keyed by its path below
the data root.  Timestamps and runtimes are not reproducible; SimLog lines holding them are
returned as None.
"""
from __future__ import annotations

import math

import numpy as np

from oracle import oracle as O

LENGTH, YDIM = 96, 192          # main.cu:271, 279
C_S = 0.577                     # the driver's C_S (main.cu:22)
L_0, T_0 = 0.000006, 0.067      # main.cu:26-27


def g(x) -> str:
    """C++ ostream default formatting of a double (precision 6, %g)."""
    return "%g" % x


def to_string_3(x) -> str:
    """main.cu:255-261: setprecision(3)."""
    return "%.3g" % x


def params(argv: list[str]) -> dict:
    """main.cu:284-321 for the 10 positional arguments."""
    c_fraction, c_num, c_space = int(argv[0]), int(argv[1]), int(argv[2])
    Re, T_num, T_pow = float(argv[3]), np.float32(argv[4]), int(argv[5])
    I_pow, P_num = np.float32(argv[6]), int(argv[7])
    ShARC, BigData = bool(int(argv[8])), bool(int(argv[9]))
    XDIM = c_num * c_space
    T = int(round(float(T_num) * math.pow(10, T_pow)))            # nearbyint (ties to even; never a tie here)
    ITERATIONS = int(np.float32(np.float32(T) * I_pow))           # unsigned * float -> float -> unsigned
    INTERVAL = ITERATIONS // P_num
    dx, dt = 1.0 / LENGTH, 1.0 / T
    SPEED = 0.8 * 1000 / T
    TAU = (SPEED * LENGTH) / (Re * C_S * C_S) + 1.0 / 2.0
    TAU2 = 1.0 / (12.0 * (TAU - (1.0 / 2.0))) + (1.0 / 2.0)
    t_scale = 1000.0 * dt * T_0
    x_scale = 1000000.0 * dx * L_0
    return dict(c_fraction=c_fraction, c_num=c_num, c_space=c_space, Re=Re, T_num=float(T_num), T_pow=T_pow,
                P_num=P_num, ShARC=ShARC, BigData=BigData, XDIM=XDIM, T=T, ITERATIONS=ITERATIONS,
                INTERVAL=INTERVAL, dx=dx, dt=dt, SPEED=SPEED, TAU=TAU, TAU2=TAU2, t_scale=t_scale,
                x_scale=x_scale, s_scale=x_scale / t_scale, Ma=1.0 * SPEED / C_S,
                p_step=T * c_fraction // c_num)


def paths(p: dict) -> dict:
    raw = f"Raw/{p['c_num']}/{p['c_fraction']}/"
    cil = f"Cilia/{p['c_num']}/{p['c_fraction']}/"
    flux = (f"/Flux/{p['c_fraction']}_{p['c_num']}_{p['c_space']}_{to_string_3(p['Re'])}_"
            f"{to_string_3(p['T_num'])}x{p['T_pow']}-flux.dat")
    return {"raw": raw, "cilia": cil, "flux": flux, "simlog": raw + "/SimLog.txt"}


def simlog_lines(p: dict) -> list[str | None]:
    """main.cu:767-790 (None = timestamp line); the completion / runtime lines follow."""
    return [None, "", f"Size: {p['XDIM']}x{YDIM}", f"Iterations: {p['ITERATIONS']}",
            f"Reynolds Number: {g(p['Re'])}", f"Relaxation times: {g(p['TAU'])}, {g(p['TAU2'])}",
            f"Spatial step: {g(p['dx'] * L_0)}m", f"Time step: {g(p['dt'] * T_0)}s", f"Mach number: {g(p['Ma'])}",
            f"Phase Step: {p['c_fraction']}/{p['c_num']}", "",
            "Big Data is ON" if p["BigData"] else "Big Data is OFF",
            "Running on ShARC" if p["ShARC"] else "Running on local GPU"]


def fluid_text(p, rho, u) -> str:
    """main.cu:954-971."""
    X, size = p["XDIM"], p["XDIM"] * YDIM
    xs, ss = p["x_scale"], p["s_scale"]
    out = []
    for j in range(size):
        x, y = j % X, j // X
        ux, uy = u[j], u[size + j]
        ab = math.sqrt(ux * ux + uy * uy)
        out.append(f"{g(x * xs)}\t{g(y * xs)}\t{g(ux * ss)}\t{g(uy * ss)}\t{g(ab * ss)}\t{g(rho[j])}\n")
        if x == X - 1:
            out.append("\n")
    return "".join(out)


def cilia_text(p, s, u_s, eps) -> str:
    """main.cu:984-994 (float positions times the double scales)."""
    xs, ss, X = p["x_scale"], p["s_scale"], p["XDIM"]
    out = []
    for k in range(LENGTH * p["c_num"]):
        out.append(f"{g(float(s[2 * k]) * xs)}\t{g(float(s[2 * k + 1]) * xs)}\t{g(float(u_s[2 * k]) * ss)}\t"
                   f"{g(float(u_s[2 * k + 1]) * ss)}\t{int(eps[k])}\n")
        if k % 96 == 95 or s[2 * k] > np.float32(X - 1) or s[2 * k] < 1:
            out.append("\n")
    return "".join(out)


def expected_run(argv: list[str]) -> tuple[dict, dict]:
    """(params, {path: text}) of the reference run with these arguments, on the oracle."""
    p = params(argv)
    P = paths(p)
    X = p["XDIM"]
    sim = O.Simulation(X, YDIM, p["TAU"], p["TAU2"])
    cil = O.Cilia(p["c_num"], float(p["c_space"]), p["T"], p["p_step"], X)
    files = {}
    flux = []
    for it in range(p["ITERATIONS"]):
        s, u_s, eps = cil.points(it)
        sim.set_lagrangian(s.copy(), u_s.copy(), eps.copy())
        sim.step(1)
        if it % p["INTERVAL"] == 0:
            if p["BigData"]:
                files[P["raw"] + f"{it}-fluid.dat"] = fluid_text(p, sim.rho, sim.u)
                files[P["cilia"] + f"{it}-cilia.dat"] = cilia_text(p, s, u_s, eps)
            flux.append(f"{g(it * p['t_scale'])}\t{g(sim.flux * p['x_scale'])}\n")
    flux.append(f"{g(p['ITERATIONS'] * p['t_scale'])}\t{g(sim.flux * p['x_scale'])}\n")
    files[P["flux"]] = "".join(flux)
    return p, files
