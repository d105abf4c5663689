"""Regenerate ib_flip_envelope.json: the oracle against itself under per-iteration population
perturbations (tests/ib_flips.py).  Runs anywhere the oracle builds (no GPU, no reference)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import ib_flips
    from oracle import oracle as O
    env = ib_flips.envelope(O)
    allrows = [r for rows in env.values() for r in rows]
    out = {"config": {"nx": ib_flips.NX, "ny": ib_flips.NY, "steps": ib_flips.STEPS, "points": 150,
                      "perturbation": "f *= 1 + mag * n, n uniform in {-2..2} per population, every iteration"},
           "runs": env,
           "max_fs_ulps": max(r["fs_ulps"] for r in allrows),
           "max_fields": max(r["fields"] for r in allrows)}
    json.dump(out, open(os.path.join(HERE, "ib_flip_envelope.json"), "w"), indent=1)
    print(out["max_fs_ulps"], out["max_fields"])


if __name__ == "__main__":
    main()
