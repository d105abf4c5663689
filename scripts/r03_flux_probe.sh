#!/bin/bash
# Diagnostic: the slab group's flux with straddling filaments (mock RCCL, 2 ranks, mode 3) for
# several flux columns: 91 (last rank, in a patch output and the boundary sweep), 71 (interior,
# no patch), 44 (rank 0, patch output + boundary), 40 (rank 0 interior).
set -o pipefail
for fc in 91 71 44 40 5 2; do
  RUN_GROUP_FLUX_COLUMN=$fc timeout -k 10 120 python3 tests/mock_rccl/run_group.py 2 96 130 25 3 f64 1 | tail -1 | cut -c1-400
done
