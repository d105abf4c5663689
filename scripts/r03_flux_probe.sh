#!/bin/bash
# Diagnostic: the slab group's flux with straddling filaments (mock RCCL, 2 ranks, mode 3), traced
# after every call against the single slab, with the installed band plans printed
set -o pipefail
IBLB_DEBUG_PLAN=1 RUN_GROUP_TRACE=1 RUN_GROUP_FLUX_COLUMN=71 timeout -k 10 120 python3 tests/mock_rccl/run_group.py 2 96 130 25 3 f64 1 2>&1 | grep -v Warn | cut -c1-250 | head -40
exit 0
