#!/bin/bash
set -eo pipefail
ROUND_TAG=${ROUND_TAG:-r01d} bash scripts/gpu_check.sh
ROUND_TAG=${ROUND_TAG:-r01d} bash scripts/tune_layout.sh
