#!/bin/bash
# round 6 (s): the ABI-v5 meta tests (mid-episode start rows vs the oracle, score_moves errors)
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_env_gpu.py -k "meta_start_row or score_moves_errors or clock_past or reset_mask"
