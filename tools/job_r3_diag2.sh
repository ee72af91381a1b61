#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/diag_partials2.py || exit $?
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "state_roundtrip or metrics_and_partials" 2>&1 | tail -3
