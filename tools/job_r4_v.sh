#!/bin/bash
# Round 4: the full GPU suite at HEAD (after the reset-branch laundering and the MT19937 host changes).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4v; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; exit $rc
