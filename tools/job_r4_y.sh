#!/bin/bash
# Round 4: lifecycle tests incl. the exit-with-a-draw-in-flight case (library destructor joins).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4y; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_lifecycle.py -m gpu -v --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -4 "$O/pytest.log"; exit $rc
