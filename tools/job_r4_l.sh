#!/bin/bash
# Round 4: the GPU training / checkpoint tests after the SB3-pickle change of the checkpoint zips.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4l; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_checkpoint.py -m "gpu or not gpu" -x -v \
  --timeout 200 --timeout-method thread > "$O/pytest_training.log" 2>&1
rc=$?; tail -3 "$O/pytest_training.log"; exit $rc
