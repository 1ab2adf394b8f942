#!/bin/bash
# direct 3x3 conv: numerics, then ResNet-50 A/B (direct kernel on / off) on the same box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -3 gpurun_out/c3_tests.log
bash scripts/gpu_env_ab.sh resnet50 DDL_CONV3X3=1 DDL_CONV3X3=0
