#!/bin/bash
# GPU pass: smoke, whole GPU suite, driver bench (N=1, all phases), rocprof kernel table of ResNet50 b1024 fp16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_gpu_tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py > gpurun_out/r3_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 -- \
    python3 tools/fwd_loop.py --model resnet50 --batch 1024 --dtype fp16 --iters 10 > gpurun_out/r3_prof_r50.log 2>&1
