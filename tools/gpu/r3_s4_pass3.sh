#!/bin/bash
# GPU pass: smoke, GPU suite, driver bench (N=1), ResNet50 b1024 fp16 + split benches, ResNet50 fp16 kernel table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_s6_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_s6_gpu_tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py > gpurun_out/r3_s6_bench.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model resnet50 --batch 1024 --dtype fp16 --steps 10 --warmup 3 --no-system \
    > gpurun_out/r3_s6_bench_r50_fp16.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model resnet50 --batch 1024 --dtype fp32 --steps 10 --warmup 3 --no-system \
    --no-extras > gpurun_out/r3_s6_bench_r50_fp32.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_s6_prof -o run -- \
    python3 tools/fwd_loop.py --model resnet50 --batch 1024 --dtype fp16 --iters 10 > gpurun_out/r3_s6_prof.log 2>&1
