#!/bin/bash
# same-box A/B: conv_glds sched_barrier keeping the first MFMA group above the second LDS wait (this tree) vs the previous commit
# (worktree ab/old, its own _C.so), whole captured forward, alternating processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_split.py -k "tile or 42 or l2_prefetch" > gpurun_out/r3_sb_test.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then T=ab/old/tools/fwd_loop.py; else T=tools/fwd_loop.py; fi
    echo "$v r$r:" && timeout -k 10 120 python -u $T --model resnet50 --batch 1024 --dtype fp16 --iters 15 || exit 1
    echo "$v r$r:" && timeout -k 10 120 python -u $T --model resnet18 --batch 400 --dtype fp32 --iters 40 || exit 1
    echo "$v r$r:" && timeout -k 10 120 python -u $T --model resnet18 --batch 400 --dtype fp16 --iters 40 || exit 1
  done
done > gpurun_out/r3_ab_sched_barrier.log 2>&1
