#!/bin/bash
# same-box A/B: conv_glds buffer-resource DMA + immediate-offset fragment reads (this tree) vs the
# previous commit (worktree ab/old, its own _C.so), whole captured forward, alternating processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then T=ab/old/tools/fwd_loop.py; else T=tools/fwd_loop.py; fi
    for dt in fp32 fp16; do
      echo -n "$v r$r: " && timeout -k 10 120 python -u $T --model resnet18 --batch 400 --dtype $dt --iters 40 || exit 1
    done
  done
done > gpurun_out/r3_ab_bufdma.log 2>&1
