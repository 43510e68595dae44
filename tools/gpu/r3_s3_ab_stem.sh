#!/bin/bash
# stem interior-row border correction hoisted: numerics (split stem tests + smoke), same-box A/B vs ab/old
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split.py -k "stem or resnet" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_stem_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_stem_smoke.log 2>&1 &&
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then T=ab/old/tools/fwd_loop.py; else T=tools/fwd_loop.py; fi
    echo "$v r$r" && timeout -k 10 120 python -u $T --model resnet18 --batch 400 --dtype fp32 --iters 40 || exit 1
  done
done > gpurun_out/r3_ab_stem.log 2>&1
