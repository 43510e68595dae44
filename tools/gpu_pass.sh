#!/bin/bash
# One GPU pass on a gpurun box: smoke, the GPU test suite, the driver-shaped
# bench (N=1) and a rocprofv3 kernel table of the headline forward.
#   tools/gpu_pass.sh TAG [smoke] [tests] [bench] [prof] [hostcost]   (default: the first four)
# Logs go to gpurun_out/TAG_*.log; each GPU step has its own time limit and the
# steps stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
STEPS=${*:-smoke tests bench prof}
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || exit 11 ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
             > $OUT/${TAG}_gpu_tests.log 2>&1 || exit 12 ;;
    bench) timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${TAG}_bench.log 2>&1 || exit 13 ;;
    prof)  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run -- \
             python -u tools/fwd_loop.py --model resnet18 --batch 400 --iters 30 > $OUT/${TAG}_prof.log 2>&1 || exit 14 ;;
    hostcost)  # coordinator host cost per round, gloo dry run (CPU only) at N=1 and N=8
      for n in 1 8; do
        timeout -k 10 300 python -u bench.py --dry-run --system --gpus $n --steps 400 --warmup 10 --sdfs-images 0 \
          --two-job-queries 2 > $OUT/${TAG}_hostcost_n$n.log 2>&1 || exit 15
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
