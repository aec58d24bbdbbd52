#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): GPU parity tests, smoke(), the default bench
# line, then the round profile (tools/profile_round.sh). Every GPU step has its own time limit and the
# chain stops at the first failure. usage: bash tools/gpu_check.sh <profile-tag> [tests|bench|prof]...
set -uo pipefail
TAG=${1:-r01}
shift || true
STEPS=${*:-tests smoke bench prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
             > gpurun_out/gpu_tests.log 2>&1 ;;
    smoke) timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 ;;
    prof) bash tools/profile_round.sh "$TAG" > gpurun_out/prof.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
