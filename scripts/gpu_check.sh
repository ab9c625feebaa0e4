#!/bin/bash
# One GPU-box call: the GPU test suite, smoke(), then one bench line per config given.
#   bash scripts/gpu_check.sh <tag> [cfg ...]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-chk}
shift
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gputest_${TAG}.txt 2>&1 || { tail -30 gpurun_out/gputest_${TAG}.txt; exit 1; }
tail -2 gpurun_out/gputest_${TAG}.txt
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.txt 2>&1 || exit 1
cat gpurun_out/smoke_${TAG}.txt
for CFG in "$@"; do
  timeout -k 10 400 python bench.py --config $CFG > gpurun_out/bench_${TAG}_${CFG}.json 2> gpurun_out/bench_${TAG}_${CFG}.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['frac'], d.get('verified'))" gpurun_out/bench_${TAG}_${CFG}.json $CFG
done
echo done
