#!/bin/bash
# Profiling recipe run on the GPU box (see DESIGN.md "Measurement"): bench, kernel-trace stats,
# then separate PMC passes (FETCH_SIZE / WRITE_SIZE never share a pass with tracing domains).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
CFG=${2:-cfg2}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config $CFG > gpurun_out/bench_${TAG}_${CFG}.json 2> gpurun_out/bench_${TAG}_${CFG}.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_${CFG}" -o run -- python bench.py --config $CFG --no-cpu --no-e2e --no-conn > gpurun_out/bench_${TAG}_${CFG}_kt.json 2> gpurun_out/prof_${TAG}_${CFG}.err || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_${TAG}_${CFG}_$C" -o run -- python bench.py --config $CFG --no-cpu --no-e2e --no-conn --steps 5 --warmup 1 > /dev/null 2> gpurun_out/pmc_${TAG}_${CFG}_$C.err || exit $?
done
echo done
