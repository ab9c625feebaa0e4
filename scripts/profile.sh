#!/bin/bash
# Profiling recipe run on the GPU box: bench line, kernel-trace stats, then separate
# PMC passes (FETCH_SIZE / WRITE_SIZE / request counters never share a pass with tracing domains).
#   bash scripts/profile.sh <tag> <cfg> [--no-bench]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
CFG=${2:-cfg2}
cd "$R"
mkdir -p gpurun_out
if [ "$3" != "--no-bench" ]; then
  timeout -k 10 400 python bench.py --config $CFG > gpurun_out/bench_${TAG}_${CFG}.json 2> gpurun_out/bench_${TAG}_${CFG}.err || exit $?
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_${CFG}" -o run -- python bench.py --config $CFG --no-cpu --no-e2e --no-conn > gpurun_out/bench_${TAG}_${CFG}_kt.json 2> gpurun_out/prof_${TAG}_${CFG}.err || exit $?
i=0
for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_${TAG}_${CFG}_$i" -o run -- python bench.py --config $CFG --no-cpu --no-e2e --no-conn --steps 5 --warmup 1 --settle-ms 0 > /dev/null 2> gpurun_out/pmc_${TAG}_${CFG}_$i.err || exit $?
done
echo done
