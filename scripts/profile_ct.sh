#!/bin/bash
# Connection-lookup profile on the GPU box: kernel-trace stats of the steady passes
# of tools/ct_ab.py --profile, then separate PMC passes over the same command.
#   bash scripts/profile_ct.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3a}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ctprof_${TAG}" -o run -- python tools/ct_ab.py --profile --steps 20 > gpurun_out/ctprof_${TAG}.txt 2>&1 || exit $?
i=0
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/ctpmc_${TAG}_$i" -o run -- python tools/ct_ab.py --profile --steps 5 > /dev/null 2> gpurun_out/ctpmc_${TAG}_$i.err || exit $?
done
echo done
