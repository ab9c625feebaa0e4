#!/bin/bash
# Scratch: PMC passes over scratch/prof_ctx.py: pmc_ctx.sh <defines> <tag> <groups-file>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V="$1"; TAG="$2"; G="${3:-scratch/pmc_groups.txt}"
i=0
while read -r C; do
  [ -z "$C" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pc_${TAG}_$i -o run -- python scratch/prof_ctx.py "$V" ${NCTX:-1} 3 > gpurun_out/pc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done < "$G"
echo ok
