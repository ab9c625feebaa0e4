#!/bin/bash
# Scratch: dump gfx950 ISA of the cfg2 kernel for a variant: scratch/isa.sh "RTN_UNROLL2" out.s [cfg]
set -e
DEFS="$1"; OUT="$2"; CFG="${3:-cfg2}"
python3 - "$CFG" > /tmp/isa/src.hip <<'PY'
import sys; sys.path.insert(0, "."); sys.path.insert(0, "tests")
import bench
from retina_amd import pc
print(pc.Program.from_spec(bench.spec_for(sys.argv[1])).source)
PY
H=""
for d in $(echo "$DEFS" | tr ',' ' '); do H="$H -D$d"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S $H /tmp/isa/src.hip -o "$OUT" 2>&1 | grep -v warning || true
grep -E "vgpr_count|sgpr_count|scratch|NumVgprs|Occupancy|lds_size" "$OUT" | head -8
