#!/bin/bash
# Scratch: end-to-end pcap throughput of retina_amd/_lib/rtn_offline on cfg2 frames.
set -e
N=${1:-16777216}
T=${TMPDIR:-/tmp}
python scratch/mk_pcap.py cfg2 $N $T/cfg2.pcap
python -c "import sys; sys.path.insert(0,'tests'); from golden.filter_sets import SETS; open('$T/cfg2.toml','w').write(SETS['cfg2'])"
for b in 1048576 4194304; do
  timeout -k 10 120 retina_amd/_lib/rtn_offline $T/cfg2.toml $T/cfg2.pcap --batch $b --no-ct
  timeout -k 10 120 retina_amd/_lib/rtn_offline $T/cfg2.toml $T/cfg2.pcap --batch $b
done
rm -f $T/cfg2.pcap
