#!/bin/bash
# Is the root-row stage worth it?  cfg3 / cfg4 with the cross-window overlap
# off (it conflicts: the next window's init rewrites the root rows), root
# rows on / off; and the default (overlap on, root rows off) beside them.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04al
mkdir -p $O
for W in cfg3 cfg4; do
  for V in "1 0" "0 0" "1 0" "0 0" "0 1" "0 1"; do
    set -- $V
    PSAMD_AB=1 PSAMD_CHAIN_ROOT_ROW=$1 PSAMD_OVERLAP=$2 timeout -k 10 200 python -u tools/host_split.py --workload $W --steps 200 --reps 1 >> $O/hs_$W.log 2>&1
    echo "$W root_row=$1 overlap=$2 $(tail -n 1 $O/hs_$W.log | cut -c1-60)"
  done
done
