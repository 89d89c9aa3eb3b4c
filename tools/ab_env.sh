#!/bin/bash
# Alternating A/B of environment settings on one bench command (PSAMD_AB=1):
#   VARIANTS="X=0 X=1" REPS=2 TAG=t bash tools/ab_env.sh [bench args]
set -o pipefail
O=gpurun_out/${TAG:-envab}; mkdir -p $O
export PSAMD_AB=1
for R in $(seq ${REPS:-2}); do for V in $VARIANTS; do
  env ${V//,/ } timeout -k 10 200 python -u bench.py --steps 500 --warmup 5 --no-cpu --no-general --sustain 0 "$@" > $O/b_${V}_$R.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), round(r['frac'],3), [x for x in d['last_step']['expand_us_per_round'] if x])" $O/b_${V}_$R.json $V
done; done
