export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# A/B of engine environment switches on the cfg3 bench (no tests):
#   VARIANTS="A=1,B=2 C=3" bash tools/ab_env.sh <tag> [bench args]
set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; shift || true
mkdir -p $O
for V in $VARIANTS; do
  env ${V//,/ } timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-general --sustain 0 "$@" > $O/bench_$V.json 2> $O/bench_$V.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), r['kernel'], round(r['frac'],3), [x for x in d['last_step']['expand_us_per_round'] if x])" $O/bench_$V.json $V
done
