export PSAMD_AB=1  # plan options from the environment (A/B tools only)
set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/xlds; mkdir -p $O
for X in 0 4096 10240 20480; do
  PSAMD_PULL_PAIR=0 PSAMD_XLDS=$X timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-general > $O/b$X.json 2> $O/b$X.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), r['kernel'], round(r['frac'],3), d['last_step']['expand_us_per_round'][11:])" $O/b$X.json $X
done
