export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# k_pull_pair A/B: parity tests under both LDS stage sizes, then the cfg3
# bench with pairs (1024- and 512-word stages) and without
set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pair1}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PSAMD_PAIR_WORDS=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest512.log 2>&1 || { tail -40 $O/pytest512.log; exit 1; }
tail -1 $O/pytest512.log
for V in ${VARIANTS:-"PSAMD_PAIR_WORDS=1024" "PSAMD_PAIR_WORDS=512" "PSAMD_PULL_PAIR=0"}; do
  env ${V//,/ } timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-general --sustain 0 > $O/bench_$V.json 2> $O/bench_$V.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), r['kernel'], round(r['frac'],3), d['last_step']['expand_us_per_round'])" $O/bench_$V.json $V
done
