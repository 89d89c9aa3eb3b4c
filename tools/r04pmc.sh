# PMC passes (separate runs, one counter group each) for round 4:
#   cfg3 bench (k_pull_chain traffic for bench.py's roofline.traffic) and the
#   4-rank peer-hash loopback (k_pull / k_pack bytes per round vs row bytes)
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/r04pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() { name=$1; shift; ctr=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc $ctr -T -f csv -d "$OUT/$name" -o run -- "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?; echo "$name rc=$rc"; return $rc; }
(cd "$ROOT" && timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_async.log" 2>&1) || { echo PYTEST_FAILED; tail -20 "$OUT/pytest_async.log"; exit 1; }
pass cfg3_fetch FETCH_SIZE python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-general --sustain 0 &&
pass cfg3_write WRITE_SIZE python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-general --sustain 0 &&
pass lb_fetch FETCH_SIZE python3 "$ROOT/tools/loopback_bench.py" --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 1 &&
pass lb_write WRITE_SIZE python3 "$ROOT/tools/loopback_bench.py" --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 1
timeout -k 10 200 python3 "$ROOT/tools/chain_profile.py" --workload cfg2 --steps 3 > "$OUT/chain_prof_cfg2.json" 2> "$OUT/chain_prof_cfg2.log"
