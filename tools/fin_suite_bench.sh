set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05final4; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
echo bench done
