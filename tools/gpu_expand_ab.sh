# k_expand A/B on one box: the compaction parity tests, then the compaction
# leg (tools/compact_probe.py) alternating PSAMD_NARROW=1 / 0 (PSAMD_AB=1).
#   TAG=nar bash tools/gpu_expand_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-nar}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groups.py tests/test_gpu_parity.py tests/test_gpu_dist.py ${EXTRA_TESTS:-} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export PSAMD_AB=1
for V in 1 0 1 0; do
  PSAMD_NARROW=$V timeout -k 10 200 python -u tools/compact_probe.py --steps 6 --timed 2 > $O/t_$V.json 2>> $O/t.err || { tail -20 $O/t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('narrow', sys.argv[2], {k: d[k] for k in d if not isinstance(d[k], (list, dict))})" $O/t_$V.json $V
done
