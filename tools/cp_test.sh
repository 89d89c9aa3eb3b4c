# compaction-path parity tests, then the A/B of tools/cp_run.sh
set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
PSENGINE_LIB_AB=${TEST_LIB:-} timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groups.py tests/test_gpu_parity.py > gpurun_out/$TAG/pytest.log 2>&1
tail -3 gpurun_out/$TAG/pytest.log
bash tools/cp_run.sh
