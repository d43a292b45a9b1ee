cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/check
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_trainer_sync.py -x -v --timeout 150 --timeout-method thread > gpurun_out/check/ts.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/check/ts.log | tail -2; [ $rc = 0 ] || exit $rc
bash tools/gpu_r03e.sh
