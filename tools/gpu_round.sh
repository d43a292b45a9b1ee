cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1
grep -E "passed|failed" gpurun_out/r02/gpu_tests.log | tail -1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1; tail -1 gpurun_out/r02/smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/r02/bench.log 2>&1; tail -1 gpurun_out/r02/bench.log | cut -c1-300
timeout -k 10 1200 bash tools/profile_bench.sh r02 > gpurun_out/r02/prof.log 2>&1; tail -2 gpurun_out/r02/prof.log
