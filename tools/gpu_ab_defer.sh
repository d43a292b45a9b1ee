cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/check
for i in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --no-sub --no-cpu-baseline --steps 40 > gpurun_out/check/ab_defer_$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u bench.py --no-sub --no-cpu-baseline --steps 40 --no-defer-texture > gpurun_out/check/ab_plain_$i.log 2>&1 || exit 1
  python3 -c "
import json
for n in ['defer','plain']:
    d=json.loads(open('gpurun_out/check/ab_'+n+'_$i.log').read().strip().split('\n')[-1]); print(n, d['ms_per_step'], d['ms_per_step_median'])"
done
