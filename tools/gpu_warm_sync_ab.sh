#!/bin/bash
# A/B of the warmup-time synchronisation before the pool reservation (GSTEX_BENCH_WARM_SYNC=1/0), driver command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r05w; mkdir -p $OUT
for r in 1 2 3; do for f in 1 0; do
GSTEX_BENCH_WARM_SYNC=$f timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/b_${f}_$r.log 2>&1 || { tail -5 $OUT/b_${f}_$r.log; exit 1; }
python3 -c "
import json,sys
d=json.loads(open('$OUT/b_${f}_$r.log').read().strip().splitlines()[-1]); s=d['step_ms_events']
print('sync=$f', d['ms_per_step'], d['ms_per_step_median'], s[:3])"
done; done
