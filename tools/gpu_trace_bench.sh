#!/bin/bash
# Per-kernel average times of the bench train step (rocprofv3 --kernel-trace --stats) for the tree's library and
# scratch/<variant> libraries; prints kernels matching $FILTER.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/tb; mkdir -p $OUT
for v in tree "$@"; do
  if [ "$v" = tree ]; then lib=gstex_amd/libgstex_hip.so; else lib=scratch/$v/libgstex_hip.so; fi
  GSTEX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 5 > $OUT/$v.log 2>&1 || { echo "FAIL $v"; exit 1; }
  echo "== $v"
  python3 - "$OUT/$v/run_kernel_stats.csv" "${FILTER:-.}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if re.search(sys.argv[2], n):
        print(f"  {n[:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
done
