#!/bin/bash
# GPU-box side: per-kernel average times of the raster loop (rocprofv3 --kernel-trace --stats) for each
# scratch/<variant>/libgstex_hip.so given; prints the kernels matching $FILTER (regex, default: all).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tv; mkdir -p $OUT
for v in "$@"; do
  GSTEX_LIB=scratch/$v/libgstex_hip.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 tools/raster_loop.py ${RL_ARGS:---photometric} --iters 10 > $OUT/$v.log 2>&1 || { echo "FAIL $v"; exit 1; }
  echo "== $v"
  python3 - "$OUT/$v/run_kernel_stats.csv" "${FILTER:-.}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if re.search(sys.argv[2], n):
        print(f"  {n[:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
done
