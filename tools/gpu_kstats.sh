#!/bin/bash
# rocprofv3 kernel statistics of the cfg3 raster loop for each scratch/<variant> given (the forward / backward kernel
# times without the host-side timing events' launch brackets).  Results: gpurun_out/kstats/<variant>_kernel_stats.csv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/kstats; mkdir -p $OUT
for v in "$@"; do
  GSTEX_LIB=scratch/$v/libgstex_hip.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/$v -o run -- python3 tools/raster_loop.py --photometric --no-geometry --iters 20 > $OUT/$v.log 2>&1 \
    || { echo "FAIL $v"; exit 1; }
  f=$(find $OUT/$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $OUT/${v}_kernel_stats.csv
  python3 - "$OUT/${v}_kernel_stats.csv" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if "raster_fwd" in n or "raster_bwd_kernel" in n or "order" in n:
        out.append(f"{n.split('(')[0][-40:]}: {float(r['AverageNs'])/1e3:.1f} us x{r['Calls']}")
print(sys.argv[2], "|", "; ".join(out))
PY
done
