#!/bin/bash
# GPU-box side (gpurun -- bash tools/gpu_kernel_ab.sh TAG "LABEL=ENV..." ...): rocprofv3 --kernel-trace --stats over
# the cfg3 training-path raster loop (tools/raster_loop.py, which also runs the binning) under each labelled
# environment, for per-kernel A/B averages; prints the KERNELS (regex) rows.  BENCH=1: over a short bench.py run instead
# (the whole training step: loss, Adam, prologue / epilogue kernels).
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2; do
  for cfg in "$@"; do
    label=${cfg%%=*}; envs=${cfg#*=}
    if [ -n "$BENCH" ]; then CMD="bench.py --no-cpu-baseline --no-sub --steps 20 --warmup 5"; else CMD="tools/raster_loop.py --photometric --no-geometry --iters 20"; fi
    env $envs timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${label}_$i -o run -- python3 $CMD > $OUT/${label}_$i.log 2>&1 || { echo "$label failed"; tail -5 $OUT/${label}_$i.log; exit 1; }
    python3 - "$OUT/${label}_$i" "$label #$i" "${KERNELS:-tile_sort|place|count_lds|tile_rank|scan}" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
pick = re.compile(sys.argv[3])
out = []
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if pick.search(n):
        out.append(f"{n.split('<')[0]} {float(r['AverageNs']) / 1000:.1f}")
print(sys.argv[2] + ": " + ", ".join(out))
PY
  done
done
