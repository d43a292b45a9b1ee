#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the raster kernels on the raster-only cfg3 loop, per library variant:
#   VARIANTS="base a32" bash tools/gpu_traffic_ab.sh   (scratch/<v>/libgstex_hip.so; "base" = the in-tree library)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/traffic; mkdir -p $OUT
for v in $VARIANTS; do
  if [ "$v" = base ]; then unset GSTEX_LIB; else export GSTEX_LIB=scratch/$v/libgstex_hip.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$v/$c -o run -- python3 tools/raster_loop.py --photometric --iters 3 > $OUT/$v_$c.log 2>&1 || { echo "$v $c failed"; exit 1; }
  done
done
python3 - $OUT $VARIANTS <<'PY'
import csv, glob, sys, collections
out, vs = sys.argv[1], sys.argv[2:]
for v in vs:
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = collections.defaultdict(float); disp = collections.defaultdict(set)
        for f in glob.glob(f"{out}/{v}/{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                k = "bwd" if "raster_bwd" in k else "fwd" if "raster_fwd" in k else "setup_bwd" if "setup_bwd" in k else None
                if k: per[k] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
        res[c] = {k: per[k] / len(disp[k]) for k in per}
    for k in ("fwd", "bwd", "setup_bwd"):
        f, w = res["FETCH_SIZE"].get(k, 0), res["WRITE_SIZE"].get(k, 0)
        print(f"{v:8s} {k:9s} fetch {2*f/1024:8.1f} MB  write {w/1024:8.1f} MB  total {(2*f+w)/1024:8.1f} MB")
PY
