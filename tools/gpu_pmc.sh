#!/bin/bash
# SQ stall/issue counter passes over the raster-only cfg3 loop for one build, summarised per kernel.
#   TAG=name [TREE=scratch/head] [LIB=scratch/x/libgstex_hip.so] [KERNELS='raster_bwd|tile_sort'] bash tools/gpu_pmc.sh
# TREE: the source tree whose python + library run (default: this one); output under gpurun_out/pmc_<TAG>/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-cur}
OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p $OUT
TREE=${TREE:-.}
cd "$TREE" || exit 1
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" \
            "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  if [ -n "$LIB" ]; then export GSTEX_LIB=$LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o run -- python3 tools/raster_loop.py --photometric --iters 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" "${KERNELS:-raster_bwd|raster_fwd}" <<'PY'
import csv, collections, glob, re, sys
out, pick = sys.argv[1], re.compile(sys.argv[2])
per = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
        if not pick.search(k):
            continue
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
with open(f"{out}/summary.txt", "w") as fh:
    for k, d in per.items():
        fh.write(f"== {k}\n")
        for c in sorted(d):
            n = len(cnt[(k, c)])
            fh.write(f"  {c:24s} {d[c] / max(n, 1):.4g}  (per launch, {n} launches)\n")
print(open(f"{out}/summary.txt").read())
PY
