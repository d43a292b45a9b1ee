#!/bin/bash
# Kernel traces of the bench's graph and eager steps (driver settings), for tools/trace_gaps.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/gtrace; mkdir -p $OUT
for v in "graph:" "eager:--no-graph"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub $flags > $OUT/$name.log 2>&1 \
    || { echo "FAIL $name"; tail -20 $OUT/$name.log; exit 1; }
  cp "$(find $OUT/$name -name '*kernel_trace.csv' | head -1)" $OUT/${name}_kernel_trace.csv
done
python3 tools/trace_gaps.py $OUT/graph_kernel_trace.csv $OUT/eager_kernel_trace.csv
