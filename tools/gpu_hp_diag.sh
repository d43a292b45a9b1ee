cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/diag
for c in cfg1 2dgs_T0 cfg3w; do timeout -k 10 300 python3 -u tools/hp_diag.py $c > gpurun_out/diag/$c.log 2>&1 || { tail -5 gpurun_out/diag/$c.log; exit 1; }; done
tail -40 gpurun_out/diag/cfg1.log
