#!/bin/bash
# GPU-box side: tools/hp_diag.py on a few parity cases for the default build and the variants named
# (scratch/<variant>/libgstex_hip.so, tools/build_variant.sh), and with the near-edge-on path off (GSTEX_HP=0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/diag
for v in default hp0 "$@"; do
  for c in cfg1 no_reg cfg3w; do
    unset GSTEX_LIB GSTEX_HP
    [ "$v" = hp0 ] && export GSTEX_HP=0
    [ "$v" != default ] && [ "$v" != hp0 ] && export GSTEX_LIB=scratch/$v/libgstex_hip.so
    timeout -k 10 300 python3 -u tools/hp_diag.py $c > gpurun_out/diag/${v}_$c.log 2>&1 || { tail -5 gpurun_out/diag/${v}_$c.log; exit 1; }
    echo "$v $c: $(grep -E '^(means|quats) ' gpurun_out/diag/${v}_$c.log | awk '{print $1, $3}' | tr '\n' ' ')"
  done
done
