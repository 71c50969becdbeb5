set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 10"
for v in base noemit scoreonly; do
  case $v in base) L="";; pf6) L=build/rows_pf6/liborbx.so;; noemit) L=build/rows_noemit/liborbx.so;; scoreonly) L=build/rows_scoreonly/liborbx.so;; esac
  ORBX_LIB=$L ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3i_$v.log 2>&1 || exit $?
  echo "$v: $(grep -o '"value": [0-9.]*\|"fast_cells": [0-9.]*\|"fast_cells_l0": [0-9.]*' gpurun_out/r3i_$v.log | tr '\n' ' ')"
done
