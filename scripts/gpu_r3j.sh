set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3j_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r3j_pytest.log; [ $rc -eq 0 ] || exit $rc
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 10"
for v in base noemit scoreonly band; do
  L=""; E=""
  case $v in noemit) L=build/rows_noemit/liborbx.so;; scoreonly) L=build/rows_scoreonly/liborbx.so;; band) E="ORBX_FAST_ROWS=0";; esac
  env ORBX_LIB=$L ORBX_FAST_ROWS=1 $E ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3j_$v.log 2>&1 || exit $?
  echo "$v serial: $(grep -o '"value": [0-9.]*\|"fast_cells": [0-9.]*\|"fast_cells_l0": [0-9.]*' gpurun_out/r3j_$v.log | tr '\n' ' ')"
done
ORBX_FAST_ROWS=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3j_pipe.log 2>&1 || exit $?
echo "base pipelined: $(grep -o '"value": [0-9.]*\|"fast_cells": [0-9.]*\|"fast_cells_l0": [0-9.]*' gpurun_out/r3j_pipe.log | tr '\n' ' ')"
