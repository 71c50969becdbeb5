set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/r3h_pytest.log | grep -v "^\s*$" | tail -25; [ $rc -eq 0 ] || exit $rc
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h_bench_rows.log 2>&1 || exit $?
ORBX_FAST_ROWS=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h_bench_band.log 2>&1 || exit $?
ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h_bench_rows_serial.log 2>&1 || exit $?
ORBX_PIPELINE=0 ORBX_FAST_ROWS=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h_bench_band_serial.log 2>&1 || exit $?
for f in rows band rows_serial band_serial; do echo "$f: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"fast_cells": [0-9.]*\|"fast_cells_l0": [0-9.]*' gpurun_out/r3h_bench_$f.log | tr '\n' ' ')"; done
