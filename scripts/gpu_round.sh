# GPU round: parity tests (one process, per-test timeout), then the default bench and the euroc bench.
# Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r2}
MODE=${2:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -6 gpurun_out/${TAG}_pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 3000 gpurun_out/${TAG}_bench.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --config euroc --cpu-seconds 0 --host-api-frames 16 > gpurun_out/${TAG}_bench_euroc.log 2>&1; rc=$?
  echo "bench euroc rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench_euroc.log
  [ $rc -eq 0 ] || exit $rc
fi
