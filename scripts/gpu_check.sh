# GPU round: parity tests, bench, rocprofv3 kernel trace + PMC traffic passes.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds ${CPU_SECONDS:-10} > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/kt" -o run -- \
      python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 --no-timing > gpurun_out/prof_kt.log 2>&1; rc=$?
  echo "rocprof kt rc=$rc"; tail -2 gpurun_out/prof_kt.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof/fetch" -o run -- \
      python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --no-timing > gpurun_out/prof_fetch.log 2>&1; rc=$?
  echo "rocprof fetch rc=$rc"; tail -2 gpurun_out/prof_fetch.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof/write" -o run -- \
      python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --no-timing > gpurun_out/prof_write.log 2>&1; rc=$?
  echo "rocprof write rc=$rc"; tail -2 gpurun_out/prof_write.log
  [ $rc -eq 0 ] || exit $rc
  find gpurun_out/prof -type f | head -50
fi
