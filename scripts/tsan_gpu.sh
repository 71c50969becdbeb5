# ThreadSanitizer run of the native concurrency driver (make tsan, on the CPU side) on a GPU box: two extractors on two
# threads and four matchers on four threads, bit-exact against their first results; TSan reports involving liborbx's
# host code fail the run.  Output: gpurun_out/tsan.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TSAN_OPTIONS="suppressions=$R/tests/native/tsan.supp halt_on_error=0 report_signal_unsafe=0 second_deadlock_stack=1"
timeout -k 10 300 build/tsan/concurrency ${1:-10} > gpurun_out/tsan.log 2>&1; rc=$?
echo "concurrency rc=$rc"; grep -c "WARNING: ThreadSanitizer" gpurun_out/tsan.log || true
tail -3 gpurun_out/tsan.log
exit $rc
