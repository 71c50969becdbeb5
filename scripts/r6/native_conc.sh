# The native multi-thread driver on the GPU box: the plain build under pytest, then the ThreadSanitizer build
# (make tsan, built on the CPU side) through scripts/tsan_gpu.sh.  usage: bash scripts/r6/native_conc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6conc}
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_concurrency.py tests/test_gpu_concurrency.py -m gpu -x -q -rf \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tsan_gpu.sh 4; rc=$?
cp gpurun_out/tsan.log gpurun_out/${T}_tsan.log
exit $rc
