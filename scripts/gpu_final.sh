# Final checks of a round: the whole -m gpu suite, smoke(), the default bench, the EuRoC bench and the N=2 gloo rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config euroc --cpu-seconds 0 --host-api-frames 16 > gpurun_out/${TAG}_bench_euroc.log 2>&1; rc=$?
echo "bench euroc rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --cpu-seconds 0 --host-api-frames 0 --no-c3 \
    > gpurun_out/${TAG}_rehearsal_2ranks_gloo.log 2>&1; rc=$?
echo "rehearsal rc=$rc"; tail -c 400 gpurun_out/${TAG}_rehearsal_2ranks_gloo.log
exit $rc
