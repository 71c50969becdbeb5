# Round 4, GPU call e: the whole GPU suite, the default bench, then the profile passes of scripts/prof_r4.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4e}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rb=$?
echo "bench rc=$rb"; tail -c 300 gpurun_out/${T}_bench.log
[ $rb -eq 0 ] || exit $rb
[ "${PROF:-1}" = 1 ] && { bash scripts/prof_r4.sh ${T}_prof || exit 1; }
exit $rc
