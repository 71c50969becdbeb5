# Round 4, GPU call g: the whole GPU suite, the default bench, then one runtime trace of the bench's steps (HIP API +
# memory copies + kernels: which call issues the slow rocclr copy kernels) and the kernel-trace profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rb=$?
echo "bench rc=$rb"; tail -c 300 gpurun_out/${T}_bench.log
[ $rb -eq 0 ] || exit $rb
O=gpurun_out/${T}_rt; rm -rf $O; mkdir -p $O
timeout -s KILL 240 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --output-format csv -d "$R/$O" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 \
    --alone-reps 0 > $O/rt.log 2>&1; echo "rt rc=$?"
[ "${PROF:-1}" = 1 ] && { bash scripts/prof_r4.sh ${T}_prof || exit 1; }
exit $rc
