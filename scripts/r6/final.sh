# Round-6 validation of a tree: the whole -m gpu suite (one process, per-test time limit), smoke(), the default bench,
# the EuRoC bench, the two-rank gloo rehearsal (bench.py --gpus 2 on one GPU) and the emulated 1/2/4/8-agent sweep.
# usage: bash scripts/r6/final.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?
tail -c 600 gpurun_out/${T}_bench.log; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config euroc --cpu-seconds 0 --host-api-frames 16 > gpurun_out/${T}_bench_euroc.log 2>&1; rc=$?
tail -c 300 gpurun_out/${T}_bench_euroc.log; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd \
    --host-fed-steps 0 > gpurun_out/${T}_rehearsal_2ranks_gloo.log 2>&1; rc=$?
tail -c 300 gpurun_out/${T}_rehearsal_2ranks_gloo.log; echo; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_emu.sh ${T}_emu
