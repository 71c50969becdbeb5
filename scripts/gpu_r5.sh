# Round-5 GPU call: the whole -m gpu suite (one process, per-test limit), the N=2 gloo rehearsal of the full step
# through `bench.py --gpus 2`, then the default N=1 bench.  Every GPU step has its own limit; a failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r5}
MODE=${2:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -8 gpurun_out/${TAG}_pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = rehearsal ]; then
  timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --cpu-seconds 0 --host-api-frames 0 --no-c3 \
      > gpurun_out/${TAG}_rehearsal_2ranks_gloo.log 2>&1; rc=$?
  echo "rehearsal rc=$rc"; tail -c 2500 gpurun_out/${TAG}_rehearsal_2ranks_gloo.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = hwq ]; then
  for q in 4 8; do
    ORBX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd \
        --host-fed-steps 0 > gpurun_out/${TAG}_hwq$q.log 2>&1 || { echo "hwq $q failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_hwq$q.log').read().strip().splitlines()[-1]); print('hwq', $q, d['value'], d['ms_per_step'])"
  done
fi
