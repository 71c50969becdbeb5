# Round 4, GPU call o: extraction tests, quadtree stage stamps, the bench, the native per-call path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4o}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_extract.py tests/test_gpu_ordering.py} -m gpu -x -q -rf --timeout 120 \
    --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 scripts/qt_prof.py 128 > gpurun_out/${T}_qtprof.log 2>&1; echo "qtprof rc=$?"; grep level gpurun_out/${T}_qtprof.log
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --no-c3 --no-cd --host-fed-steps 0 > gpurun_out/${T}_bench.log 2>&1 || exit $?
python3 - "$R/gpurun_out/${T}_bench.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(d['value'], d['ms_per_step'], d['roofline_alone']['stage_ms_alone'])
print(d['host_api']['frames_per_s'], d['host_api']['latency_ms_median'], d['host_api']['native']['frames_per_s'])
PY
