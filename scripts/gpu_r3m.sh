set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_new_mappoints.py tests/test_gpu_match.py tests/test_distinctive.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3m_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r3m_pytest.log; [ $rc -eq 0 ] || exit $rc
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 20"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r3m_tri.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $B --no-tri > gpurun_out/r3m_notri.log 2>&1 || exit $?
for v in tri notri; do echo "$v: $(grep -o '"value": [0-9.]*\|"keyframe_bow_fusion": [0-9.]*\|"keyframe_new_mappoints": [0-9.]*' gpurun_out/r3m_$v.log | tr '\n' ' ')"; done
