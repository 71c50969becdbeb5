# First calls of fresh extractors racing on threads (the host-graph capture vs another thread's configuration):
# the whole GPU suite, the race test three more times, and the native per-call driver with the timing-shifting
# resize-tail form that first showed the failure (r7r).  usage: bash scripts/r6/firstcalls.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r7fc}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_first_calls.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_race_$i.log 2>&1; rc=$?
  tail -1 gpurun_out/${T}_race_$i.log; [ $rc -eq 0 ] || exit $rc
done
for t in 4 4 0; do
  env ORBX_RESIZE_TAIL=$t timeout -k 10 120 build/host_api_bench multiagent_orb_slam2_amd/liborbx.so 300 > gpurun_out/${T}_hapi_tail$t.log 2>&1 || { tail -3 gpurun_out/${T}_hapi_tail$t.log; exit 1; }
  echo "tail=$t $(grep -o '"errors": [0-9]*' gpurun_out/${T}_hapi_tail$t.log | tr '\n' ' ') $(grep -o '"stereo_frame": {"frames_per_s": [0-9.]*' gpurun_out/${T}_hapi_tail$t.log)"
done
