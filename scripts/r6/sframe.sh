# r6zr: orbx_stereo_frame -- the stereo tests, then the host-API legs of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6zr}
timeout -k 10 400 python -u -m pytest tests/test_stereo_refine.py tests/test_gpu_extract.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 3 --cpu-seconds 0 --no-c3 --no-cd --host-fed-steps 0 > gpurun_out/${T}_bench.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.log; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1]); h=d['host_api']
print('py pair', h['frames_per_s'], h['latency_ms_median'], 'py frame', h['stereo_frame']['frames_per_s'], h['stereo_frame']['latency_ms_median'])
n=h['native']; print('native 2thr', n['frames_per_s'], 'pair', n['pair']['frames_per_s'], 'frame', n['stereo_frame'])"
