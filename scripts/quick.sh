# Quick GPU iteration: extractor parity tests, then the default bench without the CPU / C3 / host-API legs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-q}; TESTS=${2:-tests/test_gpu_extract.py}
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
echo "bench rc=$rc"
python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${TAG}_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('host_enqueue_split_ms'), d.get('stage_ms_per_step'))"
exit $rc
