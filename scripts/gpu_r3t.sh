# FAST phase 3a (opposite-tap test before scores) A/B: parity, then serial and pipelined bench, default vs ORBX_FAST_OPP=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3t_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/r3t_pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r3t_pytest.log; exit $rc; }
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 30"
for v in opp noopp opp noopp; do
  L=""; [ $v = noopp ] && L=build/noopp/liborbx.so
  ORBX_LIB=$L ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3t_${v}_s.log 2>&1 || exit $?
  ORBX_LIB=$L timeout -k 10 300 python -u bench.py $B > gpurun_out/r3t_${v}_p.log 2>&1 || exit $?
  python3 -c "
import json
s=json.loads(open('gpurun_out/r3t_${v}_s.log').read().strip().splitlines()[-1]); p=json.loads(open('gpurun_out/r3t_${v}_p.log').read().strip().splitlines()[-1])
st=s['stage_ms_per_step']
print('$v serial fast %.3f (l0 %.3f) value %s | pipelined %s %s ms' % (st['fast_cells']+st['fast_cells_l0'], st['fast_cells_l0'], s['value'], p['value'], p['ms_per_step']))"
done
