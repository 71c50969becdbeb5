# k_fast_band persistent walk A/B: parity at two grid shapes, then serial and pipelined bench per ORBX_FAST_PERSIST
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 0 64; do
  ORBX_FAST_PERSIST=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n_pytest_$p.log 2>&1; rc=$?
  echo "pytest persist=$p rc=$rc $(tail -1 gpurun_out/r3n_pytest_$p.log)"; [ $rc -eq 0 ] || exit $rc
done
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 20"
for p in ${PERSIST_LIST:-0 40 80 120 160}; do
  ORBX_FAST_PERSIST=$p ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3n_s$p.log 2>&1 || exit $?
  ORBX_FAST_PERSIST=$p timeout -k 10 300 python -u bench.py $B > gpurun_out/r3n_p$p.log 2>&1 || exit $?
  python3 - $p <<'PY'
import json, sys
p = sys.argv[1]
s = json.loads(open(f"gpurun_out/r3n_s{p}.log").read().strip().splitlines()[-1])
q = json.loads(open(f"gpurun_out/r3n_p{p}.log").read().strip().splitlines()[-1])
st = s["stage_ms_per_step"]
print(f"persist {p}: serial fast {st['fast_cells'] + st['fast_cells_l0']:.3f} ms ({st['fast_cells_l0']:.3f} l0), serial value {s['value']}, pipelined {q['value']} ({q['ms_per_step']} ms)")
PY
done
