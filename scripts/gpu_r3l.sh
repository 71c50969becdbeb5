set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3l_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r3l_pytest.log; [ $rc -eq 0 ] || exit $rc
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 20"
for v in dpp nodpp; do
  L=""; [ $v = nodpp ] && L=build/blur_nodpp/liborbx.so
  ORBX_LIB=$L ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3l_${v}_serial.log 2>&1 || exit $?
  ORBX_LIB=$L timeout -k 10 300 python -u bench.py $B > gpurun_out/r3l_${v}.log 2>&1 || exit $?
  echo "$v serial: $(grep -o '"value": [0-9.]*\|"blur7": [0-9.]*' gpurun_out/r3l_${v}_serial.log | tr '\n' ' ')  pipelined: $(grep -o '"value": [0-9.]*\|"blur7": [0-9.]*' gpurun_out/r3l_${v}.log | tr '\n' ' ')"
done
