set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_vocab.py tests/test_gpu_fusion.py tests/test_gpu_kfdb.py tests/test_gpu_cd.py tests/test_multiagent.py tests/test_gpu_new_mappoints.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3q_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/r3q_pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r3q_pytest.log; exit $rc; }
bash scripts/kt_serial.sh r3q_kts
