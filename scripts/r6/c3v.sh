# r6l: k_bf_mfma with 4 query tiles per wave (ORBX_MX_QT builds): matcher tests, C3 block; the default (2) for reference
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6l}
ORBX_LIB=build/mxqt4/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k bf > gpurun_out/${T}_pytest_qt4.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest_qt4.log; [ $rc -eq 0 ] || exit $rc
for v in 4 1; do
  ORBX_LIB=build/mxqt$v/liborbx.so timeout -k 10 300 python -u scripts/micro/c3_only.py 1 > gpurun_out/${T}_c3_qt$v.log 2>&1 || exit 1
  echo "qt$v $(tail -1 gpurun_out/${T}_c3_qt$v.log)"
done
timeout -k 10 300 python -u scripts/micro/c3_only.py 1 > gpurun_out/${T}_c3_qt2.log 2>&1 || exit 1
echo "qt2 $(tail -1 gpurun_out/${T}_c3_qt2.log)"
