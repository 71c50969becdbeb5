set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k bf \
    > gpurun_out/r5f_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5f_pytest.log
[ $rc -eq 0 ] || exit $rc
for e in "ORBX_BF_FUSED=0" "ORBX_BF_FUSED=1" "ORBX_BF_FUSED=1 ORBX_BF_WGS=512" "ORBX_BF_FUSED=1 ORBX_BF_WGS=256" "ORBX_BF_FUSED=1 ORBX_BF_WGS=128" "ORBX_BF_FUSED=0 ORBX_BF_WGS=512"; do
  echo "$e $(env $e timeout -k 10 120 python3 scripts/micro/c3_only.py 1 2>/dev/null | tr "\n" " ")" || exit 1
done
