set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r5e}
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do for e in 0 1; do
  echo "fused=$e $(ORBX_BF_FUSED=$e timeout -k 10 120 python3 scripts/micro/c3_only.py 2 2>/dev/null | tr "\n" " ")" || exit 1
done; done
