# r5cj: k_fast_wave with 2 / 8 waves per workgroup (ORBX_FAST_WPG builds) against 4 under the current schedule
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_LIB=build/wpg2/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cj_pytest.log 2>&1 || { tail -30 gpurun_out/r5cj_pytest.log; exit 1; }
tail -1 gpurun_out/r5cj_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5cjab "w4||product" "w2||build/wpg2/liborbx.so" "w8||build/wpg8/liborbx.so"
