# r5cf: k_fast_wave with the u8 score map (ORBX_FAST_U8SC=1 build, 1.3 KB less LDS per wave) under the current schedule
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_LIB=build/u8sc/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cf_pytest.log 2>&1 || { tail -30 gpurun_out/r5cf_pytest.log; exit 1; }
tail -1 gpurun_out/r5cf_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5cfab "i16||product" "u8||build/u8sc/liborbx.so"
