# r5cl: k_quadtree at 512 / 128 threads per workgroup (ORBX_QT_THREADS builds) against 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_LIB=build/qt512/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cl_pytest.log 2>&1 || { tail -30 gpurun_out/r5cl_pytest.log; exit 1; }
tail -1 gpurun_out/r5cl_pytest.log
ORBX_LIB=build/qt128/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cl_pytest128.log 2>&1 || { tail -30 gpurun_out/r5cl_pytest128.log; exit 1; }
tail -1 gpurun_out/r5cl_pytest128.log
ROUNDS=2 bash scripts/ab_envs.sh r5clab "t256||product" "t512||build/qt512/liborbx.so" "t128||build/qt128/liborbx.so"
