# FAST phase ablation: serial pipeline (every stage alone on one stream), front end only, with the stop-after-phase
# diagnostic builds (make variant V=stopK D=-DORBX_FAST_STOP=K) beside the product library.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for v in product stop1 stop2 stop3 stop4; do
  L=""; [ $v != product ] && L="ORBX_LIB=build/$v/liborbx.so"
  env $L ORBX_PIPELINE=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-c3 --host-api-frames 0 --diag-skip stereo > gpurun_out/fs_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/fs_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/fs_$v.log').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['ms_per_step'], 'fast', round(s['fast_cells'],3), 'fast_l0', round(s['fast_cells_l0'],3))"
done
