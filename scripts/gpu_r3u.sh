# k_fast_wave (one wave per cell) A/B: parity of every FAST form, then serial and pipelined bench, band vs wave (4 and 1
# waves per workgroup)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r3u}
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py ${PYK:+-k "$PYK"} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/${TAG}_pytest.log; exit $rc; }
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 30"
for v in ${FORMS:-band wave wave2 wave1 wave}; do
  E="ORBX_FAST_WAVE=0"; [ $v = wave ] && E="ORBX_FAST_WAVE=1"; [ $v = wave1 ] && E="ORBX_FAST_WAVE=1 ORBX_FAST_WPG=1"; [ $v = wave2 ] && E="ORBX_FAST_WAVE=1 ORBX_FAST_WPG=2"; [ $v = fb ] && E="ORBX_FAST_WAVE=1 ORBX_DESC_FB=1"; [ $v = wave24 ] && E="ORBX_FAST_WAVE=1 ORBX_FAST_PSMIN=24"; [ $v = wave_b0 ] && E="ORBX_FAST_WAVE=1 ORBX_BLUR_DOT2=0"; [ $v = wave1p ] && E="ORBX_FAST_WAVE=1 ORBX_FAST_TWOPASS=0"; [ $v = wave20 ] && E="ORBX_FAST_WAVE=1 ORBX_FAST_PSMIN=20"; [ $v = band_b0 ] && E="ORBX_FAST_WAVE=0 ORBX_BLUR_DOT2=0"; [ $v = blds ] && E="ORBX_BLUR_LDS=1"; [ $v = blds16 ] && E="ORBX_BLUR_LDS=1 ORBX_LIB=build/b16/liborbx.so"; [ $v = qtt ] && E="ORBX_LIB=build/qtt/liborbx.so"; [ $v = prev ] && E="ORBX_LIB=build/prev/liborbx.so"; [ $v = k4 ] && E="ORBX_QT_KEYS0=4096"; [ $v = c2 ] && E="ORBX_FAST_CELLS=2"; [ $v = sel0 ] && E="ORBX_LIB=build/sel0/liborbx.so"; [ $v = pk0 ] && E="ORBX_LIB=build/pk0/liborbx.so"; [ $v = b24 ] && E="ORBX_LIB=build/b24/liborbx.so"; [ $v = b32 ] && E="ORBX_LIB=build/b32/liborbx.so"; [ $v = c4 ] && E="ORBX_FAST_CELLS=4"; [ $v = wpe5 ] && E="ORBX_LIB=build/wpe5/liborbx.so"; [ $v = wpe6 ] && E="ORBX_LIB=build/wpe6/liborbx.so"; [ $v = k3 ] && E="ORBX_QT_KEYS0=3072"; [ $v = k4b ] && E="ORBX_QT_KEYS0=4096 ORBX_QT_KEYS1=1024"; [ $v = def ] && E="ORBX_FAST_WAVE=1"; [ $v = sp0 ] && E="ORBX_SIDE_PRIORITY=0"; [ $v = mp1 ] && E="ORBX_MAIN_PRIORITY=-1 ORBX_SIDE_PRIORITY=0"; [ $v = mp1s ] && E="ORBX_MAIN_PRIORITY=-1"; [ $v = bmp1 ] && E="ORBX_BLUR_LDS=1 ORBX_MAIN_PRIORITY=-1 ORBX_SIDE_PRIORITY=0"
  env $E ORBX_PIPELINE=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_${v}_s.log 2>&1 || exit $?
  env $E timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_${v}_p.log 2>&1 || exit $?
  python3 -c "
import json
s=json.loads(open('gpurun_out/${TAG}_${v}_s.log').read().strip().splitlines()[-1]); p=json.loads(open('gpurun_out/${TAG}_${v}_p.log').read().strip().splitlines()[-1])
st=s['stage_ms_per_step']
print('$v serial resize %.3f fast %.3f (l0 %.3f) blur %.3f desc %.3f qt %.3f+%.3f value %s | pipelined %s %s ms' % (st.get('resize', 0), st['fast_cells']+st['fast_cells_l0'], st['fast_cells_l0'], st.get('blur7', 0), st.get('describe', 0), st.get('quadtree', 0), st.get('quadtree_l0', 0), s['value'], p['value'], p['ms_per_step']))"
done
# SQ counters of the serial step with k_fast_wave (one --pmc pass per counter set)
if [ -n "$SQ" ]; then
  export ORBX_FAST_WAVE=1 ORBX_PIPELINE=0 ORBX_FAST_WPG=${SQ}
  bash scripts/prof_sq.sh ${TAG}_sq --steps 5 --warmup 2 --no-c3 --no-cd --host-fed-steps 0 --host-api-frames 0 || exit $?
  python3 scripts/sq_summary.py gpurun_out/${TAG}_sq gpurun_out/${TAG}_sq_summary.json | head -8
fi
