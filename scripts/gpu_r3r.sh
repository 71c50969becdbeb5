set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_vocab.py tests/test_gpu_fusion.py tests/test_gpu_cd.py tests/test_gpu_match.py tests/test_stereo_refine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3r_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/r3r_pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r3r_pytest.log; exit $rc; }
timeout -k 10 200 python -u scripts/micro/vocab_agg.py > gpurun_out/r3r_vocab_agg.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3r_vocab_agg.log
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 30"
for v in wide small wide small; do
  if [ $v = wide ]; then export ORBX_VOCAB_AGG_WIDE=1; else unset ORBX_VOCAB_AGG_WIDE; fi
  timeout -k 10 300 python -u bench.py $B > gpurun_out/r3r_$v.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3r_$v.log').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']
print('$v', d['value'], d['ms_per_step'], 'kf', s['keyframe_bow_fusion'], 'tri', s.get('keyframe_new_mappoints'))"
done
bash scripts/kt_serial.sh r3r_kts | grep -E "k_stereo|k_vocab|second half"
