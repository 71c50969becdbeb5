# Alternating A/B of env settings (or library builds) on the default bench without the CPU / C3 / host-API / CD /
# host-fed legs (roofline_alone kept).  Each argument is "name|ENV=1 ENV2=x|lib[|bench args]" (lib: product or a path); every
# configuration runs ROUNDS times in the order A B C A B C ...
# usage: ROUNDS=2 bash scripts/ab_envs.sh TAG "base||product" "pair|ORBX_RESIZE_PAIR=1|product" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
TAG=$1; shift
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for cfg in "$@"; do
    name=${cfg%%|*}; rest=${cfg#*|}; envs=${rest%%|*}; lib=${rest#*|}
    xa=""; case "$lib" in *"|"*) xa=${lib#*|}; lib=${lib%%|*};; esac   # optional 4th field: extra bench arguments
    L=""; [ "$lib" != product ] && [ -n "$lib" ] && L="ORBX_LIB=$lib"
    log=gpurun_out/${TAG}_${name}_r$r.log
    env $L $envs timeout -k 10 200 python bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 \
        $AB_ARGS $xa > $log 2>&1 || { echo "[$name] failed"; tail -5 $log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
a=d.get('roofline_alone',{}).get('stage_ms_alone',{}); s=d.get('stage_ms_per_step',{})
print('r$r %-8s' % '$name', d['value'], d['ms_per_step'], 'fast_busy_live', s.get('fast_busy'), 'blur_live', s.get('blur7'), 'alone', {k: round(v, 3) for k, v in a.items() if k in ('fast_busy', 'blur7', 'describe', 'resize')}, 'fuse', s.get('keyframe_fuse'), 'trk', s.get('tracking_match'))"
  done
done
