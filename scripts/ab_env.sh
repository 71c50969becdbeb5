# A/B of extractor variants selected by environment (one bench run each, short, no CPU baseline).
# usage: bash scripts/ab_env.sh TAG "ENV1" "ENV2" ...   (each ENV a space-separated list of VAR=VALUE)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --host-api-frames 0 \
      > gpurun_out/${TAG}_ab$i.log 2>&1 || { echo "run $i ($cfg) failed"; tail -5 gpurun_out/${TAG}_ab$i.log; exit 1; }
  python3 - "$cfg" gpurun_out/${TAG}_ab$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"{sys.argv[1]:50s} {d['value']:9.0f} fps {d['ms_per_step']:.3f} ms/step host {d['host_enqueue_ms_per_step']:.3f} " +
      " ".join(f"{k}={v:.3f}" for k, v in d.get("stage_ms_per_step", {}).items()))
PY
done
