# Kernel traces of the bench at --emulate-agents 1 and 8 (which kernels grow with the ring's agent load).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-emuprof}
O=gpurun_out/$TAG; rm -rf $O; mkdir -p $O
for n in 1 8; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/n$n" -o run -- python3 $R/bench.py --emulate-agents $n \
      --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 --alone-reps 0 > $O/n$n.log 2>&1 || { echo "n=$n failed"; tail -3 $O/n$n.log; exit 1; }
  python3 scripts/kernel_share.py $O/n$n/run_kernel_trace.csv ${TAG}_n$n 28 --batch-images 512 --out $O/share_n$n.json || exit 1
done
python3 - <<PY
import json
a=json.load(open("$O/share_n1.json")); b=json.load(open("$O/share_n8.json"))
ka={k["kernel"]:k for k in a["kernels"]}; kb={k["kernel"]:k for k in b["kernels"]}
rows=[]
for n in set(ka)|set(kb):
    x=ka.get(n,{}).get("ms_per_step",0); y=kb.get(n,{}).get("ms_per_step",0)
    rows.append((y-x,n,x,y,ka.get(n,{}).get("launches_per_step",0),kb.get(n,{}).get("launches_per_step",0)))
for d,n,x,y,la,lb in sorted(rows,reverse=True)[:18]: print(f"{n:40s} {x:8.4f} -> {y:8.4f} ms/step  launches {la} -> {lb}")
print("gpu busy", a["gpu_busy_ms_per_step"], b["gpu_busy_ms_per_step"])
PY
