# r6s: kernel trace + stats of the bench step at 1 and 8 emulated agents (which keyframe-path kernels grow)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6s}; O=gpurun_out/$T; rm -rf $O; mkdir -p $O
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --alone-reps 0"
for n in 1 8; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/emu$n -o run -- python3 $B --emulate-agents $n \
      > $O/emu$n.log 2>&1 || { echo "emu$n failed"; tail -5 $O/emu$n.log; exit 1; }
  echo "emu$n ok"
done
