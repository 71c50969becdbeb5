# r6r: k_fast_wave LDS attribution -- one SQ PMC pass per build: the product and the
# ORBX_FAST_ATTR diagnostics builds (1: score taps, 2: NMS reads, 3: both at conflict-free addresses; wrong keypoints),
# then the serial FAST time of each (bench roofline_alone).  Summary: scripts/r6/fattr_sum.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6r}; O=gpurun_out/$T; rm -rf $O; mkdir -p $O
B="bench.py --steps 4 --warmup 2 --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --alone-reps 0"
for v in product fattr1 fattr2 fattr3; do
  if [ $v = product ]; then unset ORBX_LIB; else export ORBX_LIB=$R/build/$v/liborbx.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
      SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $R/$O/$v -o run -- python3 $B > $O/$v.log 2>&1 \
      || { echo "$v pmc failed"; tail -5 $O/$v.log; exit 1; }
  echo "$v pmc ok"
done
unset ORBX_LIB
python3 scripts/r6/fattr_sum.py $O || exit 1
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "base||product" "fattr1||$R/build/fattr1/liborbx.so" \
  "fattr2||$R/build/fattr2/liborbx.so" "fattr3||$R/build/fattr3/liborbx.so"
