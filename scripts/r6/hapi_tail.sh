set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for r in 1 2; do for t in 0 3 4 5; do
  if [ $t = 0 ]; then E=""; else E="ORBX_RESIZE_TAIL=$t"; fi
  env $E timeout -k 10 120 build/host_api_bench multiagent_orb_slam2_amd/liborbx.so 400 > gpurun_out/r7r_tail${t}_$r.log 2>&1 || { tail -3 gpurun_out/r7r_tail${t}_$r.log; exit 1; }
  echo "tail=$t round $r: $(tail -c 400 gpurun_out/r7r_tail${t}_$r.log | tr '\n' ' ' | cut -c1-380)"
done; done
