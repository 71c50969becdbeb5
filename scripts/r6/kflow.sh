# r6zd: the stream priority range, then the keyframe stream at the lowest priority against normal
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 -c "
import torch
print('torch priority_range', torch.cuda.Stream.priority_range())
s = torch.cuda.Stream(priority=1); print('priority=1 ->', s.priority)
s = torch.cuda.Stream(priority=-1); print('priority=-1 ->', s.priority)
" || exit 1
ROUNDS=${ROUNDS:-3} bash scripts/ab_envs.sh ${TAG:-r6zd}ab "kf0||product" "kflow|ORBX_KF_PRIORITY=1|product"
