# kbench --fast (maps+cloud, cloud) for k_decode occupancy variants of the
# decide path: default, yn from global, 3 waves/SIMD at 3 workgroups per CU.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/kdv
mkdir -p $O
: > $O/kb.log
run() {  # label, env...
  local label=$1; shift
  for only in "maps+cloud" "cloud"; do
    env "$@" timeout -k 10 120 python -u scripts/kbench.py --reps 30 --fast --only "$only" | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$label\"/" >> $O/kb.log 2>&1 || return 1
  done
}
run default SLGPU_PATH=0 || exit 1
run 3k SLGPU_PATH=3 || exit 1
run yng SLGPU_LIB=$PWD/build/libslgpu_yng.so || exit 1
run w3_cu3 SLGPU_LIB=$PWD/build/libslgpu_w3.so SLGPU_DECODE_PER_CU=3 || exit 1
run w3_cu2 SLGPU_LIB=$PWD/build/libslgpu_w3.so SLGPU_DECODE_PER_CU=2 || exit 1
run default_cu1 SLGPU_DECODE_PER_CU=1 || exit 1
grep variant $O/kb.log | grep -v torch_copy | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'][:10].ljust(10), d['lib'][:14].ljust(14), 'decode %.1f'%d['decode_us'], 'count/stats %.1f'%d['count_us'], 'cloud %.1f'%d['cloud_us'], 'wall %.1f'%d['wall_us_per_call'])"
