# adaptive vs fixed mask at config 2 (the fixed mask runs no k_stats): the
# upper bound of what overlapping k_stats could save
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/kfix
mkdir -p $O
timeout -k 10 120 python -u scripts/kbench.py --reps 50 --fast --only maps+cloud > $O/a.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/kbench.py --reps 50 --fast --only "maps+cloud fixed" > $O/f.log 2>&1 || exit 1
cat $O/a.log $O/f.log | grep '"variant": "maps' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print({k:(round(v,1) if isinstance(v,float) else v) for k,v in d.items() if k in ('variant','count_us','decode_us','cloud_us','total_us','host_us_per_call','wall_us_per_call')})"
