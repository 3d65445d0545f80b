# bench.py lines for configs c1, c3, c4, c5 (and c2) on the default path and on
# the three-kernel path (SLGPU_PATH=3); no CPU baseline.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cab
mkdir -p $O
: > $O/lines.jsonl
for cfg in c1 c2 c3 c4 c5; do
  for path in default 3; do
    SLGPU_PATH=$path timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/$cfg.$path.json 2> $O/$cfg.$path.err || exit $?
    python3 -c "
import json,sys
d=json.loads(open('$O/$cfg.$path.json').read().strip().splitlines()[-1])
d['path_variant']='$path'
print(json.dumps(d))" >> $O/lines.jsonl
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/cab/lines.jsonl'):
    d=json.loads(l)
    print(d['config']['workload'][:17], d['path_variant'].ljust(8), 'ms/step %.4f'%d['ms_per_step'], 'Gpx/s %.1f'%(d['value']/1e9), 'path %.0f GB/s'%d['path']['GBps'], {k: round(v*1e3,1) for k,v in d['path']['kernel_avg_ms'].items()})
PY
