# bench.py lines for every BASELINE config (c1..c5) with the current library;
# c3 also with the CPU baseline (1-process + P-process legs).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/cfg2
mkdir -p $O
: > $O/lines.jsonl
for cfg in c1 c2 c3 c4 c5; do
  extra="--no-cpu-baseline"
  [ $cfg = c3 ] && extra="--cpu-seconds 8"
  timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 $extra > $O/$cfg.json 2> $O/$cfg.err || { tail -20 $O/$cfg.err; exit 1; }
  tail -n 1 $O/$cfg.json >> $O/lines.jsonl
done
python3 - <<'PY'
import json
for l in open('gpurun_out/cfg2/lines.jsonl'):
    d=json.loads(l)
    r=d['roofline']
    print(d['config']['workload'][:18], 'ms/step %.4f'%d['ms_per_step'], 'Gpx/s %.1f'%(d['value']/1e9), 'path frac %.3f'%r['frac'],
          'k_decode frac %.3f'%r['dominant_kernel']['frac'], {k: round(v*1e3,1) for k,v in d['path']['kernel_avg_ms'].items()})
PY
