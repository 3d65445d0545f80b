# Round 3: one bench line per BASELINE config at the configs' own scale (c4 /
# c5: 45 views per GPU = the per-GPU share of the 360-view scan on 8 GPUs;
# c3: the 36-view scan, strong scaling), each followed by rocprofv3
# --kernel-trace --stats of the same command (no CPU baseline, no secondary
# lines).  CONFIGS="c1 c3 ..." picks configs.  -> gpurun_out/r3cfg
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3cfg
mkdir -p $O
: > $O/lines.jsonl
for cfg in ${CONFIGS:-c1 c3 c4 c5}; do
  extra=""
  steps=20
  case $cfg in
    c1) steps=400; extra="--cpu-seconds 8" ;;
    c3) extra="--scaling strong --cpu-seconds 8" ;;
    c4|c5) extra="--cpu-seconds 10" ;;
  esac
  timeout -k 10 900 python -u bench.py --config $cfg --steps $steps --warmup 5 $extra > $O/$cfg.json 2> $O/$cfg.err || { tail -20 $O/$cfg.err; exit 1; }
  tail -n 1 $O/$cfg.json >> $O/lines.jsonl
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$cfg -o t -- python -u bench.py --config $cfg --steps $steps --warmup 5 $extra --no-cpu-baseline --no-secondary > $O/${cfg}_traced.json 2> $O/${cfg}_traced.err || { tail -20 $O/${cfg}_traced.err; exit 1; }
  f=$(find $O/trace_$cfg -name '*kernel_stats.csv' | head -1)
  cp "$f" $O/${cfg}_kernel_stats.csv
  rm -rf $O/trace_$cfg
  python3 - "$O" "$cfg" <<'PY'
import json, csv, sys
O, cfg = sys.argv[1], sys.argv[2]
d = json.loads(open(f'{O}/{cfg}.json').read().strip().splitlines()[-1])
r = d['roofline']
t = d['timing']['step_us']
cb = d.get('cpu_baseline') or {}
print(cfg, d['config']['workload'][:60], '| ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9),
      'path %.3f' % r['frac'], 'k_decode %.3f' % r['dominant_kernel']['frac'], 'ev_med %.1f' % t['median'],
      'cpu %.2f Mpx/s' % (cb.get('value', 0) / 1e6), 'cpu_mp %.1f Mpx/s' % ((cb.get('multi_process') or {}).get('value', 0) / 1e6))
for row in csv.DictReader(open(f'{O}/{cfg}_kernel_stats.csv')):
    if 'k_' in row['Name']:
        print(f"   {float(row['AverageNs'])/1e3:9.2f} us x{row['Calls']:>5} {row['Name'][:70]}")
PY
done
