# Round-2 evidence refresh: GPU tests; the default bench command under
# rocprofv3 --kernel-trace --stats; PMC FETCH_SIZE / WRITE_SIZE passes
# (separate runs) of the C2 step's kernels -> per-step HBM bytes; the bench
# line reading that traffic file; then every config.  -> gpurun_out/fin
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/fin
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/bench_kernel_stats.csv
APP="python -u scripts/kbench.py --reps 10 --fast --only maps+cloud"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- $APP > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- $APP > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python3 scripts/traffic_from_pmc.py $O/fetch $O/write c2 1 fast 1 $O/traffic_c2.json > /dev/null || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --traffic $O/traffic_c2.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
: > $O/configs.jsonl
for cfg in c1 c3 c4 c5; do
  extra="--no-cpu-baseline"
  [ $cfg = c3 ] && extra="--cpu-seconds 8"
  steps=20
  [ $cfg = c1 ] && steps=400  # a 25-us step: enough steps that host jitter averages out
  timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 5 $extra > $O/$cfg.json 2> $O/$cfg.err || { tail -20 $O/$cfg.err; exit 1; }
  tail -n 1 $O/$cfg.json >> $O/configs.jsonl
done
tail -n 1 $O/bench.json >> $O/configs.jsonl
python3 - <<'PY'
import json, csv
for l in open('gpurun_out/fin/configs.jsonl'):
    d=json.loads(l)
    r=d['roofline']
    print(d['config']['workload'][:18], 'ms/step %.4f'%d['ms_per_step'], 'Gpx/s %.1f'%(d['value']/1e9), 'path frac %.3f'%r['frac'],
          'k_decode frac %.3f'%r['dominant_kernel']['frac'], {k: round(v*1e3,1) for k,v in d['path']['kernel_avg_ms'].items()})
for r in csv.DictReader(open('gpurun_out/fin/bench_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>4} {r['Name'][:70]}")
PY
