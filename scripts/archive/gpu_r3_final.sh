# Round 3 evidence at HEAD: the default bench as the first GPU command on a
# fresh box (the driver's condition), the full GPU suite, the default bench
# under rocprofv3 --kernel-trace --stats, the calibrated PMC traffic of the
# c2 step, and the config lines c1 / c3 / c4 / c5 at BASELINE scale.  -> gpurun_out/r3final
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_first.json 2> $O/bench_first.err || { tail -20 $O/bench_first.err; exit 1; }
tail -c 400 $O/bench_first.json; echo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/c2_kernel_stats.csv
rm -rf $O/trace
bash scripts/gpu_r3_traffic.sh || exit 1
for cfg in c1 c3 c4 c5; do
  extra=""
  [ $cfg = c3 ] && extra="--scaling strong"
  timeout -k 10 600 python -u bench.py --config $cfg $extra --cpu-seconds 8 > $O/$cfg.json 2> $O/$cfg.err || { tail -20 $O/$cfg.err; exit 1; }
  tail -n 1 $O/$cfg.json >> $O/config_lines.jsonl
done
python3 - <<'PY'
import json, csv
O = 'gpurun_out/r3final'
for n in ('bench_first', 'bench_traced'):
    d = json.loads(open(f'{O}/{n}.json').read().strip().splitlines()[-1])
    print(n, 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'],
          'k_decode frac %.3f' % d['roofline']['dominant_kernel']['frac'])
for r in csv.DictReader(open(f'{O}/c2_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>5} {r['Name'][:60]}")
for l in open(f'{O}/config_lines.jsonl'):
    d = json.loads(l)
    print(d['config']['workload'][:24], 'ms %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'])
PY
