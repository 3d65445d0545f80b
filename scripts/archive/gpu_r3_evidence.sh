# Round-3 evidence at HEAD (pre-stats default): the default bench as the first
# GPU command on a fresh box, the default bench under rocprofv3 --kernel-trace
# --stats, the calibrated PMC traffic of the bench's steady state.  -> gpurun_out/r3ev
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3ev
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_first.json 2> $O/bench_first.err || { tail -20 $O/bench_first.err; exit 1; }
tail -c 300 $O/bench_first.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/c2_kernel_stats.csv
rm -rf $O/trace
bash scripts/gpu_r3_traffic.sh || exit 1
cp gpurun_out/r3traffic/traffic_c2.json $O/traffic_c2.json
python3 - <<'PY'
import json, csv
O = 'gpurun_out/r3ev'
for n in ('bench_first', 'bench_traced'):
    d = json.loads(open(f'{O}/{n}.json').read().strip().splitlines()[-1])
    print(n, 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'],
          'k_decode frac %.3f' % d['roofline']['dominant_kernel']['frac'], 'median us %.1f' % d['timing']['step_us']['median'])
for r in csv.DictReader(open(f'{O}/c2_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>5} {r['Name'][:60]}")
PY
