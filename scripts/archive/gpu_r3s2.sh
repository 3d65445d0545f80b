# Round 3, session 2: the default bench first on a fresh box, the GPU suite
# (incl. the verified-route tests), a same-box kbench A/B of the exact k_cloud
# (SLGPU_VERIFY32=1 verified shorter route vs 0 the exact sequence), and the
# default bench under rocprofv3 --kernel-trace --stats.  -> gpurun_out/r3s2
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2
mkdir -p $O
timeout -k 10 240 python -u bench.py > $O/bench_first.json 2> $O/bench_first.err || { tail -20 $O/bench_first.err; exit 1; }
tail -c 300 $O/bench_first.json; echo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
: > $O/kb.log
for rep in 1 2 3; do
  for v in 1 0; do
    SLGPU_VERIFY32=$v timeout -k 10 120 python -u scripts/kbench.py --reps 30 --preroll-ms 300 --only maps+cloud 2>&1 | grep variant | grep -v torch_copy | sed "s/^{/{\"label\": \"verify$v\", /" >> $O/kb.log || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/bench_kernel_stats.csv
rm -rf $O/trace
python3 - <<'PY'
import json, csv, collections
O = 'gpurun_out/r3s2'
rows = collections.defaultdict(list)
for l in open(f'{O}/kb.log'):
    d = json.loads(l)
    rows[d['label']].append(d)
for lab, ds in rows.items():
    f = lambda k: ' '.join('%.1f' % d[k] for d in ds)
    g = lambda k: ' '.join('%.1f' % d['rerun_us'][k] for d in ds)
    print(lab, 'stats', f('count_us'), '| decode', f('decode_us'), '| cloud', f('cloud_us'), '| rerun cloud', g('cloud'), '| wall', f('wall_us_per_call'))
for n in ('bench_first', 'bench_traced'):
    d = json.loads(open(f'{O}/{n}.json').read().strip().splitlines()[-1])
    t = d.get('timing', {})
    print(n, 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'],
          'step_us', {k: round(v, 1) for k, v in (t.get('step_us') or {}).items() if k != 'steps'},
          'kern', {k: round(v * 1e3, 1) for k, v in d['path']['kernel_avg_ms'].items()})
for r in csv.DictReader(open(f'{O}/bench_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>4} {r['Name'][:70]}")
PY
