# Pre-stats (sl_stack_next): its GPU tests, then same-box bench A/Bs (next-stats
# on / off, alternating) at c2 and c1, and the c2 bench under rocprofv3
# kernel stats.  -> gpurun_out/r3pre
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3pre
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prestats.py > $O/pytest_prestats.log 2>&1 || { tail -40 $O/pytest_prestats.log; exit 1; }
tail -1 $O/pytest_prestats.log
for rep in 1 2 3; do
  for mode in --next-stats --no-next-stats; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary $mode > $O/c2_$rep$mode.json 2> $O/c2_$rep$mode.err || { tail -20 $O/c2_$rep$mode.err; exit 1; }
  done
done
for rep in 1 2; do
  SLGPU_DECODE_BALANCE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary > $O/c2_bal_$rep.json 2> $O/c2_bal_$rep.err || { tail -20 $O/c2_bal_$rep.err; exit 1; }
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary > $O/c2_def_$rep.json 2> $O/c2_def_$rep.err || { tail -20 $O/c2_def_$rep.err; exit 1; }
done
for mode in --next-stats --no-next-stats; do
  timeout -k 10 200 python -u bench.py --config c1 --no-cpu-baseline --no-secondary $mode > $O/c1$mode.json 2> $O/c1$mode.err || { tail -20 $O/c1$mode.err; exit 1; }
  timeout -k 10 200 python -u bench.py --config c1 --streams 1 --no-cpu-baseline --no-secondary $mode > $O/c1s1$mode.json 2> $O/c1s1$mode.err || { tail -20 $O/c1s1$mode.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/c2_kernel_stats.csv
rm -rf $O/trace
python3 - <<'PY'
import json, csv, glob
O = 'gpurun_out/r3pre'
for f in sorted(glob.glob(f'{O}/*.json')):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    k = d['path']['kernel_avg_ms']
    print(f.split('/')[-1][:-5].ljust(22), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'med %.1f' % d['timing']['step_us']['median'], ' '.join('%s %.1f' % (n, 1e3 * v) for n, v in k.items()))
for r in csv.DictReader(open(f'{O}/c2_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>5} {r['Name'][:60]}")
PY
