# Round 3, first GPU session: the default bench as the FIRST GPU command on a
# fresh box (the driver's condition: does the pre-roll remove the round-2
# stall?), the GPU suite, the f32-fast line, the default bench under
# rocprofv3 --kernel-trace --stats, PMC FETCH/WRITE of the exact step (->
# r03 traffic file), and the SQ counters of k_cloud exact vs fast.
# -> gpurun_out/r3a
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 240 python -u bench.py > $O/bench_first.json 2> $O/bench_first.err || { tail -20 $O/bench_first.err; exit 1; }
tail -c 300 $O/bench_first.json; echo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/bench_second.json 2> $O/bench_second.err || { tail -20 $O/bench_second.err; exit 1; }
timeout -k 10 120 python -u bench.py --no-cpu-baseline --xyz fast > $O/bench_fast.json 2> $O/bench_fast.err || { tail -20 $O/bench_fast.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/bench_kernel_stats.csv
APP="python -u scripts/kbench.py --reps 10 --only maps+cloud"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- $APP > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- $APP > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python3 scripts/traffic_from_pmc.py $O/fetch $O/write c2 1 exact 1 $O/traffic_c2.json > /dev/null || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_FLAT"; do
  i=$((i+1))
  for mode in exact fast; do
    extra=""
    [ $mode = fast ] && extra="--fast"
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/sq_$mode/p$i -o p -- python -u scripts/kbench.py --reps 5 --only maps+cloud $extra > $O/sq_${mode}_$i.log 2>&1 || { echo "pmc $mode $i failed"; tail -5 $O/sq_${mode}_$i.log; exit 1; }
  done
done
for mode in exact fast; do
  echo "== $mode"
  python3 scripts/pmc_summary.py $O/sq_$mode > $O/sq_$mode.txt
  grep -A40 "k_cloud" $O/sq_$mode.txt | head -40
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --traffic $O/traffic_c2.json > $O/bench_traffic.json 2> $O/bench_traffic.err || { tail -20 $O/bench_traffic.err; exit 1; }
python3 - <<'PY'
import json, csv
O = 'gpurun_out/r3a'
for n in ('bench_first', 'bench_second', 'bench_fast', 'bench_traced', 'bench_traffic'):
    d = json.loads(open(f'{O}/{n}.json').read().strip().splitlines()[-1])
    t = d.get('timing', {})
    print(n, 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value'] / 1e9), 'frac %.3f' % d['roofline']['frac'],
          'step_us', {k: round(v, 1) for k, v in (t.get('step_us') or {}).items() if k != 'steps'},
          'no_ev %.4f' % t.get('ms_per_step_no_events', 0), 'kern', {k: round(v * 1e3, 1) for k, v in d['path']['kernel_avg_ms'].items()})
for r in csv.DictReader(open(f'{O}/bench_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>4} {r['Name'][:70]}")
PY
