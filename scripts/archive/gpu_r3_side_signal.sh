# Round 3: the side-stream histogram pass with stream memory operations
# (SLGPU_SIDE_SIGNAL=1) instead of events: the stack_ready tests under it,
# then c2 bench --stack-ready (signal / events) vs the default, interleaved,
# and a kernel trace of the signal variant.  -> gpurun_out/r3sig
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3sig
mkdir -p $O
SLGPU_SIDE_SIGNAL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stack_ready or launch_groups or three_launch or multigroup" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
SLGPU_SIDE_SIGNAL=1 SLGPU_STATS_SIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "launch_groups or three_launch or multigroup" > $O/pytest_groups.log 2>&1 || { tail -40 $O/pytest_groups.log; exit 1; }
tail -1 $O/pytest_groups.log
: > $O/lines.log
for rep in 1 2; do
  for spec in "0|--no-stack-ready" "1|--stack-ready" "0|--stack-ready"; do
    IFS='|' read -r sig flag <<< "$spec"
    SLGPU_SIDE_SIGNAL=$sig timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary $flag > $O/b_$sig$flag$rep.json 2> $O/b_$sig$flag$rep.err || { tail -20 $O/b_$sig$flag$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_$sig$flag$rep.json').read().strip().splitlines()[-1])
t=d['timing']['step_us']
print('signal=$sig $flag', 'us/step %.2f' % (1e3*d['ms_per_step']), 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], 'ev med %.1f' % t['median'])
" | tee -a $O/lines.log
  done
done
SLGPU_SIDE_SIGNAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o t -- python -u bench.py --steps 20 --warmup 5 --preroll-ms 30 --no-cpu-baseline --no-secondary --stack-ready > $O/traced.json 2> $O/traced.err || { tail -20 $O/traced.err; exit 1; }
f=$(find $O/t -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_steps.py "$f" > $O/steps.txt || exit 1
rm -rf $O/t
tail -22 $O/steps.txt
