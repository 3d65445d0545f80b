# Round 3, session 2: (1) the stack_ready / side-stream GPU tests + the
# multi-group and pool tests; (2) bench c2 with and without --stack-ready,
# twice interleaved; (3) the exact k_cloud ablation kbench (scripts/
# gpu_r3_kcloud_abl.sh).  -> gpurun_out/r3s2b, gpurun_out/r3kc
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pool.py -x -q --timeout 300 --timeout-method thread -k "stack_ready or launch_groups or three_launch or multigroup or pool or repeat or time_kernels" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/bench.log
for rep in 1 2; do
  for flag in --stack-ready --no-stack-ready; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary $flag > $O/bench$flag$rep.json 2> $O/bench$flag$rep.err || { tail -20 $O/bench$flag$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/bench$flag$rep.json').read().strip().splitlines()[-1])
t=d['timing']['step_us']
print('$flag', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], 'ev med %.1f min %.1f' % (t['median'], t['min']))
" | tee -a $O/bench.log
  done
done
bash scripts/gpu_r3_kcloud_abl.sh "$@"
