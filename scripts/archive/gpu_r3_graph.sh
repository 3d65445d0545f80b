# The headline window as one hipGraph launch (bench default) vs eager calls:
# pre-stats tests (incl. the graph-captured chain), then the driver's command
# repeatedly (first process on the box first), alternating.  -> gpurun_out/r3graph
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3graph
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/first_graph.json 2> $O/first_graph.err || { tail -20 $O/first_graph.err; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prestats.py > $O/pytest_prestats.log 2>&1 || { tail -40 $O/pytest_prestats.log; exit 1; }
tail -1 $O/pytest_prestats.log
for rep in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/graph_$rep.json 2> $O/graph_$rep.err || { tail -20 $O/graph_$rep.err; exit 1; }
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-graph > $O/eager_$rep.json 2> $O/eager_$rep.err || { tail -20 $O/eager_$rep.err; exit 1; }
done
timeout -k 10 200 python3 -u bench.py --config c1 --streams 1 --no-cpu-baseline --no-secondary > $O/c1s1_graph.json 2> $O/c1s1_graph.err || { tail -20 $O/c1s1_graph.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --config c1 --streams 1 --no-cpu-baseline --no-secondary --no-graph > $O/c1s1_eager.json 2> $O/c1s1_eager.err || { tail -20 $O/c1s1_eager.err; exit 1; }
python3 - <<'PY'
import json, glob
O = 'gpurun_out/r3graph'
for f in sorted(glob.glob(f'{O}/*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    t = d['timing']
    print(f.split('/')[-1][:-5].ljust(14), 'us/step %.2f' % (1e3 * d['ms_per_step']), 'frac %.3f' % d['roofline']['frac'],
          'enq ms %.3f' % t['host_enqueue_ms'], 'event-median %.1f' % t['step_us']['median'], t['window']['mode'][:40])
PY
