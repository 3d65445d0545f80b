# Round 3: prepared calls (sl_call_prepare / sl_call_run) -- pool / parity GPU
# tests, then c1 at 6 and 1 views in flight and c3 / c5 lines (the pool path
# now re-runs a prepared call per lane), with the k_cloud cheap-x/y A/B vs
# HEAD~ (build/libslgpu_head.so).  -> gpurun_out/r3pc
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3pc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pool or prepared or verified or golden or full_4k or pose or synthetic or fused" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/lines.log
for rep in 1 2; do
  for spec in "c1" "c1 --streams 1" "c1 --streams 8" "c2"; do
    tag=$(echo "$spec" | tr ' ' '_')
    timeout -k 10 200 python -u bench.py --config $spec --no-cpu-baseline --no-secondary > $O/$tag-$rep.json 2> $O/$tag-$rep.err || { tail -20 $O/$tag-$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/$tag-$rep.json').read().strip().splitlines()[-1])
print('$spec', 'us/step %.2f' % (1e3*d['ms_per_step']), 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'])
" | tee -a $O/lines.log
  done
done
bash scripts/gpu_r3_kcloud_abl.sh default head
