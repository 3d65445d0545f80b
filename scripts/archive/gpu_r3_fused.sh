# Round 3: k_fused (decode + look-back + cloud in one launch, SLGPU_FUSED=1) --
# the fused GPU tests, then bench A/B: c1 at 1 and 6 views in flight, c2.  -> gpurun_out/r3fu
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3fu
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fused or ab_switches or golden_fused or full_4k" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/lines.log
for rep in 1 2; do
  for F in 0 1; do
    for spec in "c1 --streams 1" "c1" "c2"; do
      tag=$(echo "$spec" | tr ' ' '_')
      SLGPU_FUSED=$F timeout -k 10 200 python -u bench.py --config $spec --no-cpu-baseline --no-secondary > $O/${tag}_F$F-$rep.json 2> $O/${tag}_F$F-$rep.err || { tail -20 $O/${tag}_F$F-$rep.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/${tag}_F$F-$rep.json').read().strip().splitlines()[-1])
print('$spec F=$F', 'us/step %.2f' % (1e3*d['ms_per_step']), 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if isinstance(v,float)})
" | tee -a $O/lines.log
    done
  done
done
