#!/bin/bash
# Round 2, session 3: GPU suite + smoke, then bench lines with 1/2/3 views in
# flight per GPU (bench.py --streams) on configs 1-5 -> gpurun_out/st
set -o pipefail
mkdir -p gpurun_out/st
O=gpurun_out/st
if [ "${ST_TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
      || { tail -30 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
for cfg in ${ST_CONFIGS:-c2 c1 c3 c4 c5}; do
  steps=20; [ $cfg = c1 ] && steps=400
  for s in ${ST_STREAMS:-1 2 3}; do
    timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 5 --streams $s --no-cpu-baseline \
        > $O/${cfg}_s$s.json 2> $O/${cfg}_s$s.err || { tail -20 $O/${cfg}_s$s.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/${cfg}_s$s.json')); print('$cfg', 's$s', round(d['value']/1e9,2), 'Gpx/s', round(d['ms_per_step']*1e3,1), 'us', round(d['roofline']['frac'],3))"
  done
done
