# Round 3: HBM traffic of the c2 step in the exact (headline) mode, with the
# PMC counters calibrated for the access widths the kernels use:
#   1. scripts/micro/store_calib (known byte counts: 16-B, 12-B, 3-B and mixed
#      point stores; 8-B and 16-B streaming reads) under --pmc WRITE_SIZE and
#      --pmc FETCH_SIZE (separate passes);
#   2. scripts/steps_app.py (40 chained steps of the bench, next-stats on) under the
#      same two passes;
#   3. scripts/traffic_from_pmc.py --calib: per kernel, reported bytes x the
#      factor of its access shapes -> profiles-ready JSON.
# -> gpurun_out/r3traffic/traffic_c2.json
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3traffic
mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_w -o w -- ./scripts/micro/store_calib > $O/cal.json 2> $O/cal_w.log || { tail -5 $O/cal_w.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_f -o f -- ./scripts/micro/store_calib > /dev/null 2> $O/cal_f.log || { tail -5 $O/cal_f.log; exit 1; }
APP="python -u scripts/steps_app.py --steps 40"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- $APP > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- $APP > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python3 scripts/traffic_from_pmc.py $O/fetch $O/write c2 1 exact 1 $O/traffic_c2.json --calib $O/cal_f $O/cal_w $O/cal.json --per-step 40 > /dev/null || exit 1
python3 -c "
import json
d = json.load(open('$O/traffic_c2.json'))
print('calibration', json.dumps(d.get('calibration')))
print('bytes/step %.1f MB raw %.1f MB' % (d['bytes_per_step'] / 1e6, d['bytes_per_step_raw'] / 1e6), {k: round(v / 1e6, 1) for k, v in d['kernels'].items()})
"
rm -rf $O/fetch $O/write $O/cal_f $O/cal_w
