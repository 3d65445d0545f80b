# Round 4: calibrated HBM bytes per step of the multi-view configs' calls
# (VERDICT r3 #1 "calibrated PMC per config"; round 3 had archive/gpu_r3_traffic.sh for c2):
#   1. scripts/micro/store_calib under --pmc WRITE_SIZE and --pmc FETCH_SIZE
#      (separate passes): the counters' factors for the kernels' access shapes;
#   2. scripts/steps_app.py --config cN (N chained calls of the config's views,
#      next-stats on) under the same two passes;
#   3. scripts/traffic_from_pmc.py --calib --per-step N -> traffic_cN.json.
#   bash scripts/gpu_r4_traffic.sh OUT c2:40 c3:10 c4:3 c5:4      (config:steps ...)
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_w -o w -- ./scripts/micro/store_calib > $O/cal.json 2> $O/cal_w.log || { tail -5 $O/cal_w.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_f -o f -- ./scripts/micro/store_calib > /dev/null 2> $O/cal_f.log || { tail -5 $O/cal_f.log; exit 1; }
for spec in "$@"; do
  cfg="${spec%%:*}"
  n="${spec#*:}"
  echo "== $cfg ($n calls)"
  sel="--config $cfg"
  [ "$cfg" = c2 ] && sel=""   # steps_app's default: config 2's chained 4K maps + cloud steps
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$cfg -o fetch -- python3 -u scripts/steps_app.py $sel --steps $n > $O/fetch_$cfg.log 2>&1 || { tail -5 $O/fetch_$cfg.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$cfg -o write -- python3 -u scripts/steps_app.py $sel --steps $n > $O/write_$cfg.log 2>&1 || { tail -5 $O/write_$cfg.log; exit 1; }
  views=$(python3 -c "print({'c2': 1, 'c3': 36, 'c4': 45, 'c5': 45}['$cfg'])")
  ring=1; [ "$cfg" = c2 ] && ring=4   # steps_app's c2 default: 3 distinct views rounded up to 4 (2 lanes), as bench.py
  python3 scripts/traffic_from_pmc.py $O/fetch_$cfg $O/write_$cfg $cfg $views exact 1 $O/traffic_$cfg.json --calib $O/cal_f $O/cal_w $O/cal.json --per-step $n --ring $ring > /dev/null || exit 1
  python3 -c "
import json
d = json.load(open('$O/traffic_$cfg.json'))
print('$cfg bytes/call %.1f MB (raw %.1f MB)' % (d['bytes_per_step'] / 1e6, d['bytes_per_step_raw'] / 1e6), {k: round(v / 1e6, 1) for k, v in d['kernels'].items()})
"
  tail -1 $O/fetch_$cfg.log
  rm -rf $O/fetch_$cfg $O/write_$cfg
done
rm -rf $O/cal_f $O/cal_w
