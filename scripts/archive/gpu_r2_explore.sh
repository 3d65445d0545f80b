# Round-2 exploration: GPU parity suite; kernel bench (C2 shape, maps+cloud and
# cloud-only, fast xyz); the decode pipelining microbenchmark; C1/C2/C3 bench
# lines.  -> gpurun_out/ex
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ex
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for only in "maps+cloud" "cloud"; do
  timeout -k 10 120 python -u scripts/kbench.py --reps 20 --fast --only "$only" 2>&1 | grep variant | grep -v torch_copy >> $O/kb.log || exit 1
done
cat $O/kb.log | cut -c 1-260
timeout -k 10 120 ./scripts/micro/decode_pipeline_bw > $O/micro.jsonl 2>&1 || { tail -5 $O/micro.jsonl; exit 1; }
cat $O/micro.jsonl
for cfg in c1 c2 c3; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || { tail -20 $O/$cfg.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/$cfg.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$cfg', 'us/step %.1f'%(d['ms_per_step']*1e3), 'Gpx/s %.1f'%(d['value']/1e9), 'path %.3f'%r['frac'], 'k_decode %.3f'%r['dominant_kernel']['frac'], {k: round(v*1e3,1) for k,v in d['path']['kernel_avg_ms'].items()}, {k: (round(v*1e3,1) if isinstance(v,float) else v) for k,v in d['path']['rerun_ms_last_group'].items() if k!='note'})"
done
