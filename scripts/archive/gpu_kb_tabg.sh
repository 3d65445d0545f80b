# decision tables: LDS (tg0) vs global for single-group workgroups (tg1) vs always global (tg2)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tabg
mkdir -p $O
SLGPU_LIB=$PWD/build/libslgpu_tg2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast_f32.py tests/test_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/lines.jsonl
for v in tg0 tg1 tg2; do
  for cfg in c1 c2 c3; do
    SLGPU_LIB=$PWD/build/libslgpu_$v.so timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $O/$v.$cfg.json 2> $O/$v.$cfg.err || { tail -20 $O/$v.$cfg.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/$v.$cfg.json').read().strip().splitlines()[-1]); d['lib']='$v'; print(json.dumps(d))" >> $O/lines.jsonl
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/tabg/lines.jsonl'):
    d=json.loads(l)
    print(d['lib'], d['config']['workload'][:18], 'us/step %.1f'%(1e3*d['ms_per_step']), 'Gpx/s %.1f'%(d['value']/1e9), {k: round(v*1e3,1) for k,v in d['path']['rerun_ms_last_group'].items() if k.startswith('k_')})
PY
