# two-level block prefix (super-block sums) and larger launch groups:
# GPU tests on the 256K-chunk build, then bench lines for c2..c5
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sup
mkdir -p $O
SLGPU_LIB=$PWD/build/libslgpu_sup256.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
SLGPU_LIB=$PWD/build/libslgpu_sup.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest16.log 2>&1 || { tail -30 $O/pytest16.log; exit 1; }
tail -1 $O/pytest16.log
: > $O/lines.jsonl
for v in default sup sup64 sup256; do
  lib=structured_light_for_3d_model_replication_amd/libslgpu.so
  [ $v != default ] && lib=build/libslgpu_$v.so
  for cfg in c2 c3 c4 c5; do
    SLGPU_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/$v.$cfg.json 2> $O/$v.$cfg.err || { tail -20 $O/$v.$cfg.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/$v.$cfg.json').read().strip().splitlines()[-1]); d['lib']='$v'; print(json.dumps(d))" >> $O/lines.jsonl
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/sup/lines.jsonl'):
    d=json.loads(l)
    print(d['lib'].ljust(7), d['config']['workload'][:18], 'us/step %.1f'%(1e3*d['ms_per_step']), 'Gpx/s %.1f'%(d['value']/1e9), 'groups', d['path']['launch_groups'], {k: round(v*1e3,1) for k,v in d['path']['kernel_avg_ms'].items()})
PY
