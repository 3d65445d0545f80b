# Round 3: c2 (exact headline) with 1 / 2 / 3 views in flight (ReconstructorPool
# lanes, --streams), interleaved twice, then the default c2 bench under
# rocprofv3 --kernel-trace --stats (kernel table for DESIGN 5.0).  -> gpurun_out/r3c2s
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3c2s
mkdir -p $O
: > $O/lines.log
for rep in 1 2; do
  for S in 1 2 3; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary --streams $S > $O/s$S-$rep.json 2> $O/s$S-$rep.err || { tail -20 $O/s$S-$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/s$S-$rep.json').read().strip().splitlines()[-1])
t=d['timing']['step_us']
print('S=$S', 'ms/step %.4f' % d['ms_per_step'], 'Gpx/s %.1f' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], 'ev med %.1f' % t['median'])
" | tee -a $O/lines.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/traced.json 2> $O/traced.err || { tail -20 $O/traced.err; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $O/c2_kernel_stats.csv
rm -rf $O/trace
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r3c2s/c2_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>5} {r['Name'][:70]}")
PY
# this build vs HEAD's (build/libslgpu_head.so): kbench exact maps+cloud
bash scripts/gpu_r3_kcloud_abl.sh default head
