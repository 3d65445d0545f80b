# Round-4 evidence driver (run on the GPU box through gpurun):
#   bash scripts/gpu_r4.sh OUT 'kind|label|ENV=v ...|args' ...
# kinds:
#   tests  pytest -m gpu with args (e.g. "tests/test_gpu_prestats.py -k multi")   -> OUT/label.log
#   bench  python bench.py args                                                   -> OUT/lines.jsonl (+ label)
#   prof   rocprofv3 --kernel-trace --stats of python bench.py args               -> OUT/label_kernel_stats.csv
#   trace  rocprofv3 --kernel-trace of python bench.py args (+ trace_overlap.py) -> OUT/label_kernel_trace.csv
#   pmc    rocprofv3 --pmc <args: counters> of scripts/steps_app.py $PMC_APP      -> OUT/label_counters.csv
#   app    rocprofv3 --kernel-trace --stats of an arbitrary program: args         -> OUT/label_kernel_stats.csv
#   run    any command (args), stdout to OUT/label.log
# Every step runs under its own time limit; the first failure ends the script.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
for spec in "$@"; do
  IFS='|' read -r kind label envs args <<< "$spec"
  echo "== $kind $label [$envs] $args"
  case $kind in
    tests)
      env $envs timeout -k 10 900 python -u -m pytest -m gpu -q --maxfail 25 --timeout 300 --timeout-method thread $args \
        > "$O/$label.log" 2>&1 || { tail -40 "$O/$label.log"; exit 1; }
      tail -1 "$O/$label.log" ;;
    bench)
      env $envs timeout -k 10 600 python3 -u bench.py $args > "$O/$label.json" 2> "$O/$label.err" \
        || { tail -20 "$O/$label.err"; exit 1; }
      python3 - "$O/$label.json" "$label" >> "$O/lines.jsonl" <<'PY' || exit 1
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d["label"] = sys.argv[2]
print(json.dumps(d))
PY
      python3 - "$O/$label.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("  ms/step %.4f  Gpx/s %.2f  path %.3f  k_decode %.3f  verified %s" % (
    d["ms_per_step"], d["value"] / 1e9, r["frac"], r["dominant_kernel"]["frac"], d.get("verified")))
PY
      ;;
    prof)
      rm -rf "$O/trace_$label"
      env $envs timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$label" -o t \
        -- python3 -u bench.py $args > "$O/$label.json" 2> "$O/$label.err" || { tail -20 "$O/$label.err"; exit 1; }
      f=$(find "$O/trace_$label" -name '*kernel_stats.csv' | head -1)
      cp "$f" "$O/${label}_kernel_stats.csv"
      rm -rf "$O/trace_$label"
      python3 - "$O/${label}_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_" in r["Name"]:
        print("  %9.2f us x%6s %5.1f%% %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], float(r["Percentage"]), r["Name"][:70]))
PY
      ;;
    trace)
      rm -rf "$O/trace_$label"
      env $envs timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_$label" -o t \
        -- python3 -u bench.py $args > "$O/$label.json" 2> "$O/$label.err" || { tail -20 "$O/$label.err"; exit 1; }
      f=$(find "$O/trace_$label" -name '*kernel_trace.csv' | head -1)
      cp "$f" "$O/${label}_kernel_trace.csv"
      rm -rf "$O/trace_$label"
      python3 scripts/trace_overlap.py "$O/${label}_kernel_trace.csv" ;;
    pmc)
      rm -rf "$O/pmc_$label"
      env $envs timeout -s KILL 120 rocprofv3 --pmc $args --output-format csv -d "$O/pmc_$label" -o p \
        -- python3 -u scripts/steps_app.py ${PMC_APP:-} > "$O/$label.log" 2>&1 || { tail -20 "$O/$label.log"; exit 1; }
      f=$(find "$O/pmc_$label" -name '*counter_collection.csv' | head -1)
      cp "$f" "$O/${label}_counters.csv"
      rm -rf "$O/pmc_$label" ;;
    app)
      rm -rf "$O/trace_$label"
      env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$label" -o t \
        -- $args > "$O/$label.log" 2>&1 || { tail -20 "$O/$label.log"; exit 1; }
      f=$(find "$O/trace_$label" -name '*kernel_stats.csv' | head -1)
      cp "$f" "$O/${label}_kernel_stats.csv"
      rm -rf "$O/trace_$label" ;;
    run)
      env $envs timeout -k 10 600 $args > "$O/$label.log" 2>&1 || { tail -20 "$O/$label.log"; exit 1; }
      tail -3 "$O/$label.log" ;;
    *) echo "unknown step kind $kind"; exit 2 ;;
  esac
done
echo "== done"
