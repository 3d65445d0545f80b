# Round-6 evidence at HEAD, one box (run through gpurun):
#   bash scripts/gpu_r6_final.sh OUT
# 1. calibrated PMC traffic per config (gpu_r4_traffic.sh -> gpurun_out/OUT_traffic/; SKIP_TRAFFIC=1:
#    the committed profiles/r06_traffic/ files instead);
# 2. the GPU suite and smoke;
# 3. the driver's default bench command, then every config's bench line, each
#    followed by rocprofv3 --kernel-trace --stats of the same command (gpu_r4.sh
#    -> gpurun_out/OUT/), the lines reading step 1's traffic files.
# Every step has its own time limit; the first failure ends the script.
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$1
T=gpurun_out/${O}_traffic
if [ "${SKIP_TRAFFIC:-0}" = 1 ]; then  # the committed traffic files (the bytes did not change)
  T=profiles/r06_traffic
else
  bash scripts/gpu_r4_traffic.sh ${O}_traffic c2:32 c3:10 c4:3 c5:4 || exit 1
fi
NB="--no-cpu-baseline --no-secondary --single-shot 0"
bash scripts/gpu_r4.sh $O \
  "tests|suite||tests" \
  "run|smoke||python scripts/run_smoke.py" \
  "bench|c2_default||--steps 20 --warmup 5 --traffic $T/traffic_c2.json" \
  "prof|c2_prof||--steps 20 --warmup 5 $NB --ring-control 0 --traffic $T/traffic_c2.json" \
  "prof|c2_streams1_prof||--steps 20 --warmup 5 --streams 1 $NB --ring-control 0 --traffic $T/traffic_c2.json" \
  "bench|c1||--config c1 --steps 400 --warmup 20 --cpu-seconds 6" \
  "prof|c1_prof||--config c1 --steps 400 --warmup 20 $NB" \
  "bench|c3||--config c3 --scaling strong --steps 20 --warmup 3 --cpu-seconds 6 --traffic $T/traffic_c3.json" \
  "prof|c3_prof||--config c3 --scaling strong --steps 20 --warmup 3 $NB --traffic $T/traffic_c3.json" \
  "bench|c4||--config c4 --steps 6 --warmup 2 --cpu-seconds 6 --traffic $T/traffic_c4.json" \
  "prof|c4_prof||--config c4 --steps 6 --warmup 2 $NB --traffic $T/traffic_c4.json" \
  "bench|c5||--config c5 --steps 8 --warmup 2 --cpu-seconds 6 --traffic $T/traffic_c5.json" \
  "prof|c5_prof||--config c5 --steps 8 --warmup 2 $NB --traffic $T/traffic_c5.json"
