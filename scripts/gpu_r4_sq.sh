# SQ counters of the cloud-only k_decode<11,0,322,1>
# (5 x 4K views per launch, the c5 shape) against the microbenchmark of its
# bare access pattern at the same scale (scripts/micro/cloud_decode_floor:
# 24 planes + 12-bit records of 5 views, 995 MB per launch, HBM-resident),
# and of the posed exact k_cloud beside it (the c5 call: poses on),
# plus both kernels' timings.  -> gpurun_out/r4sq (copied to profiles/r04_sq/)
set -u -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4sq
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 120 ./scripts/micro/cloud_decode_floor 5 > $O/floor_v5.jsonl 2> $O/floor.err || { tail -5 $O/floor.err; exit 1; }
timeout -k 10 120 ./scripts/micro/cloud_decode_floor 1 > $O/floor_v1.jsonl 2>> $O/floor.err || { tail -5 $O/floor.err; exit 1; }
cat $O/floor_v5.jsonl $O/floor_v1.jsonl
timeout -k 10 300 python3 -u scripts/kbench.py --views 5 --only cloud --reps 20 --preroll-ms 300 > $O/kbench_c5shape.jsonl 2> $O/kbench.err || { tail -5 $O/kbench.err; exit 1; }
tail -2 $O/kbench_c5shape.jsonl
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
k=0
for P in "$P1" "$P2" "$P3"; do
  k=$((k+1))
  rm -rf $O/p$k $O/q$k
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$k -o p -- ./scripts/micro/cloud_decode_floor 5 > $O/p$k.log 2>&1 || { tail -5 $O/p$k.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/q$k -o q -- python3 -u scripts/steps_app.py --views 5 --cloud-only --poses --steps 6 > $O/q$k.log 2>&1 || { tail -5 $O/q$k.log; exit 1; }
  cp $(find $O/p$k -name '*counter_collection.csv' | head -1) $O/floor_pass$k.csv
  cp $(find $O/q$k -name '*counter_collection.csv' | head -1) $O/decode_pass$k.csv
  rm -rf $O/p$k $O/q$k
done
echo done
