set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ablate.log
for d in 0 2 4 8 12 14; do
  SLGPU_DEBUG=$d timeout -k 10 120 python -u scripts/kbench.py --reps 10 >> gpurun_out/ablate.log 2>&1 || exit $?
done
grep variant gpurun_out/ablate.log | grep -v torch | grep '"cloud"'
OUT=gpurun_out/prof3
mkdir -p $OUT
APP="python -u scripts/kbench.py --reps 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/sq1 -o sq1 -- $APP > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/sq2 -o sq2 -- $APP > $OUT/sq2.log 2>&1 || echo "sq2 failed"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $APP > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $APP > $OUT/write.log 2>&1 || exit $?
echo done
