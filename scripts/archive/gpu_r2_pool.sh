#!/bin/bash
# core.ReconstructorPool: GPU pool tests, then bench lines per views in flight
set -o pipefail
mkdir -p gpurun_out/pool
timeout -k 10 200 python -u -m pytest tests/test_gpu_pool.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pool/pytest.log 2>&1 || { tail -30 gpurun_out/pool/pytest.log; exit 1; }
tail -2 gpurun_out/pool/pytest.log
ST_TESTS=0 ST_CONFIGS="${PL_CONFIGS:-c1 c5}" ST_STREAMS="${PL_STREAMS:-1 2 4 6}" bash scripts/gpu_r2_streams.sh
