#!/bin/bash
# c2: k_decode grid cap (SLGPU_DECODE_PER_CU) x views in flight (bench.py --streams)
set -o pipefail
mkdir -p gpurun_out/cs
for cap in 1 2; do
  for s in 1 2 3; do
    SLGPU_DECODE_PER_CU=$cap timeout -k 10 200 python -u bench.py --config c2 --steps 30 --warmup 5 --streams $s \
        --no-cpu-baseline > gpurun_out/cs/c2_cap${cap}_s$s.json 2> gpurun_out/cs/c2_cap${cap}_s$s.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/cs/c2_cap${cap}_s$s.json')); print('cap $cap s $s', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))"
  done
done
