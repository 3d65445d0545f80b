# per-kernel VGPR / scratch / occupancy / LDS of libslgpu (CPU-side, hipcc remarks)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared \
  -I /root/repo/include /root/repo/structured_light_for_3d_model_replication_amd/csrc/slgpu.hip /root/repo/structured_light_for_3d_model_replication_amd/csrc/slmerge.hip /root/repo/structured_light_for_3d_model_replication_amd/csrc/slcalib.hip -o /tmp/_ru.so \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | grep -oE "(Function Name: \S+|VGPRs: [0-9]+|AGPRs: [0-9]+|ScratchSize \[bytes/lane\]: [0-9]+|Occupancy \[waves/SIMD\]: [0-9]+|LDS Size \[bytes/block\]: [0-9]+)" | paste - - - - - -
