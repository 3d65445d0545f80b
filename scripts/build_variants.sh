# Measurement-only builds of libslgpu.so into build/ (never the shipped
# library): build/libslgpu_<name>.so for each "name:flags" argument, e.g.
#   bash scripts/build_variants.sh nodec:-DSLGPU_ABLATE=512 aonly:-DSLGPU_ABLATE=1024
set -eu
cd "$(dirname "$0")/.."
mkdir -p build
SRC="structured_light_for_3d_model_replication_amd/csrc"
for spec in "$@"; do
  name="${spec%%:*}"
  flags="${spec#*:}"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-function \
    -Wno-pass-failed -I include $flags $SRC/slgpu.hip $SRC/slmerge.hip $SRC/slcalib.hip -o build/libslgpu_$name.so &
done
wait
ls -la build/
