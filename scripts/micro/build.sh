# Build the DUST microbenchmark variants into bin/ (run on the CPU container).
set -e
cd "$(dirname "$0")/../.."
mkdir -p bin
for v in 0; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDUST_VARIANT=$v -o bin/dust_micro_$v \
    scripts/micro/dust_micro.hip rna_clique_amd/csrc/dust.hip
done
