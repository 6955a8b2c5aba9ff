# Build the DUST microbenchmark into scratch/ (run on the CPU container).
set -e
cd "$(dirname "$0")/../.."
mkdir -p scratch
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-rdc -o scratch/dust_micro \
  scripts/micro/dust_micro.hip rna_clique_amd/csrc/dust.hip
