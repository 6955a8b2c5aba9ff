# Build the DUST microbenchmark variants into bin/ (run on the CPU container).
set -e
cd "$(dirname "$0")/../.."
mkdir -p bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-rdc -o bin/dust_micro \
  scripts/micro/dust_micro.hip rna_clique_amd/csrc/dust.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-rdc -DRC_DUST_PROF -o bin/dust_micro_prof \
  scripts/micro/dust_micro.hip rna_clique_amd/csrc/dust.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-rdc -DRC_DUST_PROF -DRC_DUST_NO_B -o bin/dust_micro_noB \
  scripts/micro/dust_micro.hip rna_clique_amd/csrc/dust.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-rdc -o bin/dust_micro_plain \
  scripts/micro/dust_micro.hip rna_clique_amd/csrc/dust.hip
