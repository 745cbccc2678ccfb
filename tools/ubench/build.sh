#!/bin/bash
# Build the microbenchmarks from source (binaries are git-ignored; they travel
# to the GPU box with the gpurun snapshot).  Usage: tools/ubench/build.sh [name...]
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
names=${*:-"rates p2bench mulbench"}
for n in $names; do
    case $n in
        host_perm) $HIPCC --cuda-host-only -O3 -march=native -std=c++17 -I../../linea_stark_prover_amd/csrc -o host_perm_bin host_perm.cpp ;;
        host_spin) $HIPCC --cuda-host-only -O3 -std=c++17 -mbmi2 -madx -I../../linea_stark_prover_amd/csrc -I../../include -o host_spin host_spin.cpp -lpthread ;;
        *) $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -o "$n" "$n.hip" ;;
    esac
done
