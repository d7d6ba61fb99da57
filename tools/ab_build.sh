#!/bin/bash
# Build a variant of libtfhe_hip.so into build_ab/<name>/ with extra hipcc flags (kernel A/B tests).
# usage: tools/ab_build.sh <name> [extra hipcc flags...]
set -e
NAME=$1; shift
OUT=build_ab/$NAME
mkdir -p $OUT
H="/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -mcode-object-version=5"
$H "$@" -I tfhe_amd/csrc -c ${KSRC:-tfhe_amd/csrc/pbs_kernels.hip} -o $OUT/pbs_kernels.o
$H -x hip -c tfhe_amd/csrc/api.cpp -o $OUT/api.o
g++ -O2 -fPIC -std=c++17 -ffp-contract=off -c tfhe_amd/csrc/client.cpp -o $OUT/client.o
$H -shared -fPIC --offload-arch=gfx950 -o $OUT/libtfhe_hip.so $OUT/pbs_kernels.o $OUT/api.o $OUT/client.o -pthread
echo built $OUT/libtfhe_hip.so
