#!/bin/bash
# Build a variant of libtfhe_hip.so into build_ab/<name>/ with extra hipcc flags (kernel A/B tests;
# tools/ab_run.sh benches every variant on the GPU box).
# usage: tools/ab_build.sh <name> [extra hipcc flags...]
set -e
NAME=$1; shift
make -s -C tfhe_amd -j8 B=../build_ab/$NAME/obj LIB=../build_ab/$NAME/libtfhe_hip.so EXTRA="$*"
echo built build_ab/$NAME/libtfhe_hip.so
