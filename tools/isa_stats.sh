#!/bin/bash
# Static ISA stats of the blind-rotate kernel: VGPRs, spills, VALU / s_nop / LDS counts.
# usage: tools/isa_stats.sh [source.hip] [extra hipcc flags...]
SRC=${1:-tfhe_amd/csrc/pbs_kernels.hip}; shift
D=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mcode-object-version=5 -I$(dirname $SRC) "$@" \
  -c $SRC -o $D/k.o -save-temps=obj -Rpass-analysis=kernel-resource-usage 2> $D/remarks.txt || { tail -20 $D/remarks.txt; exit 1; }
S=$(ls $D/*gfx950*.s)
awk '/^_ZN4tfhe19blind_rotate_kernelILb0ELb1/,/s_endpgm/' $S > $D/br.s
echo "VGPR $(grep -A12 'blind_rotate_kernelILb0ELb1' $D/remarks.txt | grep -m1 ' VGPRs:' | sed 's/.*VGPRs: \([0-9]*\).*/\1/') spill $(grep -A12 'blind_rotate_kernelILb0ELb1' $D/remarks.txt | grep -m1 'VGPRs Spill' | sed 's/.*Spill: \([0-9]*\).*/\1/') valu $(grep -cE '^\s+v_' $D/br.s) nop $(grep -cE '^\s+s_nop' $D/br.s) ds $(grep -cE '^\s+ds_' $D/br.s) mad64 $(grep -c v_mad_u64 $D/br.s) cnd $(grep -c v_cndmask $D/br.s) cmp $(grep -c v_cmp $D/br.s) perm $(grep -c permlane $D/br.s)"
cp $D/br.s /tmp/br_last.s
rm -rf $D
