#!/bin/bash
# SnS MAC grid A/B on one box: the SnS GPU tests, then tools/sns_bench.py at B = 1024 for each
# TFHE_HIP_SNS_MACG (ciphertext-group slots of the MAC grid; 0 = one group per workgroup).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sns.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sns_tests.log 2>&1 || { tail -30 gpurun_out/sns_tests.log; exit 1; }
tail -2 gpurun_out/sns_tests.log
# each case: "MACG:INVOCC" (TFHE_HIP_SNS_INVOCC = waves per SIMD of the inverse kernel)
for cs in ${CASES:-8:0 8:3 8:0 8:3}; do
  g=${cs%%:*}; o=${cs##*:}
  TFHE_HIP_SNS_MACG=$g TFHE_HIP_SNS_INVOCC=$o timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 2 > gpurun_out/sns_g${g}_o$o.json 2> gpurun_out/sns_g${g}_o$o.err || { tail gpurun_out/sns_g${g}_o$o.err; exit 1; }
  echo "MACG $g INVOCC $o: $(cat gpurun_out/sns_g${g}_o$o.json)"
done
if [ -n "${TAG:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 tools/sns_bench.py --batch 1024 --steps 1 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -5 gpurun_out/prof_${TAG}.log; exit 1; }
  find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
  cut -c1-120 gpurun_out/${TAG}_kernel_stats.csv | head -5
  timeout -k 10 300 python tools/sns_bench.py --batch 1024 --steps 3 > gpurun_out/${TAG}_bench.json 2>/dev/null && cat gpurun_out/${TAG}_bench.json
fi
echo ALL_OK
