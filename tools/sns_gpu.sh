set -u
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sns.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sns_tests.log 2>&1 || { tail -30 gpurun_out/sns_tests.log; exit 1; }
tail -2 gpurun_out/sns_tests.log
timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 2 > gpurun_out/sns_fft.json 2>gpurun_out/sns_fft.err || { tail gpurun_out/sns_fft.err; exit 1; }
cat gpurun_out/sns_fft.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sns2 -o run --output-format csv -- python3 tools/sns_bench.py --batch 1024 --steps 1 > gpurun_out/prof_sns2.log 2>&1 || { tail -5 gpurun_out/prof_sns2.log; exit 1; }
find gpurun_out/prof_sns2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/sns2_kernel_stats.csv \;

if [ "${CHUNKS:-0}" = "1" ]; then
  for c in 256 512; do TFHE_HIP_SNS_CHUNK=$c timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 2 > gpurun_out/sns_c$c.json 2>&1 || exit 1; echo "chunk $c: $(cat gpurun_out/sns_c$c.json)"; done
fi
echo ALL_OK
