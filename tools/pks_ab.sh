#!/bin/bash
# On the GPU box: tools/pks_bench.py on every build_ab/* variant (ms per 8-GLWE call, LWE/s, consistency).
cd "${GRAFT_REPO_ROOT:-.}"
for d in build_ab/*/; do n=$(basename $d); TFHE_HIP_LIB=$PWD/$d/libtfhe_hip.so timeout -k 10 200 python tools/pks_bench.py 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.readlines()[-1]);print('$n', d['ms_per_call'], d['lwe_per_s'], d['consistent'])" || exit 1; done
