#!/bin/bash
# round-3 probe: GPU suite, bench with/without the wgrad side stream, halo static-priority A/B
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03c_gputest.log 2>&1
timeout -k 10 300 env CNNITMO_SIDE_STREAM=0 python -u bench.py --no-cpu --infer-batch 0 --k4-batch 0 --ns-batch 0 > $O/r03c_noside.json 2> $O/r03c_noside.err
timeout -k 10 400 python -u bench.py > $O/r03c_bench.json 2> $O/r03c_bench.err
timeout -k 10 300 bash tools/ab_libs.sh dec6,dec7,dec8,dec9,enc4b,crossb fwd,dgrad cnn_itmo_amd/lib/variants/libhaloprio.so > $O/r03c_ab_haloprio.txt 2>&1
