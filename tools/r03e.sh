#!/bin/bash
# round-3: kernel-trace profile of the training step; halo DMA-window offset A/B
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 300 bash tools/ab_libs.sh dec6,dec7,dec8,dec9,enc4b,crossb fwd,dgrad cnn_itmo_amd/lib/variants/libpftoff2.so cnn_itmo_amd/lib/variants/libpftoff4.so > gpurun_out/r03e_ab_pftoff.txt 2>&1
bash tools/profile_round.sh r03e --steps 5 --warmup 2 --infer-batch 0 --k4-batch 0 --ns-batch 0
