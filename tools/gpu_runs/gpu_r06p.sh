#!/bin/bash
# round 6 (p): the ABI-v5 meta tree -- whole GPU suite, smoke, bench lines, kernel traces, PMC
# passes (env + learner), then the GEMM-form weight-gradient A/B and probes
bash tools/gpu_runs/gpu_r06_final.sh || exit 1
bash tools/gpu_runs/gpu_r06i.sh && bash tools/gpu_runs/gpu_r06l.sh
