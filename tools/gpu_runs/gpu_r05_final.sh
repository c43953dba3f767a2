#!/bin/bash
# GPU box: the round's final tree -- whole GPU suite, smoke, bench lines (default + driver command),
# rocprofv3 kernel-trace summaries of the env and learner legs, PMC passes
bash tools/gpu_runs/gpu_r05_all.sh || exit 1
bash tools/gpu_runs/gpu_r05_prof.sh || exit 1
