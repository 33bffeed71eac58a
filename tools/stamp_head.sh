#!/bin/bash
# Records the current commit in HEAD_COMMIT (git-ignored, travels with gpurun's
# snapshot): PMC summaries and bench lines measured on the box name the commit.
cd "$(dirname "$0")/.." && echo "$(git rev-parse --short HEAD)$(git diff --quiet HEAD -- mjrl_amd include bench.py || echo +dirty)" > HEAD_COMMIT
